set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/gemm_perf.py --sizes 4096 8192 16384 --iters 20 --warmup 5 --rounds 3 > gpurun_out/gemm_perf.log 2>&1
rc=$?
cat gpurun_out/gemm_perf.log
exit $rc
