cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gemm_gpu.py -x -q > gpurun_out/pytest_gemm.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gemm.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
for k in mfma256b mfma256c mfma256b mfma256c; do
timeout -k 10 300 python scripts/gemm_perf.py --sizes 4096 8192 16384 --kernel $k --iters 20 --rounds 3 --no-torch > gpurun_out/perf_$k.log 2>&1 || exit $?; cat gpurun_out/perf_$k.log
done
