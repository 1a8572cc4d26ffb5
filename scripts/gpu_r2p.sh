#!/bin/bash
# Round-2 pass P: fp32 W4 with the LDS-staged non-temporal epilogue (exactness + A/B vs f32_256s
# control and hipBLASLt), then the reference-compatible CLIs and the native executor at 1 GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2p}
mkdir -p $OUT
step() { local name=$1; shift; echo "== $name"; "$@" > $OUT/$name.log 2>&1; local rc=$?; tail -${TAILN:-6} $OUT/$name.log | cut -c1-220; echo "== $name rc=$rc"; return $rc; }
step f32_tests timeout -k 10 200 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "f32" &&
TAILN=12 step f32_ab timeout -k 10 400 python -u scripts/ab_kernels.py --dtype float32 --rounds 5 --iters 10 \
  --kernels f32_w4,f32_256s,torch --shapes 4096,4096,4096 8192,8192,8192 16384,16384,16384 4096,1024,4096 &&
TAILN=14 step cli_single timeout -k 10 300 ./run_benchmark.sh 1 bfloat16 --check &&
TAILN=14 step cli_batch timeout -k 10 300 ./run_scaling_benchmark.sh 1 batch_parallel bfloat16 &&
TAILN=14 step cli_matrix timeout -k 10 300 ./run_scaling_benchmark.sh 1 matrix_parallel bfloat16 --check &&
TAILN=14 step native_indep timeout -k 10 200 pytorch_distributed_matmul_benchmark_amd/runtime/pdmb_bench --gpus 1 --sizes 16384 --check &&
TAILN=14 step native_matrix timeout -k 10 200 pytorch_distributed_matmul_benchmark_amd/runtime/pdmb_bench --gpus 1 --sizes 16384 --mode matrix_parallel --overlap --check
