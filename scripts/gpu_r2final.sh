#!/bin/bash
# Round-2 closing pass: full validation (scripts/gpu_validate.sh) plus the fp8 driver bench and the
# native executor's fp8 / bf16 16k numbers.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash scripts/gpu_validate.sh r2final || exit $?
OUT=gpurun_out/r2final
step() { local name=$1; shift; echo "== $name"; "$@" > $OUT/$name.log 2>&1; local rc=$?; tail -${TAILN:-3} $OUT/$name.log | cut -c1-300; echo "== $name rc=$rc"; return $rc; }
step bench_fp8 timeout -k 10 300 python bench.py --dtype float8_e4m3fn --steps 20 --warmup 5 --extra-steps 5 --extra-warmup 2 &&
TAILN=10 step native_fp8 timeout -k 10 200 pytorch_distributed_matmul_benchmark_amd/runtime/pdmb_bench --gpus 1 --sizes 16384 --dtype float8_e4m3fn --check &&
TAILN=10 step native_bf16 timeout -k 10 200 pytorch_distributed_matmul_benchmark_amd/runtime/pdmb_bench --gpus 1 --sizes 16384 --check
