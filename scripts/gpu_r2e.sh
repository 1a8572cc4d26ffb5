#!/bin/bash
# Round-2 GPU pass E: tile family + fp32 W4 exactness, interleaved sweeps vs hipBLASLt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r2e
mkdir -p $OUT
step() { local name=$1; shift; echo "== $name"; "$@" > $OUT/$name.log 2>&1; local rc=$?; tail -12 $OUT/$name.log; echo "== $name rc=$rc"; return $rc; }
step gemm_tests timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 300 --timeout-method thread &&
step f32_ab timeout -k 10 300 python scripts/ab_kernels.py --kernels f32_256s,f32_w4 --dtype float32 --sizes 8192 16384 --rounds 3 --iters 5 &&
step f32_torch timeout -k 10 300 python scripts/gemm_perf.py --sizes 16384 --dtype float32 --rounds 3 --iters 5 &&
step sweep timeout -k 10 500 python scripts/splitk_sweep.py --rounds 4 --arms auto w4:1 w4:2 t256x128:1 t256x128:2 t128:1 t128:2 t128x2:1 --shapes 8192x1024x8192 4096x2048x4096 4096x1024x4096 4096x512x4096 2048x2048x2048 8192x2048x8192 16384x2048x16384 16384x16384x16384
