#!/bin/bash
# Round-2 GPU pass B: T128 + sc1 split-K tests, sweep vs hipBLASLt, MFMA shape probe,
# CU-mask overlap proxy, then the whole GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r2b
mkdir -p $OUT
step() { local name=$1; shift; echo "== $name"; "$@" > $OUT/$name.log 2>&1; local rc=$?; tail -12 $OUT/$name.log; echo "== $name rc=$rc"; return $rc; }
step gemm_tests timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_overlap_gpu.py -x -q --timeout 300 --timeout-method thread &&
step sweep timeout -k 10 400 python scripts/splitk_sweep.py --rounds 4 &&
step probe timeout -k 10 120 pytorch_distributed_matmul_benchmark_amd/runtime/mfma_probe --rounds 5 &&
step cumask timeout -k 10 300 python scripts/cu_mask_overlap.py &&
step all_tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
