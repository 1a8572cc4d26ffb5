#!/bin/bash
# Round-2 GPU pass A: GPU tests (split-K, surface), split-K sweep vs hipBLASLt,
# 1-GPU bench, and the 2-rank self-launch rehearsal (gloo, ranks share the GPU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r2a
mkdir -p $OUT
step() { local name=$1; shift; echo "== $name"; "$@" > $OUT/$name.log 2>&1; local rc=$?; tail -15 $OUT/$name.log; echo "== $name rc=$rc"; return $rc; }
step pytest_gpu timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread &&
step splitk timeout -k 10 300 python scripts/splitk_sweep.py --rounds 4 &&
step bench timeout -k 10 300 python bench.py &&
step bench_selflaunch2 timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --size 4096 --steps 3 --warmup 1 --extra-steps 2 --extra-warmup 1
