#!/bin/bash
# Round-2 GPU pass C: CU-budget planner + RCCL-like comm proxy overlap experiment, full GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r2c
mkdir -p $OUT
step() { local name=$1; shift; echo "== $name"; "$@" > $OUT/$name.log 2>&1; local rc=$?; tail -12 $OUT/$name.log; echo "== $name rc=$rc"; return $rc; }
step cumask timeout -k 10 400 python scripts/cu_mask_overlap.py &&
step all_tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
