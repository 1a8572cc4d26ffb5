#!/bin/bash
# round-5 session w: host cost per GEMM call after the planner memo; full GPU suite
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7w; mkdir -p $OUT
timeout -k 10 240 python scripts/host_overhead.py > $OUT/host_overhead.jsonl 2>&1 || exit $?
cat $OUT/host_overhead.jsonl | grep '^{'
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=8 -q -rs --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log; exit $rc
