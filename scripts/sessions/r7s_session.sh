#!/bin/bash
# round-5 session s: full GPU suite after f32_t64 + the 3-way split; fp32 2304^2 x 4096 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7s; mkdir -p $OUT
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=8 -q -rs --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/ab_kernels.py --dtype float32 --rounds 5 --sessions 2 --kernels auto,auto@PDMB_SPLIT3=0,torch \
  --shapes 2304,2304,4096 > $OUT/ab_f32_2304.jsonl 2> $OUT/ab_f32_2304.err || exit $?
grep summary $OUT/ab_f32_2304.jsonl | cut -c1-200
