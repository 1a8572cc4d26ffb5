#!/bin/bash
# round-5 session g (PDMB_EXPERIMENTS=1 build in the tree): W4S power attribution at 16k,
# then the experiment-kernel tests (the opt-in marker)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; export TMPDIR=/tmp PDMB_EXPERIMENTS=1; OUT=gpurun_out/r7g; mkdir -p $OUT
echo "== power $(date +%T)"
timeout -k 10 400 python scripts/power_attrib.py --rounds 3 --seconds 2 > $OUT/power.log 2>&1; rc=$?
grep '^{' $OUT/power.log > $OUT/power.jsonl; cat $OUT/power.jsonl | cut -c1-300; [ $rc -eq 0 ] || exit $rc
echo "== experiment tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests -m "gpu and experiments" -x -q --timeout 300 --timeout-method thread > $OUT/exp_tests.log 2>&1; rc=$?
tail -3 $OUT/exp_tests.log; exit $rc
