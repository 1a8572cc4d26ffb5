#!/bin/bash
# round-5 session i: validation of the tree (GPU suite, smoke, driver bench, kernel trace of the bench)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; export TMPDIR=/tmp; OUT=gpurun_out/r7i; mkdir -p $OUT
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=8 -q -rs --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -4 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke $(date +%T)"
timeout -k 10 180 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
echo "== bench $(date +%T)"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit $?
grep '^{' $OUT/bench.log > $OUT/bench.json; cut -c1-400 $OUT/bench.json
echo "== rocprof $(date +%T)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rocprof -o bench -- python3 bench.py --steps 20 --warmup 5 --extra-steps 0 > $OUT/rocprof.log 2>&1 || exit $?
find $OUT/rocprof -name "*kernel_stats.csv" | head -2
echo "== done $(date +%T)"
