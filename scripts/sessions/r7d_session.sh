#!/bin/bash
# round-5 session d: IPC handle probe (with the pool phase), the overlap proxy
# (per-piece-count measured shares), the whole GPU suite with skip reasons
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; export TMPDIR=/tmp; OUT=gpurun_out/r7d; mkdir -p $OUT
echo "== probe $(date +%T)"
timeout -k 10 120 python scripts/ipc_handle_probe.py --trials 5 > $OUT/probe.jsonl 2> $OUT/probe.err || exit $?
cat $OUT/probe.jsonl | cut -c1-220
echo "== proxy $(date +%T)"
timeout -k 10 600 python scripts/overlap_proxy.py > $OUT/proxy.log 2>&1 || exit $?
grep '^{' $OUT/proxy.log > $OUT/proxy.jsonl
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -15 $OUT/tests.log; echo "tests rc=$rc"; exit $rc
