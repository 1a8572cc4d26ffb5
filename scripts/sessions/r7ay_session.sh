#!/bin/bash
# round-5 session ay: random-shape exactness fuzz of auto after the round-5
# planner work (small grids favoured: --max 4096, then a wider pass)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7ay; mkdir -p $OUT
timeout -k 10 500 python scripts/shape_fuzz.py --count 60 --seed 11 --max 4096 > $OUT/fuzz_small.jsonl 2> $OUT/fuzz.err || exit $?
timeout -k 10 500 python scripts/shape_fuzz.py --count 25 --seed 12 --max 9000 > $OUT/fuzz_wide.jsonl 2>> $OUT/fuzz.err || exit $?
echo done
