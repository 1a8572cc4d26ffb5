#!/bin/bash
# GPU validation pass used with gpurun: tests, bench, reference CLI, rocprof.
# Each GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
step() { local name=$1; shift; echo "== $name"; "$@" > $OUT/$name.log 2>&1; local rc=$?; tail -25 $OUT/$name.log; echo "== $name rc=$rc"; return $rc; }
step pytest_gpu timeout -k 10 600 python -m pytest tests -m gpu -x -q &&
step bench timeout -k 10 300 python bench.py &&
step basic timeout -k 10 300 python matmul_benchmark.py --check &&
step rocprof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/rocprof -o bench -- python3 bench.py --steps 10 --warmup 3
