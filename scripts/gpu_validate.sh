#!/bin/bash
# Full GPU validation of the tree (arg: output tag under gpurun_out/): GPU suite, smoke, 1-GPU bench, rocprof
# kernel stats of the bench, 2-rank self-launch rehearsal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-validate}
mkdir -p $OUT
step() { local name=$1; shift; echo "== $name"; "$@" > $OUT/$name.log 2>&1; local rc=$?; tail -8 $OUT/$name.log; echo "== $name rc=$rc"; return $rc; }
step all_tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread &&
step smoke timeout -k 10 120 python __graft_entry__.py smoke &&
step bench timeout -k 10 300 python bench.py &&
step rocprof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/rocprof -o bench -- python3 bench.py --steps 20 --warmup 5 &&
step selflaunch timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --size 4096 --steps 3 --warmup 1 --extra-steps 2 --extra-warmup 1 &&
step selflaunch4 timeout -k 10 300 python bench.py --gpus 4 --dist-backend gloo --size 4096 --steps 3 --warmup 1 --extra-steps 2 --extra-warmup 1
