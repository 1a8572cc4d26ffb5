#!/bin/bash
# Round 6 session ZB (shipping build): f32_w4l on every whole-wave fp32 grid
# (K >= 4096). Cold first launches of multi-wave grids in fresh processes; the
# whole GPU suite, smoke, bench (closing validation C).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r8zb; mkdir -p $OUT
for s in "8192 8192 8192" "16384 16384 16384" "16384 2048 16384" "4096 4096 4096 2"; do
  timeout -k 5 60 python scripts/w4s_probe.py $s --kernel auto >> $OUT/probe.jsonl 2>> $OUT/probe.err || { echo "probe $s rc=$?"; cat $OUT/probe.jsonl; exit 1; }
done
cut -c1-200 $OUT/probe.jsonl
bash scripts/gpu_session.sh r8zb tests smoke bench || exit $?
echo "exit 0"
