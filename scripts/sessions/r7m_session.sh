#!/bin/bash
# round-5 session m (experiment build): fp8 one-wave tile timeline (8192x2048x8192, 4096^3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PDMB_EXPERIMENTS=1
mkdir -p gpurun_out/r7m
timeout -k 10 300 python scripts/tile_timeline.py --kernels fp8_w4 --dtype float8_e4m3fn \
  --shapes 8192,2048,8192 4096,4096,4096 8192,2048,16384 --repeats 5 > gpurun_out/r7m/timeline_fp8.jsonl 2> gpurun_out/r7m/timeline_fp8.err || exit $?
timeout -k 10 300 python scripts/tile_timeline.py --kernels w4 \
  --shapes 8192,2048,8192 16384,16384,16384 --repeats 3 > gpurun_out/r7m/timeline_bf16.jsonl 2> gpurun_out/r7m/timeline_bf16.err || exit $?
cut -c1-900 gpurun_out/r7m/timeline_fp8.jsonl
