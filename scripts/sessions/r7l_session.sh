#!/bin/bash
# round-5 session l: fp8 one-wave PMC (8192x2048x8192, auto vs hipBLASLt), shard tables, bench kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r7l
(export OUT=gpurun_out/r7l/pmc SHAPE=8192,2048,8192 DT=float8_e4m3fn KS=auto REPS=4; bash scripts/gpu_pmc.sh > gpurun_out/r7l/pmc.log 2>&1) || exit $?
python scripts/pmc_summary.py gpurun_out/r7l/pmc > gpurun_out/r7l/pmc_summary.md 2>&1; tail -30 gpurun_out/r7l/pmc_summary.md
bash scripts/gpu_session.sh r7l ab_fp32_shards shard_table rocprof_bench
