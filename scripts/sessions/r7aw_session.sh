#!/bin/bash
# round-5 session aw: PMC of the new exact-fp32 f32_t64x2 plan (auto, split 2)
# against f32_t128x2 unsplit (the old plan) and hipBLASLt on 4608^2 x 4096
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
DT=float32 OUT=gpurun_out/r7aw/pmc_f32_4608 SHAPE=4608,4608,4096 REPS=10 KS=auto,f32_t128x2 bash scripts/gpu_pmc.sh || exit $?
python scripts/pmc_summary.py gpurun_out/r7aw/pmc_f32_4608 > gpurun_out/r7aw/pmc_f32_4608.md || exit $?
echo done
