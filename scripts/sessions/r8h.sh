#!/bin/bash
# Round 6 session H (shipping build): exact fp32 at 16k, the instruction mix per
# MFMA of the three native fp32 kernels (f32_t128x2 = auto, f32_w4, f32_256s)
# against hipBLASLt's (locate the 98.2 vs 98.9 % MFMA-busy gap
# before building another fp32 kernel), with the clock / MFMA busy / L2 passes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
MIX=1 DT=float32 N=16384 KS=f32_t128x2,f32_w4,f32_256s REPS=3 OUT=gpurun_out/r8h/pmc \
  timeout -k 10 1000 bash scripts/gpu_pmc.sh > gpurun_out/r8h.log 2>&1; rc=$?
mkdir -p gpurun_out/r8h; mv gpurun_out/r8h.log gpurun_out/r8h/pmc.log
python scripts/pmc_summary.py gpurun_out/r8h/pmc --cycle f32_t128x2,f32_w4,f32_256s,torch
exit $rc
