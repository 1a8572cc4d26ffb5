#!/bin/bash
# Round 6 session Z (shipping build): W4S and fp8 W4S issue the first two
# K-tiles' DMA pieces of every tile with 5 wait states after any preceding
# instruction (common.h dma16_at_pad: hipcc restored spilled soffsets with
# v_readlane 2 states before those pieces; tests/test_sgpr_vmem_hazard.py).
# The whole GPU suite, smoke, bench; then the bf16 / fp8 tables against
# hipBLASLt as in r8k (settled, two sessions) to price the padding.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/gpu_session.sh r8z tests smoke bench || exit $?
OUT=gpurun_out/r8z
for dt in bfloat16 float8_e4m3fn; do
  timeout -k 10 400 python scripts/ab_kernels.py --dtype $dt --rounds 4 --iters 20 --settle 1 --sessions 2 \
    --kernels auto,torch --sizes 4096 8192 16384 > $OUT/table_$dt.jsonl 2> $OUT/table_$dt.err || exit $?
  grep '"summary"' $OUT/table_$dt.jsonl | cut -c1-230
done
echo "exit 0"
