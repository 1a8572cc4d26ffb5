#!/bin/bash
# round-5 session ac: exact-fp32 f32_t128x2 with a static wave priority on odd workgroups (PDMB_F32_PRIO=1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7ac; mkdir -p $OUT
timeout -k 10 900 python scripts/ab_kernels.py --dtype float32 --rounds 3 --iters 5 --sessions 2 \
  --kernels auto,auto@PDMB_F32_PRIO=1,torch \
  --shapes 8192,8192,8192 16384,16384,16384 4096,12288,12288 8192,2048,8192 4096,2048,4096 \
  > $OUT/ab_f32_prio.jsonl 2> $OUT/ab.err || exit $?
echo done
