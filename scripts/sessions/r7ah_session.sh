#!/bin/bash
# round-5 session ah: the open gap tables (VERDICT r4 weak #3 exact fp32, #5 fp8
# 1-2-wave grids) and the reference's default sizes re-measured with settled,
# position-balanced arms (ab_kernels --settle 1, rounds a multiple of the arms):
# the earlier A/Bs timed auto right after hipBLASLt (profiles/r7af_*)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7ah; mkdir -p $OUT
timeout -k 10 900 python scripts/ab_kernels.py --dtype float32 --rounds 4 --iters 5 --settle 1 --sessions 2 \
  --kernels auto,torch \
  --shapes 1024,16384,16384 16384,1024,16384 4096,4096,14336 2048,8192,8192 8192,2048,8192 \
           4096,12288,12288 8192,8192,28672 4096,4096,4096 8192,8192,8192 16384,16384,16384 \
           4096,512,4096 4096,1024,4096 8192,1024,8192 2048,2048,2048 4096,2048,4096 \
  > $OUT/ab_f32_gap_table_settled.jsonl 2> $OUT/ab_f32.err || exit $?
echo f32 done
timeout -k 10 900 python scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 4 --iters 20 --settle 1 --sessions 2 \
  --kernels auto,torch \
  --shapes 5120,5120,4096 5120,5120,5120 8192,2048,8192 4096,16384,4096 10240,8192,2048 16384,2048,16384 \
           4096,4096,4096 8192,8192,8192 16384,16384,16384 8192,8192,1024 2048,8192,8192 \
  > $OUT/ab_fp8_gap_table_settled.jsonl 2> $OUT/ab_fp8.err || exit $?
echo fp8 done
timeout -k 10 900 python scripts/ab_kernels.py --dtype bfloat16 --rounds 4 --iters 10 --settle 1 --sessions 2 \
  --kernels auto,torch \
  --shapes 4096,4096,4096 8192,8192,8192 16384,16384,16384 3072,3072,3072 2304,2304,4096 8192,2048,8192 \
  > $OUT/ab_bf16_table_settled.jsonl 2> $OUT/ab_bf16.err || exit $?
echo done
