#!/bin/bash
# round-5 session r: 3-way split-K in auto (auto vs PDMB_SPLIT3=0 vs hipBLASLt), 2 sessions, on the grids it changes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7r; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_fp8_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "splitk or f32 or tile_family or tiled_random" > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/ab_kernels.py --dtype float32 --rounds 5 --sessions 2 --kernels auto,auto@PDMB_SPLIT3=0,torch \
  --shapes 1536,1536,4096 2560,256,8192 2560,512,8192 2560,1024,8192 5120,512,4096 2560,2048,4096 1536,3072,1024 \
  > $OUT/ab_f32.jsonl 2> $OUT/ab_f32.err || exit $?
timeout -k 10 600 python scripts/ab_kernels.py --dtype bfloat16 --rounds 5 --sessions 2 --kernels auto,auto@PDMB_SPLIT3=0,torch \
  --shapes 2560,4096,16384 5120,2048,16384 2560,512,8192 1024,1024,4096 5120,256,8192 \
  > $OUT/ab_bf16.jsonl 2> $OUT/ab_bf16.err || exit $?
timeout -k 10 600 python scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 5 --sessions 2 --kernels auto,auto@PDMB_SPLIT3=0,torch \
  --shapes 2560,512,16384 5120,256,16384 1536,1536,16384 \
  > $OUT/ab_fp8.jsonl 2> $OUT/ab_fp8.err || exit $?
echo done
