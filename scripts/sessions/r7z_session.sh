#!/bin/bash
# round-5 session z: the 3-way reducer prefetch (T128, 4-stage fp32 tiles): tests, then A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7z; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_fp8_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "split3 or splitk or tiled_random or tile_family or f32_t128" > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/ab_kernels.py --dtype bfloat16 --rounds 7 --sessions 2 \
  --kernels auto,auto@PDMB_SPLITK_PREFETCH=0,auto@PDMB_SPLIT3=0,torch \
  --shapes 1024,1024,4096 512,2048,4096 2048,512,4096 2560,512,8192 \
  > $OUT/ab_bf16_split3_pf.jsonl 2> $OUT/ab_bf16.err || exit $?
timeout -k 10 600 python scripts/ab_kernels.py --dtype bfloat16 --rounds 5 --sessions 2 --kernels auto,torch \
  --shapes 4096,1024,4096 2048,2048,2048 > $OUT/ab_bf16_t128_unsplit.jsonl 2> $OUT/ab_bf16_u.err || exit $?
timeout -k 10 600 python scripts/ab_kernels.py --dtype float32 --rounds 5 --sessions 2 \
  --kernels auto,auto@PDMB_SPLITK_PREFETCH=0,torch --shapes 1536,1536,4096 2560,256,8192 4096,1024,4096 \
  > $OUT/ab_f32_split3_pf.jsonl 2> $OUT/ab_f32.err || exit $?
echo done
