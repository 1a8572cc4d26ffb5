#!/bin/bash
# round-5 session aa: fp8 W4S with the C stores folded into each tile's last K-tile (ktile_w4s_last)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7aa; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_fp8_gpu.py tests/test_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "fp8" > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/race_screen.py --tails --reps 20 > $OUT/race_tails.jsonl 2> $OUT/race.err || exit $?
grep -c '"bad_runs": 0' $OUT/race_tails.jsonl
timeout -k 10 900 python scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 5 --sessions 2 \
  --kernels auto,auto@PDMB_FP8_W4S_FUSE=0,torch \
  --shapes 8192,8192,1024 16384,16384,2048 8192,8192,8192 16384,16384,16384 4096,16384,4096 10240,8192,2048 \
           5120,5120,5120 16384,2048,16384 \
  > $OUT/ab_fp8_w4s_fuse.jsonl 2> $OUT/ab.err || exit $?
echo done
