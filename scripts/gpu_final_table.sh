#!/bin/bash
# Round-2 summary table: the auto kernel vs hipBLASLt in the same process for
# every dtype at the reference's default sizes (4k / 8k / 16k).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for dt in bfloat16 float16 float32 float8_e4m3fn; do
  timeout -k 10 400 python scripts/ab_kernels.py --dtype $dt --kernels auto,torch \
      --sizes 4096 8192 16384 --rounds 5 --iters 10 > gpurun_out/final_$dt.jsonl 2>> gpurun_out/final.err
  rc=$?
  echo "$dt rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
