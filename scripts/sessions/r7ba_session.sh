#!/bin/bash
# round-5 session ba: short-K grids (epilogue-heavy), auto vs hipBLASLt, settled,
# bf16 and fp8
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7ba; mkdir -p $OUT
for dt in bfloat16 float8_e4m3fn; do
timeout -k 10 600 python scripts/ab_kernels.py --dtype $dt --rounds 4 --iters 20 --settle 1 --sessions 2 \
  --kernels auto,torch \
  --shapes 8192,8192,1024 16384,16384,512 4096,4096,512 8192,4096,1024 16384,8192,1024 16384,16384,1024 \
  > $OUT/ab_${dt}_short_k.jsonl 2> $OUT/ab_${dt}.err || exit $?
done
echo done
