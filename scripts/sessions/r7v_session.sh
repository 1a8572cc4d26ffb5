#!/bin/bash
# round-5 session v: the reference CLI at small squares, native vs torch backend, every dtype
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7v; mkdir -p $OUT
for dt in bfloat16 float16 float32 float8_e4m3fn; do
  for be in native torch; do
    timeout -k 10 300 python matmul_benchmark.py --sizes 1024 2048 4096 --dtype $dt --backend $be \
      --json $OUT/cli_${dt}_${be}.json > $OUT/cli_${dt}_${be}.log 2>&1 || exit $?
  done
done
grep -h "TFLOPS" $OUT/cli_*_native.log | head -20
echo done
