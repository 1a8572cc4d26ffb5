#!/bin/bash
# Round 6 session A: the self-checking bench on one GPU (headline + secondary
# modes, every dtype once), then the ws = 8 driver form on one GPU (8 gloo
# ranks share it) at 4096, phases traced.
set -o pipefail
mkdir -p gpurun_out/r8a
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 240 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
  > gpurun_out/r8a/bench1.json 2> gpurun_out/r8a/bench1.err &&
for dt in float32 float8_e4m3fn float16; do
  timeout -k 10 150 python -u bench.py --dtype $dt --size 8192 --steps 5 --warmup 2 --extra-steps 3 \
    > gpurun_out/r8a/bench1_$dt.json 2> gpurun_out/r8a/bench1_$dt.err || exit $?
done &&
PDMB_BENCH_TRACE=1 timeout -k 10 300 python -u bench.py --gpus 8 --dist-backend gloo --size 4096 \
  --steps 3 --warmup 1 --extra-steps 2 --extra-warmup 1 \
  > gpurun_out/r8a/bench8_4k.json 2> gpurun_out/r8a/bench8_4k.err
echo "exit $?"
