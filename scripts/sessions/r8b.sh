#!/bin/bash
# Round 6 session B: the driver's ws = 8 job shape rehearsed on one GPU at the
# DEFAULT size and flags (16k bf16: headline, rank-0 references, serialized and
# overlapped batch / matrix modes with auto collectives, every mode checked),
# 8 gloo ranks sharing the GPU, each phase traced with time and peak memory.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r8b
PDMB_BENCH_TRACE=1 timeout -k 10 900 python -u bench.py --gpus 8 --dist-backend gloo \
  > gpurun_out/r8b/bench8_16k.json 2> gpurun_out/r8b/bench8_16k.err
echo "exit $?"
