#!/bin/bash
# Round 6 closing validation A (shipping build): the whole GPU suite, smoke, the
# driver-form bench and its kernel trace; then auto vs hipBLASLt on the fp8
# short-K grids the K4 form now streams (settled, two sessions).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/gpu_session.sh r8f tests smoke bench rocprof_bench || exit $?
timeout -k 10 400 python scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 4 --iters 20 --settle 1 --sessions 2 \
  --kernels auto,torch --shapes 16384,16384,512 8192,8192,512 16384,8192,512 6144,6144,512 \
  > gpurun_out/r8f/ab_fp8_k512_auto.jsonl 2> gpurun_out/r8f/ab_fp8_k512_auto.err || exit $?
grep '"summary"' gpurun_out/r8f/ab_fp8_k512_auto.jsonl | cut -c1-200
