#!/bin/bash
# Round-2 pass M: which hipBLASLt kernels win where this repo still trails (fp8 at one 256^2 tile
# per CU, exact fp32): rocprofv3 kernel traces of the vendor calls.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2m}
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/fp8 -o vk -- python3 scripts/vendor_kernels.py \
  --dtype float8_e4m3fn --shapes 4096,4096,4096 8192,2048,8192 8192,8192,8192 > $OUT/fp8.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/f32 -o vk -- python3 scripts/vendor_kernels.py \
  --dtype float32 --shapes 16384,16384,16384 8192,8192,8192 --iters 5 > $OUT/f32.log 2>&1 || exit $?
ls -R $OUT | head -20
