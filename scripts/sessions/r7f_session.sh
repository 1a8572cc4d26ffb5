#!/bin/bash
# round-5 session f: 192-row tiles — race screen, shape fuzz, the 20-shape sweep
# (auto vs auto without them vs hipBLASLt), cross-session A/B of the target shapes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; export TMPDIR=/tmp; OUT=gpurun_out/r7f; mkdir -p $OUT
SW="4096,4096,1024 4096,4096,14336 4096,14336,4096 8192,8192,1024 8192,8192,28672 8192,28672,8192 16384,4096,4096 4096,16384,4096 2048,8192,8192 8192,2048,8192 12288,12288,4096 4096,12288,12288 10240,8192,2048 6144,6144,12288 1024,16384,16384 16384,1024,16384 5120,5120,5120 7168,7168,7168 3072,8192,3072 11008,4096,4096 3072,3072,3072 2304,2304,4096"
step() { local n=$1 t=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; grep '^{' $OUT/$n.log > $OUT/$n.jsonl; tail -2 $OUT/$n.log | cut -c1-200; [ $rc -eq 0 ] || { echo "$n rc=$rc"; exit $rc; }; }
step race 300 python scripts/race_screen.py --reps 100 --kernels t192,t192x128,fp8_t192:float8_e4m3fn,fp8_t192x128:float8_e4m3fn
step fuzz 300 python scripts/shape_fuzz.py --count 40 --seed 5
for dt in bfloat16 float16 float8_e4m3fn; do
  step sweep_$dt 500 python scripts/ab_kernels.py --dtype $dt --kernels auto,auto@PDMB_T192=0,torch --rounds 3 --iters 10 --shapes $SW
done
step sessions 500 python scripts/ab_kernels.py --dtype bfloat16 --kernels auto,torch --rounds 5 --sessions 2 --shapes 3072,3072,3072 2304,2304,4096
step sessions_fp16 400 python scripts/ab_kernels.py --dtype float16 --kernels auto,torch --rounds 5 --sessions 2 --shapes 3072,3072,3072 2304,2304,4096
step sessions_fp8 400 python scripts/ab_kernels.py --dtype float8_e4m3fn --kernels auto,torch --rounds 5 --sessions 2 --shapes 3072,3072,3072 2304,2304,4096 5120,5120,4096 8192,2048,8192
echo "== done $(date +%T)"
