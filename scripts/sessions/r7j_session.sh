#!/bin/bash
# round-5 session j: T192 on every grid the planner now gives it (auto vs PDMB_T192=0 vs hipBLASLt)
# (first run: bf16 set 1 -> profiles/r7j_t192_ab_bf16.jsonl; this set: the multi-wave T192x128 picks)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; export TMPDIR=/tmp; OUT=gpurun_out/r7j; mkdir -p $OUT
BF="2304,4096,16384 3584,2560,16384 4608,2048,16384 9216,1024,16384 1024,9216,16384 2560,4608,16384 2304,8192,16384 3072,3584,8192 2048,4608,8192"
F8="6144,6144,6144 6144,3072,8192 12288,1536,8192 3040,3040,8192 2304,2304,8192 4608,1024,8192 1536,6144,8192 3072,1536,16384 3040,6080,16384 2048,2304,8192"
echo "== bf16 $(date +%T)"
timeout -k 10 500 python scripts/ab_kernels.py --kernels auto,auto@PDMB_T192=0,torch --shapes $BF --rounds 5 --sessions 2 > $OUT/ab_bf16.jsonl 2> $OUT/ab_bf16.err || exit $?
echo "== fp8 $(date +%T)"
timeout -k 10 500 python scripts/ab_kernels.py --kernels auto,auto@PDMB_T192=0,torch --dtype float8_e4m3fn --shapes $F8 --rounds 5 --sessions 2 > $OUT/ab_fp8.jsonl 2> $OUT/ab_fp8.err || exit $?
echo "== done $(date +%T)"
