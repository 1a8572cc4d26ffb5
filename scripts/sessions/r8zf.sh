#!/bin/bash
# Round 6 session ZF (shipping build): first-launch screen of the shipping
# kernels: each probe is one auto GEMM in a fresh process under a 45 s limit
# (the r8s-r8u hang was on first launches). W4S bf16 / fp16, fp8 W4S / W4,
# f32_w4l, lean f32_t128, T128 / T256x128, repeated.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r8zf; mkdir -p $OUT
for rep in 1 2 3; do
  for s in "bfloat16 16384 16384 16384" "bfloat16 8192 8192 8192" "float16 8192 8192 4096" "float8_e4m3fn 8192 8192 8192" \
           "float8_e4m3fn 4096 4096 4096" "float32 8192 8192 8192" "float32 4096 4096 4096" "float32 4096 1024 4096" \
           "bfloat16 4096 2048 4096" "bfloat16 4096 1024 4096" "float8_e4m3fn 16384 16384 512"; do
    timeout -k 5 45 python scripts/cold_probe.py $s >> $OUT/probe.jsonl 2>> $OUT/probe.err || { echo "probe $s rc=$?"; tail -3 $OUT/probe.jsonl; exit 1; }
  done
  echo "rep $rep done $(date +%T)"
done
python3 -c "
import json; r=[json.loads(l) for l in open('$OUT/probe.jsonl')]
print(len(r), 'probes;', sum(x['exact'] for x in r), 'exact;', sorted(set(x['kernel'] for x in r)))"
echo "exit 0"
