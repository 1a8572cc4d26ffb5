#!/bin/bash
# Full 1/2/4/8-GPU scaling sweep on one node (the BASELINE metric):
# every scaling mode (+ overlap variants) at 16k bf16 → results/sweep.jsonl →
# scaling table. Usage: scripts/scaling_sweep.sh [GPU counts...] (default 1 2 4 8)
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
COUNTS=${*:-1 2 4 8}
OUT=${OUT:-$HERE/results/sweep.jsonl}
SIZES=${SIZES:-16384}
mkdir -p "$(dirname "$OUT")"
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}
PORT=29800
for n in $COUNTS; do
  for spec in "independent" "batch_parallel" "batch_parallel --overlap" "matrix_parallel" "matrix_parallel --overlap" "ring_parallel"; do
    PORT=$((PORT + 1))
    # shellcheck disable=SC2086
    timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node="$n" \
      --master-addr=127.0.0.1 --master-port=$PORT "$HERE/matmul_scaling_benchmark.py" \
      --sizes $SIZES --iterations 50 --warmup 10 --dtype bfloat16 --mode $spec --json "$OUT"
  done
done
python3 "$HERE/scripts/scaling_table.py" "$OUT" --markdown
