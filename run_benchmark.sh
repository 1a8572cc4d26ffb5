#!/bin/bash
# Launcher for matmul_benchmark.py (reference: run_benchmark.sh).
# Usage: ./run_benchmark.sh [NUM_GPUS=1] [DTYPE=bfloat16] [extra matmul_benchmark.py flags...]
# Differences: paths resolve relative to this file (works from any cwd), all
# visible GPUs are usable (no ROCR/HIP_VISIBLE_DEVICES=0..5 cap), rendezvous on
# 127.0.0.1, RCCL debug only when RCCL_DEBUG=1.
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
NUM_GPUS=${1:-1}
DTYPE=${2:-bfloat16}
shift $(( $# > 2 ? 2 : $# ))
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}
if [ "${RCCL_DEBUG:-0}" = "1" ]; then export NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,ENV; fi

echo "Starting distributed matrix multiplication benchmark with $NUM_GPUS GPU(s)"
echo "Data type: $DTYPE"
echo ""
ARGS=(--sizes 4096 8192 16384 --iterations 50 --warmup 10 --dtype "$DTYPE" "$@")
if [ "$NUM_GPUS" -eq 1 ]; then
    echo "Running in single GPU mode..."
    exec python3 "$HERE/matmul_benchmark.py" "${ARGS[@]}"
else
    echo "Running in distributed mode with $NUM_GPUS GPUs..."
    exec python3 -m torch.distributed.run --nnodes=1 --nproc-per-node="$NUM_GPUS" \
        --master-addr=127.0.0.1 --master-port="${MASTER_PORT:-29500}" \
        "$HERE/matmul_benchmark.py" "${ARGS[@]}"
fi
