#!/bin/bash
# Launcher for matmul_scaling_benchmark.py (reference: run_scaling_benchmark.sh).
# Usage: ./run_scaling_benchmark.sh [NUM_GPUS=2] [MODE=independent] [DTYPE=bfloat16] [extra flags...]
#   MODE: independent | batch_parallel | matrix_parallel
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
NUM_GPUS=${1:-2}
MODE=${2:-independent}
DTYPE=${3:-bfloat16}
shift $(( $# > 3 ? 3 : $# ))
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}
if [ "${RCCL_DEBUG:-0}" = "1" ]; then export NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,ENV; fi

echo "Starting matrix multiplication scaling benchmark"
echo "  GPUs: $NUM_GPUS"
echo "  Mode: $MODE (independent, batch_parallel, matrix_parallel)"
echo "  Data type: $DTYPE"
echo ""
ARGS=(--sizes 4096 8192 16384 --iterations 50 --warmup 10 --mode "$MODE" --dtype "$DTYPE" "$@")
if [ "$NUM_GPUS" -eq 1 ]; then
    echo "Running in single GPU mode..."
    exec python3 "$HERE/matmul_scaling_benchmark.py" "${ARGS[@]}"
else
    echo "Running in distributed mode with $NUM_GPUS GPUs..."
    exec python3 -m torch.distributed.run --nnodes=1 --nproc-per-node="$NUM_GPUS" \
        --master-addr=127.0.0.1 --master-port="${MASTER_PORT:-29503}" \
        "$HERE/matmul_scaling_benchmark.py" "${ARGS[@]}"
fi
