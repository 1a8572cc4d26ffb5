#!/bin/bash
# Kernel + memory-copy trace of ONE rank of a 2-rank gloo rehearsal of the
# peer-memory collectives on one GPU (scripts/ipc_pulls.py by default; PROG=
# bench.py ARGS="--gpus 2 --dist-backend gloo ... --allgather ipc" for the bench).
# Rank 1 runs plain in the background; rank 0 runs under rocprofv3 (tracing
# every rank through torchrun crashed rocprofv3's teardown, with or without
# IPC: profiles/r4t_rocprof_ipc2_exit_segv.log). ENGINE: kernel | sdma.
#   OUT=gpurun_out/x ENGINE=sdma bash scripts/ipc_trace2.sh
set -u
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${OUT:-$ROOT/gpurun_out/ipc_trace2}
ENGINE=${ENGINE:-kernel}
mkdir -p "$OUT"
export MASTER_ADDR=127.0.0.1 MASTER_PORT=${PORT:-29641} WORLD_SIZE=2 PDMB_IPC_ENGINE=$ENGINE
PROG=${PROG:-scripts/ipc_pulls.py}  # or bench.py with ARGS
ARGS=${ARGS:-}
(export RANK=1 LOCAL_RANK=1; cd "$ROOT" && timeout -k 10 300 python3 "$PROG" $ARGS > "$OUT/rank1_$ENGINE.log" 2>&1) &
P1=$!
export RANK=0 LOCAL_RANK=0 TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/rp_$ENGINE" -o r0 -- \
  python3 "$ROOT/$PROG" $ARGS > "$OUT/rank0_$ENGINE.log" 2>&1
R0=$?
wait $P1
R1=$?
echo "rank0 rc=$R0 rank1 rc=$R1"
[ $R0 -eq 0 ] && [ $R1 -eq 0 ]
