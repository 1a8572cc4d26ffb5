#!/bin/bash
# Round 6 closing: the N > 1 job shape on the final shipping tree, rehearsed with
# 2 / 4 / 8 gloo ranks sharing one GPU (the driver's RCCL runs need a node).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/gpu_session.sh r8zm selflaunch2 selflaunch4 selflaunch8 || exit $?
echo "exit 0"
