#!/bin/bash
# Round 6 closing validation F (the final shipping tree, after the thin-round
# experiment arms): the whole GPU suite, smoke, bench and its kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/gpu_session.sh r8zk tests smoke bench rocprof_bench || exit $?
echo "exit 0"
