#!/bin/bash
# Round 6 closing validation E (the final shipping tree): the whole GPU suite,
# smoke, bench and its kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/gpu_session.sh r8zh tests smoke bench rocprof_bench || exit $?
echo "exit 0"
