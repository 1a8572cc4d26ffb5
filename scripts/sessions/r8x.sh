#!/bin/bash
# Round 6 closing validation B (shipping build, after the r8l-r8w fp32 work
# left the shipping kernels unchanged): the whole GPU suite, smoke, the
# driver-form bench and its kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/gpu_session.sh r8x tests smoke bench rocprof_bench || exit $?
echo "exit 0"
