#!/bin/bash
# Round 6 closing: every reference launcher at N = 1 on the final shipping build,
# with --check, plus run_benchmark.sh in fp16 and exact fp32.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/gpu_session.sh r8zi cli cli_dtypes || exit $?
echo "exit 0"
