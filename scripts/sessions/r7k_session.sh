#!/bin/bash
# round-5 session k: validation (r7i) then the second T192 A/B (r7j)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/r7i_session.sh && bash scripts/r7j_session.sh
