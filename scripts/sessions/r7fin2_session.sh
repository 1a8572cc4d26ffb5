#!/bin/bash
# round-5 closing validation (second, after the small-grid planner work): GPU suite, smoke, driver-form bench, kernel trace of the bench, 2-/4-rank gloo rehearsals
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/gpu_session.sh r7fin2 tests smoke bench rocprof_bench selflaunch2 selflaunch4
