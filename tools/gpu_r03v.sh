#!/bin/bash
# HEAD: the whole -m gpu suite, the config-2 profile (rocprof trace + PMC + bench),
# then the config-4 profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_suite.sh r03v r03v || exit 1
bash profiles/run_profile.sh r03v_c4 --config 4 || { echo C4_PROFILE_FAIL; exit 1; }
echo C4_OK
