#!/bin/bash
# Round-3 end: rocprofv3 kernel stats + PMC traffic of the default GraphSAGE bench, then smoke,
# the whole -m gpu suite and the default bench line (scripts/gpu_check.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/gpu_profile.sh || exit $?
bash scripts/gpu_check.sh
