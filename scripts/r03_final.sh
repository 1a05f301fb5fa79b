#!/usr/bin/env bash
# Round-3 closing GPU session: smoke, the whole -m gpu suite and the default bench (scripts/gpu_check.sh), then
# the profile session of the same library (scripts/prof_r03.sh TAG).  usage: bash scripts/r03_final.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_check.sh "smoke tests bench" || exit $?
grep -q " failed" gpurun_out/pytest_gpu.log && { grep FAILED gpurun_out/pytest_gpu.log; exit 1; }
bash scripts/prof_r03.sh "${1:-v2}"
