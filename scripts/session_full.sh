#!/usr/bin/env bash
# Full GPU session: smoke, GPU parity suite, bench with CPU baseline, then rocprofv3 trace + PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
bash scripts/gpu_check.sh "smoke tests bench" "-x -v --timeout 120 --timeout-method thread" || exit $?
grep -q "rc=0" <(grep "pytest_gpu rc" gpurun_out/session.log) || { echo "tests failed"; exit 1; }
bash scripts/prof_pmc.sh "$TAG" --steps 3 --warmup 1 --no-cpu
