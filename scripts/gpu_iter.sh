#!/usr/bin/env bash
# One build -> measure iteration on the GPU box: the full GPU parity suite, the phase attribution of
# the fast kernel (profiling variant, if built) and a short bench at one lane per trajectory.
# usage: bash scripts/gpu_iter.sh [pytest -k expr]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
K=${1:-}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "[iter] tests rc=$rc: $(tail -n 1 gpurun_out/pytest_gpu.log)"
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -20; [ $rc -ne 1 ] && exit $rc; fi
LANES="${LANES:-1}" bash scripts/ab_phase.sh "${VARIANTS:-base}"
