#!/usr/bin/env bash
# Phase attribution of the fast tube step at several batch sizes, one lane per trajectory (profiling
# build libdtmpc_prof.so): per-step cycles of each phase on a quiet chip vs at full occupancy.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIB=$PWD/differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt/libdtmpc_prof.so
for B in ${BATCHES:-4096 65536}; do
  DTMPC_TUBE_LANES=1 DTMPC_LIBRARY=$LIB timeout -k 10 300 python scripts/phase_prof.py --batch $B > gpurun_out/phase_b$B.log 2>&1 || exit $?
  echo "== B=$B"; grep -v amdgpu.ids gpurun_out/phase_b$B.log | grep -v winners
done
