#!/usr/bin/env bash
# Phase attribution + A/B on the GPU box: per-phase cycles of the fast kernel (profiling variant) at one
# and two lanes per trajectory, then short benches of the listed library variants and lane counts.
# usage: bash scripts/ab_phase.sh "VARIANTS" (each V = libdtmpc_V.so, "base" = libdtmpc.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIBDIR=$PWD/differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt
if [ -f $LIBDIR/libdtmpc_prof.so ]; then
  for L in ${PLANES:-1 2}; do
    DTMPC_TUBE_LANES=$L DTMPC_LIBRARY=$LIBDIR/libdtmpc_prof.so timeout -k 10 300 python scripts/phase_prof.py > gpurun_out/phase_l$L.log 2>&1; rc=$?
    echo "[ab] phase lanes=$L rc=$rc"; cat gpurun_out/phase_l$L.log | grep -v amdgpu.ids
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
fi
for v in ${1:-base}; do
  lib=$LIBDIR/libdtmpc_$v.so; [ "$v" = base ] && lib=$LIBDIR/libdtmpc.so
  for L in ${LANES:-1 2}; do
    DTMPC_TUBE_LANES=$L DTMPC_LIBRARY=$lib timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu > gpurun_out/b_${v}_l$L.log 2>&1; rc=$?
    echo "[ab] $v lanes=$L bench rc=$rc $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/b_${v}_l$L.log) $(grep -o '"flagged_trajectories": [0-9]*' gpurun_out/b_${v}_l$L.log)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
exit 0
