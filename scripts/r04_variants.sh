#!/usr/bin/env bash
# Round-4 root-cause variant libraries (CPU, this container): the obstacle count of the paper (M = 5) only,
# each one translation unit rebuilt (build.py --variant, the rest from the product objects).
#   lds0 / lds1        f32 tube kernel, gains in the workspace / the general 40-byte records in LDS (13 steps)
#   far1 / far0        f64 tube kernel, OCML sincos far branch out of line (default) / inlined
#   *c                 the same with -ffp-contract=off on that unit
set -eu
cd "$(dirname "$0")/.."
B=differentiable-tube-mpc_amd/build.py
M="-D DTMPC_FAST_M_ONLY=5"
python $B --variant lds0 $M --only dtmpc_fast &
python $B --variant lds1 $M -D DTMPC_FAST_LDS_STEPS=13 -D DTMPC_FAST_LDS_GENERAL=1 --only dtmpc_fast &
DTMPC_EXTRA_FLAGS=-ffp-contract=off python $B --variant lds0c $M --only dtmpc_fast &
DTMPC_EXTRA_FLAGS=-ffp-contract=off python $B --variant lds1c $M -D DTMPC_FAST_LDS_STEPS=13 -D DTMPC_FAST_LDS_GENERAL=1 --only dtmpc_fast &
wait
python $B --variant far1 $M --only dtmpc_fast64 &
python $B --variant far0 $M -D DTMPC_FAST64_FAR=0 --only dtmpc_fast64 &
DTMPC_EXTRA_FLAGS=-ffp-contract=off python $B --variant far1c $M --only dtmpc_fast64 &
DTMPC_EXTRA_FLAGS=-ffp-contract=off python $B --variant far0c $M -D DTMPC_FAST64_FAR=0 --only dtmpc_fast64 &
wait
