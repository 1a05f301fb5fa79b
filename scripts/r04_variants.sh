#!/usr/bin/env bash
# Round-4 experiment libraries (CPU, this container): the paper's obstacle count (M = 5) only, one translation
# unit rebuilt per variant and linked against the product build's other objects (build.py --on-product).
#   lds0 / lds1        f32 tube kernel, gains in the workspace / the general 40-byte records in LDS (13 steps)
#   far1 / far0        f64 tube kernel, OCML sincos far branch out of line (default) / inlined
#   *c                 the same with -ffp-contract=off on that unit
#   lead3 / lead4      four-lane line search with its step inputs 3 / 4 steps ahead (default 2)
set -eu
cd "$(dirname "$0")/.."
B="python differentiable-tube-mpc_amd/build.py --on-product"
M="-D DTMPC_FAST_M_ONLY=5"
$B --variant lds0 $M --only dtmpc_fast &
$B --variant lds1 $M -D DTMPC_FAST_LDS_STEPS=13 -D DTMPC_FAST_LDS_GENERAL=1 --only dtmpc_fast &
DTMPC_EXTRA_FLAGS=-ffp-contract=off $B --variant lds0c $M --only dtmpc_fast &
DTMPC_EXTRA_FLAGS=-ffp-contract=off $B --variant lds1c $M -D DTMPC_FAST_LDS_STEPS=13 -D DTMPC_FAST_LDS_GENERAL=1 --only dtmpc_fast &
$B --variant far1 $M --only dtmpc_fast64 &
$B --variant far0 $M -D DTMPC_FAST64_FAR=0 --only dtmpc_fast64 &
wait
DTMPC_EXTRA_FLAGS=-ffp-contract=off $B --variant far1c $M --only dtmpc_fast64 &
DTMPC_EXTRA_FLAGS=-ffp-contract=off $B --variant far0c $M -D DTMPC_FAST64_FAR=0 --only dtmpc_fast64 &
$B --variant lead3 $M -D DTMPC_FAST_LS_LEAD4=3 --only dtmpc_fast &
$B --variant lead4 $M -D DTMPC_FAST_LS_LEAD4=4 --only dtmpc_fast &
wait
