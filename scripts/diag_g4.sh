#!/usr/bin/env bash
# the f64 general-record tube kernel at M = 4 (tests/test_gpu_instantiations.py [f64-4-0]) on A/B variant libraries
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/diagg4
mkdir -p $O
for v in "$@"; do
  DTMPC_LIBRARY=$PWD/differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt/libdtmpc_$v.so timeout -k 10 200 \
    python -u -m pytest tests/test_gpu_instantiations.py -m gpu -q -s -rxX --timeout 120 --timeout-method thread \
    -k "test_tube_step_instantiations and f64-4-0" > $O/$v.txt 2>&1
  rc=$?
  echo "$v rc=$rc"
  [ $rc -le 1 ] || exit $rc
done
