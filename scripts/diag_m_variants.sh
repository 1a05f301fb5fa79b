#!/usr/bin/env bash
# scripts/diag_m.py (receding part, M = 8) on A/B variant libraries named on the command line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/diagm
mkdir -p $O
for v in "$@"; do
  DIAG_M=8 DTMPC_LIBRARY=$PWD/differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt/libdtmpc_$v.so timeout -k 10 200 python scripts/diag_m.py > $O/v_$v.txt 2>&1 || exit $?
done
