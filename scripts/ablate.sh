#!/usr/bin/env bash
# Phase profiles of several profiling builds (libdtmpc_<v>.so).  usage: bash scripts/ablate.sh "a0 a1 ..."
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in $1; do
  DTMPC_LIBRARY=$PWD/differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt/libdtmpc_$v.so \
    timeout -k 10 200 python scripts/phase_prof.py > gpurun_out/pp_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"; grep -E "^kernel|linesearch|backward|commit|per step" gpurun_out/pp_$v.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
