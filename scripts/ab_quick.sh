#!/usr/bin/env bash
# Quick A/B on the GPU box: for each variant library, the tube-step parity tests + a short bench.
# usage: bash scripts/ab_quick.sh "V1 V2" [pytest -k expr]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIBDIR=differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt
K=${2:-tube_step}
for v in $1; do
  export DTMPC_LIBRARY=$PWD/$LIBDIR/libdtmpc_$v.so
  timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "$K" > gpurun_out/t_$v.log 2>&1; rc=$?
  echo "[ab] $v tests rc=$rc $(tail -n 1 gpurun_out/t_$v.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu > gpurun_out/b_$v.log 2>&1; rc=$?
  echo "[ab] $v bench rc=$rc $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/b_$v.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
exit 0
