#!/usr/bin/env bash
# A/B a kernel variant on the GPU box: GPU parity tests + quick bench with the product library and with
# libdtmpc_<variant>.so (build.py --variant).  usage: bash scripts/ab_variant.sh VARIANT [pytest -k expr]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=$1
K=${2:-}
mkdir -p gpurun_out
LIBDIR=differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[ab] $name rc=$rc"; tail -n 3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
KARG=(); [ -n "$K" ] && KARG=(-k "$K")
step tests_base 900 python -m pytest tests -m gpu -q -rf "${KARG[@]}"
step bench_base 300 python bench.py --steps 5 --warmup 1 --no-cpu
export DTMPC_LIBRARY=$PWD/$LIBDIR/libdtmpc_$V.so
step tests_$V 900 python -m pytest tests -m gpu -q -rf "${KARG[@]}"
step bench_$V 300 python bench.py --steps 5 --warmup 1 --no-cpu
exit 0
