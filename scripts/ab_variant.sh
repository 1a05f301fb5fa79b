#!/usr/bin/env bash
# A/B kernel variants on the GPU box: GPU parity tests + quick bench with the product library and with
# each libdtmpc_<variant>.so (build.py --variant).  usage: bash scripts/ab_variant.sh "V1 V2" [pytest -k expr]
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
for v in $V; do
  export DTMPC_LIBRARY=$PWD/$LIBDIR/libdtmpc_$v.so
  step tests_$v 900 python -m pytest tests -m gpu -q -rf "${KARG[@]}"
  step bench_$v 300 python bench.py --steps 5 --warmup 1 --no-cpu
done
exit 0
