#!/usr/bin/env bash
# Isolation run: the one-lane f64 fused tests against variant libraries (libdtmpc_<v>.so), each in its own
# time-limited pytest process; stops at the first crash / timeout.  usage: bash scripts/r03_isolate.sh "va vb" "-k expr"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/isolate
mkdir -p "$OUT"
D=$PWD/differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt
for v in $1; do
  DTMPC_LIBRARY=$D/libdtmpc_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -s \
    --timeout 200 --timeout-method thread -k "$2" > "$OUT/$v.log" 2>&1
  rc=$?
  echo "== $v rc=$rc"; grep -E "passed|failed|fast64 vs generic lanes=1\] x:" "$OUT/$v.log" | tail -n 4
  [ $rc -le 1 ] || exit $rc
done
