#!/usr/bin/env bash
# f64 log experiment (libdtmpc_exp.so: the product library with dtmpc_fast64 rebuilt from a scratch copy whose
# smooth-min log is fdlibm's e_log, 5 obstacles only): f64 parity tests against it, then same-box timing
# against the product library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/exp
mkdir -p "$OUT"
D=$PWD/differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt
DTMPC_LIBRARY=$D/libdtmpc_exp.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -s --timeout 300 \
  --timeout-method thread -k "fast64 or (tube_step_vs_oracle and f64) or closed_loop_vs_reference_loop_f64" > "$OUT/pytest.log" 2>&1
rc=$?
grep -E "passed|failed|fast64 vs generic lanes=1\] (x|Unom):" "$OUT/pytest.log" | tail -n 5
[ $rc -le 1 ] || exit $rc
for BL in "65536 1" "8192 4"; do
  set -- $BL
  for lib in libdtmpc.so libdtmpc_exp.so; do
    DTMPC_LIBRARY=$D/$lib DTMPC_TUBE_LANES=$2 timeout -k 10 300 python bench.py --dtype f64 --batch $1 --steps 10 --warmup 2 \
      --no-cpu --no-steady --no-extra > "$OUT/$lib.$1.log" 2>&1 || exit $?
    echo "$lib B=$1 lanes=$2 $(grep -o '"kernel_ms": [0-9.]*' "$OUT/$lib.$1.log")" | tee -a "$OUT/ab.txt"
  done
done
