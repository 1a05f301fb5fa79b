#!/usr/bin/env bash
# Round-3 GPU session for the f64 instantiation of the fused kernel: its parity tests, then the f64 tube
# step per lane form against the generic f64 kernel (DTMPC_FAST64=0) at the bench batch and at 8,192.
# Each GPU step has its own time limit; any failure ends the session (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03_f64
mkdir -p "$OUT"
KEXPR=${1:-"fast64 or (tube_step_vs_oracle and f64) or (chunked and f64) or (gamma0 and f64) or closed_loop_vs_reference_loop_f64"}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 300 --timeout-method thread \
  -k "$KEXPR" > "$OUT/pytest.log" 2>&1
rc=$?
grep -E "PASS|FAIL|Error|fast64 vs|decisions" "$OUT/pytest.log" | tail -n 40
[ $rc -eq 0 ] || exit $rc
for B in 65536 8192; do
  for v in "fast 1" "fast 2" "generic 1"; do
    set -- $v
    F=1; [ "$1" = generic ] && F=0
    DTMPC_FAST64=$F DTMPC_TUBE_LANES=$2 timeout -k 10 300 python bench.py --dtype f64 --batch $B --steps 5 --warmup 1 \
      --no-cpu --no-steady --no-extra > "$OUT/b${B}_$1_l$2.log" 2>&1 || exit $?
    echo "B=$B $1 lanes=$2 $(grep -o '"kernel_ms": [0-9.]*' "$OUT/b${B}_$1_l$2.log") $(grep -o '"value": [0-9.e+]*' "$OUT/b${B}_$1_l$2.log")" | tee -a "$OUT/sweep.txt"
  done
done
