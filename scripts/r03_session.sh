#!/usr/bin/env bash
# Round-3 GPU session: focused parity tests of the fast kernel, then a batch x lanes sweep of the tube
# step.  Each GPU step has its own time limit; any failure ends the session (no retries).
# usage: bash scripts/r03_session.sh [TAG] [pytest -k expression]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-a}
KEXPR=${2:-"lanes_bitwise or chunked or gamma0 or tube_step_vs_oracle"}
OUT=gpurun_out/r03_$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "$KEXPR" > "$OUT/pytest.log" 2>&1
rc=$?
tail -n 15 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
for B in 4096 8192 16384 32768 65536; do
  for L in 1 2 4; do
    [ "$B" -ge 32768 ] && [ "$L" = 4 ] && continue
    DTMPC_TUBE_LANES=$L timeout -k 10 120 python bench.py --batch $B --steps 10 --warmup 2 --no-cpu > "$OUT/b${B}_l$L.log" 2>&1 || exit $?
    echo "B=$B lanes=$L $(grep -o '"kernel_ms": [0-9.]*' "$OUT/b${B}_l$L.log") $(grep -o '"value": [0-9.e+]*' "$OUT/b${B}_l$L.log")" | tee -a "$OUT/sweep.txt"
  done
done
