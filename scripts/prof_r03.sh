#!/usr/bin/env bash
# Round-3 profile session (GPU box): the exact bench invocation under rocprofv3 --kernel-trace --stats
# (23 launches, the 3 warm-up ones excluded by index in scripts/trace_summary.py), then the HBM counter
# passes (one counter group per pass, no trace domains with --pmc) and the known-byte calibration, then
# one plain bench run in the same session for the side-by-side kernel_ms.
# usage: bash scripts/prof_r03.sh TAG
set -u
TAG=${1:-v1}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
run() {
  echo "[prof] $*"
  timeout -k 10 300 "$@" >> "$OUT/prof.log" 2>&1
  local rc=$?
  echo "[prof] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
BENCH="bench.py --no-cpu --no-steady"
run rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $BENCH
python3 scripts/trace_summary.py "$OUT/trace" "$OUT/trace_summary.json" --warmup 3 || exit 1
SHORT="bench.py --steps 5 --warmup 1 --no-cpu --no-steady --no-extra"
run rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 $SHORT
run rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 $SHORT
run rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d "$OUT/sq1" -o run --output-format csv -- python3 $SHORT
run rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d "$OUT/sq2" -o run --output-format csv -- python3 $SHORT
run rocprofv3 --pmc FETCH_SIZE -d "$OUT/cal_fetch" -o run --output-format csv -- python3 scripts/pmc_calib.py
run rocprofv3 --pmc WRITE_SIZE -d "$OUT/cal_write" -o run --output-format csv -- python3 scripts/pmc_calib.py
python3 scripts/pmc_summary.py "$OUT" "$OUT/pmc.json" --batch 65536 > /dev/null || exit 1
timeout -k 10 300 python3 bench.py --no-cpu > "$OUT/bench.json.log" 2>&1 || exit 1
tail -n 1 "$OUT/bench.json.log"
echo "[prof] done"
