#!/usr/bin/env bash
# Round-4 evidence for the small-batch legs and the receding driver (GPU box): the B = 4,096 tube step (BASELINE
# configs 3/4, four lanes per trajectory) under rocprofv3 --kernel-trace --stats and its HBM counter passes (one
# counter group per pass, no trace domains with --pmc) + the known-byte calibration, summarised for bench.py's
# config3/config4 `traffic`; then a kernel trace of the receding driver (scripts/bench_callers.py --receding-only).
# usage: bash scripts/prof_r04_small.sh TAG
set -u
TAG=${1:-v1}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_small_$TAG
mkdir -p "$OUT"
run() {
  echo "[prof] $*"
  timeout -k 10 300 "$@" >> "$OUT/prof.log" 2>&1
  local rc=$?
  echo "[prof] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
pmc() {  # one counter pass: a hard kill at 90 s (a pass that asks for more than the block holds hangs)
  echo "[prof] pmc $*"
  timeout -s KILL 90 rocprofv3 "$@" >> "$OUT/prof.log" 2>&1
  local rc=$?
  echo "[prof] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
B4="bench.py --batch 4096 --steps 20 --warmup 8 --no-cpu --no-steady --no-extra"
run rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $B4
python3 scripts/trace_summary.py "$OUT/trace" "$OUT/trace_summary.json" --warmup 8 --timed-last 20 --batch 4096 --algo-bytes 1123631104 || exit 1
S4="bench.py --batch 4096 --steps 5 --warmup 1 --no-cpu --no-steady --no-extra"
pmc --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 $S4
pmc --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 $S4
pmc --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d "$OUT/sq1" -o run --output-format csv -- python3 $S4
pmc --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d "$OUT/sq2" -o run --output-format csv -- python3 $S4
pmc --pmc FETCH_SIZE -d "$OUT/cal_fetch" -o run --output-format csv -- python3 scripts/pmc_calib.py
pmc --pmc WRITE_SIZE -d "$OUT/cal_write" -o run --output-format csv -- python3 scripts/pmc_calib.py
python3 scripts/pmc_summary.py "$OUT" "$OUT/pmc.json" --batch 4096 > /dev/null || exit 1
run rocprofv3 --kernel-trace --stats -d "$OUT/receding" -o run --output-format csv -- python3 scripts/bench_callers.py --receding-only --f64
echo "[prof] done"
