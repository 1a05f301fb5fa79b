#!/usr/bin/env bash
# Round-4 profile session (GPU box): the exact default bench invocation of the headline under rocprofv3
# --kernel-trace --stats (warm-up launches excluded by index in scripts/trace_summary.py), the HBM counter
# passes (one counter group per pass, no trace domains with --pmc), the known-byte calibration, the same for
# the f64 leg (fk64::tube_fast_kernel, workload tube_f64), then a plain bench run for the side-by-side numbers.
# usage: bash scripts/prof_r04.sh TAG
set -u
TAG=${1:-v1}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT" "$OUT/f64"
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
BENCH="bench.py --no-cpu --no-steady --no-extra --warmup 8"
run rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $BENCH
python3 scripts/trace_summary.py "$OUT/trace" "$OUT/trace_summary.json" --warmup 8 --timed-last 20 || exit 1
SHORT="bench.py --steps 5 --warmup 1 --no-cpu --no-steady --no-extra"
pmc --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 $SHORT
pmc --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 $SHORT
pmc --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d "$OUT/sq1" -o run --output-format csv -- python3 $SHORT
pmc --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d "$OUT/sq2" -o run --output-format csv -- python3 $SHORT
pmc --pmc FETCH_SIZE -d "$OUT/cal_fetch" -o run --output-format csv -- python3 scripts/pmc_calib.py
pmc --pmc WRITE_SIZE -d "$OUT/cal_write" -o run --output-format csv -- python3 scripts/pmc_calib.py
python3 scripts/pmc_summary.py "$OUT" "$OUT/pmc.json" --batch 65536 > /dev/null || exit 1
# the f64 leg (the reference's configured precision)
B64="bench.py --dtype f64 --steps 5 --warmup 1 --no-cpu --no-steady --no-extra"
run rocprofv3 --kernel-trace --stats -d "$OUT/f64/trace" -o run --output-format csv -- python3 $B64
python3 scripts/trace_summary.py "$OUT/f64/trace" "$OUT/f64/trace_summary.json" --warmup 8 --timed-last 5 --kernel fk64::tube_fast_kernel --algo-bytes 35956195328 || exit 1
pmc --pmc FETCH_SIZE -d "$OUT/f64/fetch" -o run --output-format csv -- python3 $B64
pmc --pmc WRITE_SIZE -d "$OUT/f64/write" -o run --output-format csv -- python3 $B64
pmc --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d "$OUT/f64/sq1" -o run --output-format csv -- python3 $B64
cp -r "$OUT/cal_fetch" "$OUT/cal_write" "$OUT/f64/"
python3 scripts/pmc_summary.py "$OUT/f64" "$OUT/f64/pmc.json" --batch 65536 --kernel fk64::tube_fast_kernel --workload tube_f64 > /dev/null || exit 1
timeout -k 10 600 python3 bench.py --no-cpu > "$OUT/bench.json.log" 2>&1 || exit 1
tail -n 1 "$OUT/bench.json.log"
echo "[prof] done"
