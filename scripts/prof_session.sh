#!/usr/bin/env bash
# Profile session (GPU box; rounds 5-6, ROUND=r06 by default), every bench leg's dominant kernel: rocprofv3 --kernel-trace --stats of the
# leg's own bench invocation (scripts/trace_summary.py: the timed launches' mean), then one --pmc pass per counter
# group (no trace domains with --pmc): calibrated HBM bytes (FETCH_SIZE / WRITE_SIZE against the known-byte
# record_stream_kernel) and the issue counters (SQ_INSTS_VALU per wave, GRBM_GUI_ACTIVE) bench.py turns into the
# HBM roofline's `traffic` and the `issue` roofline (scripts/pmc_summary.py; bench.py matches workload, batch and
# the library's sha256).  usage: [ROUND=r06] bash scripts/prof_session.sh TAG [LEG...]   (legs: tube tube_f64 tube_b4096
# nominal_ddp_f32 nominal_ddp_f64 receding_f32 receding_f64; default all)
set -u
TAG=${1:-v1}
shift
LEGS=${*:-tube tube_f64 tube_b4096 nominal_ddp_f32 nominal_ddp_f64 receding_f32 receding_f64}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${ROUND:-r06}_$TAG
mkdir -p "$OUT"
run() {
  echo "[prof] $*"
  timeout -k 10 300 "$@" >> "$OUT/prof.log" 2>&1
  local rc=$?
  echo "[prof] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
pmc() {  # one counter pass: a hard kill at 120 s (a pass that asks for more than the block holds hangs)
  echo "[prof] pmc $*"
  timeout -s KILL 120 rocprofv3 "$@" >> "$OUT/prof.log" 2>&1
  local rc=$?
  echo "[prof] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
pmc --pmc FETCH_SIZE -d "$OUT/cal/cal_fetch" -o run --output-format csv -- python3 scripts/pmc_calib.py
pmc --pmc WRITE_SIZE -d "$OUT/cal/cal_write" -o run --output-format csv -- python3 scripts/pmc_calib.py
leg() {  # NAME KERNEL WORKLOAD BATCH ALGO_BYTES TRACE_WARMUP TIMED SKIP -- bench args (SKIP: the counter passes'
  # first dispatches to drop -- the receding leg's warm-up launch is of another size)
  local name=$1 kern=$2 wl=$3 batch=$4 algo=$5 warm=$6 timed=$7 skip=$8
  shift 9
  local d="$OUT/$name"
  mkdir -p "$d"
  run rocprofv3 --kernel-trace --stats -d "$d/trace" -o run --output-format csv -- python3 bench.py "$@"
  python3 scripts/trace_summary.py "$d/trace" "$d/trace_summary.json" --warmup "$warm" --timed-last "$timed" \
    --kernel "$kern" --batch "$batch" --algo-bytes "$algo" > /dev/null || exit 1
  pmc --pmc FETCH_SIZE -d "$d/fetch" -o run --output-format csv -- python3 bench.py "$@"
  pmc --pmc WRITE_SIZE -d "$d/write" -o run --output-format csv -- python3 bench.py "$@"
  pmc --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    -d "$d/sq1" -o run --output-format csv -- python3 bench.py "$@"
  pmc --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES \
    -d "$d/sq2" -o run --output-format csv -- python3 bench.py "$@"
  cp -r "$OUT/cal/cal_fetch" "$OUT/cal/cal_write" "$d/"
  python3 scripts/pmc_summary.py "$d" "$d/pmc.json" --batch "$batch" --kernel "$kern" --workload "$wl" --skip "$skip" > /dev/null || exit 1
  echo "[prof] $name done"
}
Q="--no-cpu --no-steady --no-extra"
for l in $LEGS; do
  case $l in
    tube) leg tube fk::tube_fast_kernel tube 65536 17978097664 8 20 0 -- $Q --warmup 8 --steps 20 ;;
    tube_f64) leg tube_f64 fk64::tube_fast_kernel tube_f64 65536 35956195328 1 5 0 -- $Q --dtype f64 --warmup 1 --steps 5 ;;
    tube_b4096) leg tube_b4096 fk::tube_fast_kernel tube 4096 1123631104 8 20 0 -- $Q --batch 4096 --warmup 8 --steps 20 ;;
    nominal_ddp_f32) leg nominal_ddp_f32 fk::ilqr_fast_kernel nominal_ddp_f32 4096 313425920 3 20 0 -- --workload nominal-ddp --dtype f32 --warmup 3 --steps 20 ;;
    nominal_ddp_f64) leg nominal_ddp_f64 fk64::ilqr_fast_kernel nominal_ddp_f64 4096 626851840 3 20 0 -- --workload nominal-ddp --dtype f64 --warmup 3 --steps 20 ;;
    receding_f32) leg receding_f32 fk::receding_fast_kernel receding_f32 65536 0 1 3 1 -- --workload receding --dtype f32 ;;
    receding_f64) leg receding_f64 fk64::receding_fast_kernel receding_f64 65536 0 1 3 1 -- --workload receding --dtype f64 ;;
    *) echo "unknown leg $l"; exit 2 ;;
  esac
done
echo "[prof] all done"
