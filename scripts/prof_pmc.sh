#!/usr/bin/env bash
# rocprofv3 passes over a short bench run (GPU box).  Kernel trace + stats in one pass; each PMC group
# in its own pass (no trace domains combined with --pmc).  usage: bash scripts/prof_pmc.sh TAG [bench args]
set -u
TAG=${1:-r01}
shift || true
ARGS=${*:-"--steps 8 --warmup 2 --no-cpu"}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
run() {
  echo "[prof] $*"
  timeout -k 10 600 "$@" >> "$OUT/prof.log" 2>&1
  local rc=$?
  echo "[prof] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py $ARGS
run rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 bench.py $ARGS
run rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 bench.py $ARGS
run rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d "$OUT/sq1" -o run --output-format csv -- python3 bench.py $ARGS
run rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d "$OUT/sq2" -o run --output-format csv -- python3 bench.py $ARGS
run rocprofv3 --pmc FETCH_SIZE -d "$OUT/cal_fetch" -o run --output-format csv -- python3 scripts/pmc_calib.py
run rocprofv3 --pmc WRITE_SIZE -d "$OUT/cal_write" -o run --output-format csv -- python3 scripts/pmc_calib.py
run rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d "$OUT/tcc" -o run --output-format csv -- python3 bench.py $ARGS
echo "[prof] done"
