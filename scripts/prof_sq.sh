#!/usr/bin/env bash
# SQ counter passes (stall attribution) over a short bench run of one library (GPU box).
# usage: bash scripts/prof_sq.sh TAG [libdtmpc_<variant>.so]
set -u
TAG=${1:-sq}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
[ -n "${2:-}" ] && export DTMPC_LIBRARY=$PWD/differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt/$2
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
ARGS="--steps 2 --warmup 1 --no-cpu"
i=0
for P in "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVE_CYCLES" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU_TRANS_F32" \
         "SQ_IFETCH SQ_INSTS_BRANCH SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_BUSY_CYCLES"; do
  i=$((i+1))
  echo "[sq] pass $i: $P"
  timeout -s KILL 240 rocprofv3 --pmc $P -d "$OUT/p$i" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "[sq] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
