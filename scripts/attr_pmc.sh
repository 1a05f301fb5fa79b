#!/usr/bin/env bash
# Per-phase attribution (GPU box): one SQ pass per library variant (a phase run twice, build.py -D DTMPC_DIAG_*).
# usage: bash scripts/attr_pmc.sh "dbase dBW2 dLS2 dCM2"
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
L=$PWD/differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt
for v in $1; do
  DTMPC_LIBRARY=$L/libdtmpc_$v.so timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY -d gpurun_out/attr/$v -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/attr_$v.log 2>&1
  rc=$?; echo "[attr] $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
