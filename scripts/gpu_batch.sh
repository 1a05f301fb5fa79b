#!/usr/bin/env bash
# One GPU session: parity suite, caller-path throughput, commit store attribution, variant A/B.
# Stops at the first GPU step that faults, aborts or times out (exit status > 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
chk() { local rc=$1; echo "[batch] $2 rc=$rc"; if [ "$rc" -gt 1 ]; then exit "$rc"; fi; }
bash scripts/gpu_iter.sh "" > gpurun_out/batch_iter.log 2>&1; rc=$?; grep -E "\[iter\]|\[ab\]" gpurun_out/batch_iter.log; chk $rc iter
timeout -k 10 300 python scripts/bench_callers.py > gpurun_out/callers.json 2> gpurun_out/callers.err; rc=$?; cat gpurun_out/callers.json; chk $rc callers
bash scripts/diag_nostore.sh; chk $? nostore
L=$PWD/differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt
for v in cmrc ffma; do
  DTMPC_LIBRARY=$L/libdtmpc_$v.so timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "tube_step or full_batch or chunk or closed_loop or fused" > gpurun_out/t_$v.log 2>&1; rc=$?
  tail -n1 gpurun_out/t_$v.log; chk $rc "tests $v"
done
LANES=1 PLANES=none bash scripts/ab_phase.sh "${AB:-base cmrc ffma base cmrc ffma}"; chk $? ab
