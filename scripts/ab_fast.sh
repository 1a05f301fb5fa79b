#!/usr/bin/env bash
# Fast-path check on the GPU box: tube-step parity tests (fast kernel, both lane counts), then a short
# bench of the fast kernel at 1 and 2 lanes per trajectory and of the generic kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
K=${1:-"tube_step or closed_loop or full_batch or dist"}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/t_fast.log 2>&1; rc=$?
echo "[ab] tests rc=$rc $(tail -n 1 gpurun_out/t_fast.log)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in "fast1 DTMPC_TUBE_LANES=1" "fast2 DTMPC_TUBE_LANES=2" "generic DTMPC_FAST=0"; do
  set -- $v
  env $2 timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu > gpurun_out/b_$1.log 2>&1; rc=$?
  echo "[ab] $1 bench rc=$rc $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/b_$1.log) $(grep -o '"flagged_trajectories": [0-9]*' gpurun_out/b_$1.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
