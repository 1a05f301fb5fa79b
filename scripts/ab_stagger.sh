#!/usr/bin/env bash
# A/B of the workgroup start stagger (DTMPC_FAST_STAGGER sleep rounds) on the bench workload.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${1:-0 4 8 16 32 0}; do
  DTMPC_FAST_STAGGER=$v timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu > gpurun_out/b_st$v.log 2>&1 || exit $?
  echo "[st] stagger=$v $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/b_st$v.log)"
done
