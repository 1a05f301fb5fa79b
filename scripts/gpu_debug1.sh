#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/dump_gpu.py > gpurun_out/dump.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r01 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/prof.log 2>&1
echo "prof rc=$?"
