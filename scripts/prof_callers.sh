#!/usr/bin/env bash
# Kernel trace of the callers' benchmark (general IFT step, receding driver): per-kernel time split.
# usage: bash scripts/prof_callers.sh TAG
set -u
TAG=${1:-v1}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/callers_$TAG
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- python3 scripts/bench_callers.py > "$OUT/log.txt" 2>&1 || exit $?
echo "[prof] done"
