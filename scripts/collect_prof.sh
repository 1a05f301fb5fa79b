#!/usr/bin/env bash
# Copy one profile session's summaries (scripts/prof_r05.sh TAG, gpurun_out/prof5_TAG) into profiles/r05 under the
# names bench.py and DESIGN.md cite: kernel_trace_<leg>_TAG.json, kernel_stats_<leg>_TAG.csv, pmc_<leg>_TAG.json.
# usage: bash scripts/collect_prof.sh TAG
set -eu
TAG=$1
cd "$(dirname "$0")/.."
for d in gpurun_out/prof5_$TAG/*/; do
  leg=$(basename "$d")
  [ -f "$d/pmc.json" ] || continue
  cp "$d/trace_summary.json" "profiles/r05/kernel_trace_${leg}_$TAG.json"
  cp "$d/trace/run_kernel_stats.csv" "profiles/r05/kernel_stats_${leg}_$TAG.csv"
  cp "$d/pmc.json" "profiles/r05/pmc_${leg}_$TAG.json"
  echo "$leg"
done
