#!/usr/bin/env bash
# Copy one profile session's summaries (scripts/prof_session.sh TAG, gpurun_out/prof_ROUND_TAG) into profiles/ROUND
# under the names bench.py and DESIGN.md cite: kernel_trace_<leg>_TAG.json, kernel_stats_<leg>_TAG.csv,
# pmc_<leg>_TAG.json.  usage: [ROUND=r06] bash scripts/collect_prof.sh TAG
set -eu
TAG=$1
cd "$(dirname "$0")/.."
R=${ROUND:-r06}
mkdir -p "profiles/$R"
for d in gpurun_out/prof_${R}_$TAG/*/; do
  leg=$(basename "$d")
  [ -f "$d/pmc.json" ] || continue
  cp "$d/trace_summary.json" "profiles/$R/kernel_trace_${leg}_$TAG.json"
  cp "$d/trace/run_kernel_stats.csv" "profiles/$R/kernel_stats_${leg}_$TAG.csv"
  cp "$d/pmc.json" "profiles/$R/pmc_${leg}_$TAG.json"
  echo "$leg"
done
