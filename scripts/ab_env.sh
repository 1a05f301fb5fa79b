#!/usr/bin/env bash
# Same-box A/B of an environment switch of the product library: bench.py alternately with and without it.
# usage: bash scripts/ab_env.sh "VAR=value" [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq ${2:-2}); do
  for v in base "$1"; do
    if [ "$v" = base ]; then e=(); else e=("$v"); fi
    env "${e[@]}" timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu > gpurun_out/abenv_$r.log 2>&1; rc=$?
    echo "[abenv] $v bench rc=$rc $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/abenv_$r.log)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
