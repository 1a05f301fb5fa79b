#!/usr/bin/env bash
# Same-box A/B of f64 fused-kernel variants (libdtmpc_<v>.so built with --only dtmpc_fast64): the f64 tube
# step at the bench batch (one lane) and at 8,192 (every lane form).  usage: bash scripts/ab_f64.sh "v1 v2 ..."
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_f64
mkdir -p "$OUT"
D=differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt
for v in $1; do
  for BL in "65536 1" "8192 1" "8192 2" "8192 4"; do
    set -- $BL
    DTMPC_LIBRARY=$PWD/$D/libdtmpc_$v.so DTMPC_TUBE_LANES=$2 timeout -k 10 300 python bench.py --dtype f64 --batch $1 \
      --steps 5 --warmup 1 --no-cpu --no-steady --no-extra > "$OUT/${v}_b$1_l$2.log" 2>&1 || exit $?
    echo "$v B=$1 lanes=$2 $(grep -o '"kernel_ms": [0-9.]*' "$OUT/${v}_b$1_l$2.log")" | tee -a "$OUT/ab.txt"
  done
done
