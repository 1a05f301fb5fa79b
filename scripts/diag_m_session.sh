#!/usr/bin/env bash
# per-obstacle-count diagnostics (scripts/diag_m.py) and the f64 bench, product library vs an A/B variant
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=${1:-pin64}
O=gpurun_out/diagm
mkdir -p $O
VL=$PWD/differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt/libdtmpc_$V.so
for k in; do
  timeout -k 10 240 python bench.py --dtype f64 --steps 5 --warmup 8 --no-cpu --no-steady --no-extra > $O/bench_prod_$k.txt 2>&1 || exit $?
  DTMPC_LIBRARY=$VL timeout -k 10 240 python bench.py --dtype f64 --steps 5 --warmup 8 --no-cpu --no-steady --no-extra > $O/bench_${V}_$k.txt 2>&1 || exit $?
done
DIAG_TUBE=1 timeout -k 10 400 python scripts/diag_m.py > $O/d_prod.txt 2>&1 || exit $?
DIAG_TUBE=1 DTMPC_LIBRARY=$VL timeout -k 10 400 python scripts/diag_m.py > $O/d_$V.txt 2>&1
