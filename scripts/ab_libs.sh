#!/usr/bin/env bash
# Same-box A/B of experiment libraries (differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt/libdtmpc_<name>.so,
# built by build.py --variant NAME --on-product): the bitwise check of the variants' closed loop against the first
# (scripts/diag_g0.py, f32, one lane, two closed-loop steps of B = 700), then the headline bench alternated
# A B A B so that clock drift falls on both.  Each GPU step under its own time limit; a crash ends the session.
# usage: bash scripts/ab_libs.sh TAG NAME_A NAME_B [NAME_C ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1
shift
OUT=gpurun_out/ab_$TAG
mkdir -p "$OUT"
L=differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt
run() {  # name seconds cmd...
  local name=$1 secs=$2
  shift 2
  echo "[ab] $name: $*" | tee -a "$OUT/session.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[ab] $name rc=$rc" | tee -a "$OUT/session.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[ab] stop after $name" | tee -a "$OUT/session.log"; exit $rc; fi
}
# env: DIAG=0 skips the bitwise check (DIAG_CFG: its configuration, e.g. DT=f64,L=1); BENCH_ARGS replaces the headline bench arguments (e.g. the f64 leg);
# the name "product" is the product library libdtmpc.so
lib() { if [ "$1" = product ]; then echo "$PWD/$L/libdtmpc.so"; else echo "$PWD/$L/libdtmpc_$1.so"; fi; }
BARGS=${BENCH_ARGS:---steps 20 --warmup 8 --no-cpu --no-steady --no-extra}
if [ "${DIAG:-1}" = 1 ]; then
  for v in "$@"; do
    run diag_$v 180 env DTMPC_LIBRARY=$(lib $v) python scripts/diag_g0.py run "$OUT/$v.npz" "${DIAG_CFG:-L=1}"
  done
  first=$1
  for v in "$@"; do
    [ "$v" = "$first" ] || run cmp_$v 60 python scripts/diag_g0.py cmp "$OUT/$first.npz" "$OUT/$v.npz"
  done
fi
for rep in 1 2; do
  for v in "$@"; do
    run bench_${v}_$rep 300 env DTMPC_LIBRARY=$(lib $v) python bench.py $BARGS
  done
done
for f in "$OUT"/bench_*.log; do echo "$(basename "$f") $(tail -n 1 "$f" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["kernel_ms"],4), round(d["ms_per_step"],4))')"; done | tee "$OUT/summary.txt"
echo "[ab] done"
