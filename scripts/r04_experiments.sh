#!/usr/bin/env bash
# Round-4 GPU experiments (one gpurun call; libraries from scripts/r04_variants.sh).  Each GPU step under its
# own time limit; a crash / timeout ends the session.  Results: gpurun_out/r04_exp_<TAG>/.
#  1. root cause, LDS general records: diag_g0 (B = 700 f32, 2 closed-loop steps) on lds0 / lds1 / lds0c / lds1c
#  2. root cause, f64 inline far sincos: diag_g0 DT=f64 on far1 / far0 / far1c / far0c and the generic f64
#     kernel, + test_tube_step_fast64_vs_generic[1] on far0 / far0c
#  3. small batches: B = 4,096 four-lane tube step, prefetch lead 2 (the product library) / 3 / 4
#  4. PMC at B = 4,096 (SQ issue / wait split)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-e1}
STEPS=${2:-"lds far lead pmc"}
OUT=gpurun_out/r04_exp_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
L=variants
run() {  # name seconds cmd...
  local name=$1 secs=$2
  shift 2
  echo "[exp] $name: $*" | tee -a "$OUT/session.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[exp] $name rc=$rc" | tee -a "$OUT/session.log"
  tail -n 3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[exp] stop after $name" | tee -a "$OUT/session.log"; exit $rc; fi
}
for st in $STEPS; do
case $st in
lds)
for v in lds0 lds1 lds0c lds1c; do
  run diag_$v 180 env DTMPC_LIBRARY=$PWD/$L/libdtmpc_$v.so python scripts/diag_g0.py run "$OUT/$v.npz" "G0=0,L=1"
done
run cmp_lds 60 python scripts/diag_g0.py cmp "$OUT/lds0.npz" "$OUT/lds1.npz"
run cmp_ldsc 60 python scripts/diag_g0.py cmp "$OUT/lds0c.npz" "$OUT/lds1c.npz"
;;
far)
for v in far1 far0 far1c far0c; do
  run diag_$v 240 env DTMPC_LIBRARY=$PWD/$L/libdtmpc_$v.so python scripts/diag_g0.py run "$OUT/$v.npz" "DT=f64,L=1"
done
run diag_gen64 240 env DTMPC_LIBRARY=$PWD/$L/libdtmpc_far1.so python scripts/diag_g0.py run "$OUT/gen64.npz" "DT=f64,L=1,F64=0"
run cmp_far 60 python scripts/diag_g0.py cmp "$OUT/far1.npz" "$OUT/far0.npz" "$OUT/gen64.npz"
run cmp_farc 60 python scripts/diag_g0.py cmp "$OUT/far1c.npz" "$OUT/far0c.npz"
run cmp_far_gen 60 python scripts/diag_g0.py cmp "$OUT/gen64.npz" "$OUT/far1.npz" "$OUT/far0.npz" "$OUT/far1c.npz" "$OUT/far0c.npz"
for v in far0 far0c; do
  run t64_$v 300 env DTMPC_LIBRARY=$PWD/$L/libdtmpc_$v.so python -u -m pytest tests/test_gpu_parity.py -m gpu -q -s --timeout 240 -k "fast64_vs_generic and 1"
done
;;
lead)
run b4096_lead2 300 env DTMPC_TUBE_LANES=4 python bench.py --batch 4096 --steps 20 --warmup 5 --no-cpu --no-steady --no-extra
for v in lead3 lead4; do
  run b4096_$v 300 env DTMPC_LIBRARY=$PWD/$L/libdtmpc_$v.so DTMPC_TUBE_LANES=4 python bench.py --batch 4096 --steps 20 --warmup 5 --no-cpu --no-steady --no-extra
done
;;
recdiag)
run diag_receding 300 python scripts/diag_receding.py 1024
;;
pmc)
run pmc4096 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU -d "$OUT/pmc4096" -o run --output-format csv -- python3 bench.py --batch 4096 --steps 3 --warmup 1 --no-cpu --no-steady --no-extra
;;
esac
done
echo "[exp] done" | tee -a "$OUT/session.log"
