#!/usr/bin/env bash
# Same-box A/B of variant libraries (build.py --variant NAME --only UNIT --on-product) on chosen bench legs, the
# variants alternated REPS times; one line per run: leg, variant, rep, kernel_ms.  Every run under its own limit;
# the first failure ends the call.  usage: VARIANTS="product a b" LEGS="h b4096 f64 f64b8192 ddp rc rc64" REPS=3 bash scripts/ab_pair.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
L=differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt
Q="--no-cpu --no-steady --no-extra"
for rep in $(seq 1 "${REPS:-3}"); do for leg in ${LEGS:-h}; do for v in ${VARIANTS:-product}; do
  if [ "$v" = product ]; then lib=$PWD/$L/libdtmpc.so; else lib=$PWD/$L/libdtmpc_$v.so; fi
  case $leg in
    h) args="--steps 40 --warmup 8 $Q" ;;
    b4096) args="--batch 4096 --steps 40 --warmup 8 $Q" ;;
    b8192) args="--batch 8192 --steps 40 --warmup 8 $Q" ;;
    b16384) args="--batch 16384 --steps 40 --warmup 8 $Q" ;;
    b32768) args="--batch 32768 --steps 40 --warmup 8 $Q" ;;
    f64b32768) args="--dtype f64 --batch 32768 --steps 10 --warmup 3 $Q" ;;
    f64) args="--dtype f64 --steps 8 --warmup 3 $Q" ;;
    f64b8192) args="--dtype f64 --batch 8192 --steps 20 --warmup 5 $Q" ;;
    ddp) args="--workload nominal-ddp --dtype f32 --steps 20 --warmup 5" ;;
    rc) args="--workload receding --dtype f32" ;;
    rc64) args="--workload receding --dtype f64" ;;
    *) echo "unknown leg $leg"; exit 2 ;;
  esac
  DTMPC_LIBRARY=$lib timeout -k 10 300 python bench.py $args > "$OUT/${leg}_${v}_$rep.log" 2>&1 || exit $?
  echo "$leg $v $rep $(grep -o -E '"(kernel_ms|launch_ms)": [0-9.]*' "$OUT/${leg}_${v}_$rep.log" | head -n 1)" | tee -a "$OUT/ab.txt"
done; done; done
