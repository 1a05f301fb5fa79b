#!/usr/bin/env bash
# GPU session (one gpurun call): smoke, the whole -m gpu suite with the parity prints (-s), then a
# short default bench line.  Every GPU step runs under its own time limit; a crash / timeout / abort ends
# the session (pytest assertion failures, exit 1, do not).  Logs: gpurun_out/session_<TAG>/.
# usage: bash scripts/gpu_session.sh TAG [steps: smoke tests bench] [pytest -k expression]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-s1}
STEPS=${2:-"smoke tests bench"}
KEXPR=${3:-}
OUT=gpurun_out/session_$TAG
mkdir -p "$OUT"
run() {  # name seconds cmd...
  local name=$1 secs=$2
  shift 2
  echo "[gpu] $name: $*" | tee -a "$OUT/session.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[gpu] $name rc=$rc" | tee -a "$OUT/session.log"
  tail -n 4 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "[gpu] stopping after $name (rc=$rc)" | tee -a "$OUT/session.log"
    exit $rc
  fi
  return 0
}
# a library variant by name (build.py --variant NAME): "product" is libdtmpc.so itself
lib() { if [ "$1" = product ]; then echo "$PWD/differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt/libdtmpc.so";
        else echo "$PWD/differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt/libdtmpc_$1.so"; fi; }
for s in $STEPS; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests)
      if [ -n "$KEXPR" ]; then
        run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf -s --timeout 300 --timeout-method thread -k "$KEXPR"
      else
        run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf -s --timeout 300 --timeout-method thread
      fi ;;
    bench) run bench 900 python bench.py --steps 10 --warmup 3 ;;
    b4096) run b4096 300 python bench.py --batch 4096 --steps 20 --warmup 8 --no-cpu --no-steady --no-extra ;;
    callers) run callers 600 python scripts/bench_callers.py --receding-only --f64 ;;
    f64lanes)  # the lane rule re-checked on the f64 fused kernel (DTMPC_TUBE_LANES forces the count)
      for b in 65536 16384; do for l in 1 2 4; do
        DTMPC_TUBE_LANES=$l run f64_b${b}_l$l 300 python bench.py --dtype f64 --batch $b --steps 5 --warmup 8 --no-cpu --no-steady --no-extra
      done; done ;;
    bench_quick) run bench_quick 600 python bench.py --steps 10 --warmup 3 --no-cpu --no-steady ;;
    probe) run stream_probe 300 python -u scripts/stream_probe.py ;;  # the headline's record stream
    reuse)  # VARIANTS: the stale-workspace check (scripts/diag_reuse.py, pre-filled workspace) per library, f64 two lanes
      for v in ${VARIANTS:-product}; do
        FILL=0xff DTMPC_LIBRARY=$(lib $v) run reuse_$v 180 python -u scripts/diag_reuse.py DT=f64,L=2,SEED=5 0 0 256 0
      done ;;
    ab)  # VARIANTS alternated twice: B = 4,096 tube step, the headline, config 2 (and the f64 legs with AB_F64=1)
      for rep in 1 2; do for v in ${VARIANTS:-product}; do
        DTMPC_LIBRARY=$(lib $v) run ab_b4096_${v}_$rep 300 python bench.py --batch 4096 --steps 20 --warmup 8 --no-cpu --no-steady --no-extra
        DTMPC_LIBRARY=$(lib $v) run ab_b65536_${v}_$rep 300 python bench.py --steps 20 --warmup 8 --no-cpu --no-steady --no-extra
        DTMPC_LIBRARY=$(lib $v) run ab_ddp_${v}_$rep 300 python bench.py --workload nominal-ddp --steps 20 --warmup 5
        if [ "${AB_F64:-0}" = 1 ]; then
          DTMPC_LIBRARY=$(lib $v) run ab_f64_${v}_$rep 300 python bench.py --dtype f64 --steps 5 --warmup 3 --no-cpu --no-steady --no-extra
          DTMPC_LIBRARY=$(lib $v) run ab_f64b8192_${v}_$rep 300 python bench.py --dtype f64 --batch 8192 --steps 10 --warmup 5 --no-cpu --no-steady --no-extra
        fi
      done; done ;;
    ab64)  # VARIANTS alternated twice: the f64 tube step at B = 65,536 (one lane) and 8,192 (four lanes)
      for rep in 1 2; do for v in ${VARIANTS:-product}; do
        DTMPC_LIBRARY=$(lib $v) run ab64_b65536_${v}_$rep 300 python bench.py --dtype f64 --steps 5 --warmup 3 --no-cpu --no-steady --no-extra
        DTMPC_LIBRARY=$(lib $v) run ab64_b8192_${v}_$rep 300 python bench.py --dtype f64 --batch 8192 --steps 10 --warmup 5 --no-cpu --no-steady --no-extra
      done; done ;;
    reusetest)  # VARIANTS: tests/test_gpu_reuse.py (every lane form, f32 and f64) per library
      for v in ${VARIANTS:-product}; do
        DTMPC_LIBRARY=$(lib $v) run reusetest_$v 300 python -u -m pytest tests/test_gpu_reuse.py -m gpu -q -rf --timeout 120 --timeout-method thread
      done ;;
    parity)  # VARIANTS: the tube-step / iLQR oracle gates and the bitwise lane / record / chunk checks per library
      for v in ${VARIANTS:-product}; do
        DTMPC_LIBRARY=$(lib $v) run parity_$v 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lanes.py -m gpu -q -rf -s --timeout 300 --timeout-method thread -k "${PARITY_K:-tube_step or ilqr_batched or lanes or records}"
      done ;;
    *) echo "unknown step $s" ;;
  esac
done
grep -h "^\[f32 vs f64\|^\[tie-aware\|^\[decisions" "$OUT/pytest_gpu.log" > "$OUT/parity_lines.txt" 2>/dev/null
exit 0
