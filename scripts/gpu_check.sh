#!/usr/bin/env bash
# Guarded GPU session: each step has its own time limit; a crash / timeout / abort ends the session
# (pytest assertion failures, exit 1, do not).  Logs go to gpurun_out/.
# usage: bash scripts/gpu_check.sh "smoke tests bench" [extra pytest args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS="${1:-smoke tests bench}"
PYARGS="${2:-}"

run() {  # name seconds cmd...
  local name=$1 secs=$2
  shift 2
  echo "[gpu_check] $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[gpu_check] $name rc=$rc" | tee -a gpurun_out/session.log
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "[gpu_check] stopping after $name (rc=$rc)" | tee -a gpurun_out/session.log
    exit $rc
  fi
  return 0
}

for s in $STEPS; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 1200 python -m pytest tests -m gpu -q -rf $PYARGS ;;
    bench) run bench 900 python bench.py --steps 10 --warmup 2 ;;
    bench_quick) run bench_quick 600 python bench.py --steps 5 --warmup 1 --no-cpu ;;
    *) echo "unknown step $s" ;;
  esac
done
exit 0
