#!/usr/bin/env bash
# Batch x lane-form sweep of the product library (bench.py headline leg only): kernel_ms (HIP events) and the
# DDP+IFT iters/s value for each (dtype, B, lanes); "auto" = the library's default lane rule (dtmpc_tube_lanes_dtype).
# usage: bash scripts/sweep_lanes.sh [out]   (on the GPU box)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/sweep_lanes.txt}
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
run() {  # dtype B lanes
  local env=()
  [ "$3" = auto ] || env=(DTMPC_TUBE_LANES=$3)
  env "${env[@]}" timeout -k 10 200 python bench.py --dtype "$1" --batch "$2" --steps 10 --warmup 3 --no-cpu --no-steady \
    --no-extra > gpurun_out/sweep.log 2>&1 || return $?
  echo "$1 B=$2 lanes=$3 $(tail -n 1 gpurun_out/sweep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("kernel_ms=%.4f value=%.4g" % (d["kernel_ms"], d["value"]))')" | tee -a "$OUT"
}
for B in 4096 8192 16384 32768 65536; do
  for L in auto 1 2 4; do run f32 $B $L || exit $?; done
done
for B in 8192 16384 65536; do
  for L in auto 1 4; do run f64 $B $L || exit $?; done
done
