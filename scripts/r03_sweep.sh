#!/usr/bin/env bash
# Batch x lane-form sweep of the final round-3 library: f32 tube step at B = 4,096 ... 65,536 (the default lane
# form and each forced one), f64 at 8,192 and 65,536, and the per-GPU shard of BASELINE config 5 at 2 / 4 / 8
# GPUs (strong scaling: 32,768 / 16,384 / 8,192 trajectories).  kernel_ms from bench.py (HIP events).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sweep_v2
mkdir -p "$OUT"
one() {  # dtype B lanes(or "") tag
  local f=$OUT/$1_b$2_l${3:-auto}.log
  DTMPC_TUBE_LANES=$3 timeout -k 10 300 python bench.py --dtype $1 --batch $2 --steps 10 --warmup 2 --no-cpu \
    --no-steady --no-extra > "$f" 2>&1 || exit $?
  python3 - "$f" "$1" "$2" "${3:-auto}" <<'PY' | tee -a "$OUT/sweep.txt"
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]} B={sys.argv[3]} lanes={sys.argv[4]} kernel_ms={d['kernel_ms']:.4f} ms_per_step={d['ms_per_step']:.4f} value={d['value']:.4g}")
PY
}
for B in 4096 8192 16384 32768 65536; do
  one f32 $B ""
  for L in 1 2 4; do
    [ "$B" -ge 32768 ] && [ "$L" = 4 ] && continue
    one f32 $B $L
  done
done
for L in 1 2 4; do one f64 8192 $L; done
for L in 1 2; do one f64 65536 $L; done
