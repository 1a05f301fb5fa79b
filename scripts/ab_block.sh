#!/usr/bin/env bash
# Same-box A/B of the fused kernels' workgroup size at small batches: the product library (64-thread
# workgroups below the wave slots) vs libdtmpc_bs256.so (-D DTMPC_TUBE_SMALL_BLOCK=0, always 256).
# usage: bash scripts/ab_block.sh OUT.txt
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${1:-gpurun_out/ab_block.txt}
mkdir -p "$(dirname "$OUT")"
V=differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt/libdtmpc_bs256.so
for B in 4096 8192 16384 32768 65536; do
  for lib in product bs256; do
    if [ $lib = product ]; then unset DTMPC_LIBRARY; else export DTMPC_LIBRARY=$PWD/$V; fi
    r=$(timeout -k 10 120 python bench.py --batch $B --steps 10 --warmup 2 --no-cpu --no-steady --no-extra) || exit 1
    echo "B=$B lib=$lib $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("kernel_ms", round(d["kernel_ms"],4), "value", round(d["value"]))')" | tee -a "$OUT"
  done
done
for lib in product bs256; do
  if [ $lib = product ]; then unset DTMPC_LIBRARY; else export DTMPC_LIBRARY=$PWD/$V; fi
  r=$(timeout -k 10 120 python bench.py --workload nominal-ddp --steps 20 --warmup 3) || exit 1
  echo "nominal-ddp B=4096 lib=$lib $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("ms", round(d["ms_per_step"],4), "value", round(d["value"]))')" | tee -a "$OUT"
done
