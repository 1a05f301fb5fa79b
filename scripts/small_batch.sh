set -u
cd "${GRAFT_REPO_ROOT:-.}"
for B in 4096 16384 32768; do for L in 1 2; do
  DTMPC_TUBE_LANES=$L timeout -k 10 120 python bench.py --batch $B --steps 20 --warmup 3 --no-cpu > gpurun_out/small_${B}_$L.log 2>&1 || exit $?
  echo "B=$B lanes=$L $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/small_${B}_$L.log) $(grep -o '"value": [0-9.e+]*' gpurun_out/small_${B}_$L.log)"
done; done
