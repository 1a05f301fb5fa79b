set -u
cd ${GRAFT_REPO_ROOT}
O=gpurun_out/r03_e; mkdir -p $O
L=$PWD/differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -k "gamma0 or chunked" > $O/pytest.log 2>&1
echo "pytest rc=$? $(tail -n 1 $O/pytest.log)"
ab() {  # name lib lanes batch
  DTMPC_LIBRARY=$2 DTMPC_TUBE_LANES=$3 timeout -k 10 120 python bench.py --batch $4 --steps 20 --warmup 3 --no-cpu > $O/ab_$1.log 2>&1 || exit $?
  echo "$1 $(grep -o '"kernel_ms": [0-9.]*' $O/ab_$1.log)" | tee -a $O/ab.txt
}
for r in 1 2; do
  ab main65k_$r $L/libdtmpc.so 1 65536
  ab nolds65k_$r $L/libdtmpc_nolds.so 1 65536
done
for r in 1 2; do
  ab main4k_$r $L/libdtmpc.so 4 4096
  ab nolds4k_$r $L/libdtmpc_nolds.so 4 4096
done
for cfg in "4 4096" "2 4096" "1 4096" "1 65536"; do
  set -- $cfg
  DTMPC_LIBRARY=$L/libdtmpc_prof.so DTMPC_TUBE_LANES=$1 timeout -k 10 120 python scripts/phase_prof.py --batch $2 > $O/phase_l$1_b$2.txt 2>&1 || exit $?
  echo "== lanes $1 batch $2"; cat $O/phase_l$1_b$2.txt
done
