set -u
cd ${GRAFT_REPO_ROOT}
O=gpurun_out/r03_d; mkdir -p $O
L=$PWD/differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt
DTMPC_LIBRARY=$L/libdtmpc_k4.so timeout -k 10 120 python -u scripts/diag_g0.py run $O/k4_g0.npz "G0=0,L=1" > $O/diag.txt 2>&1 || exit 1
DTMPC_LIBRARY=$L/libdtmpc_k4.so timeout -k 10 120 python -u scripts/diag_g0.py run $O/k4_g1.npz "G0=1,L=1" >> $O/diag.txt 2>&1 || exit 1
python scripts/diag_g0.py cmp $O/k4_g1.npz $O/k4_g0.npz | tee -a $O/diag.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_systems.py tests/test_gpu_parity.py -m gpu -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?"; grep -E "passed|failed" $O/pytest.log | tail -3; grep FAILED $O/pytest.log | head -20
for B in 4096 8192 16384 32768 65536; do
  for LN in 1 2 4; do
    [ "$B" -ge 32768 ] && [ "$LN" = 4 ] && continue
    DTMPC_TUBE_LANES=$LN timeout -k 10 120 python bench.py --batch $B --steps 10 --warmup 2 --no-cpu > "$O/b${B}_l$LN.log" 2>&1 || exit $?
    echo "B=$B lanes=$LN $(grep -o '"kernel_ms": [0-9.]*' "$O/b${B}_l$LN.log") $(grep -o '"value": [0-9.e+]*' "$O/b${B}_l$LN.log")" | tee -a "$O/sweep.txt"
  done
done
