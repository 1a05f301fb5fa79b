set -u
cd ${GRAFT_REPO_ROOT}
O=gpurun_out/r03_f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?"; grep -E "passed|failed" $O/pytest.log | tail -2; grep -E "FAILED|^\[decisions" $O/pytest.log | head -60
for B in 4096 8192 16384 32768; do
  for LN in 1 2 4; do
    [ "$B" -ge 32768 ] && [ "$LN" = 4 ] && continue
    DTMPC_TUBE_LANES=$LN timeout -k 10 120 python bench.py --batch $B --steps 10 --warmup 2 --no-cpu > "$O/b${B}_l$LN.log" 2>&1 || exit $?
    echo "B=$B lanes=$LN $(grep -o '"kernel_ms": [0-9.]*' "$O/b${B}_l$LN.log") $(grep -o '"value": [0-9.e+]*' "$O/b${B}_l$LN.log")" | tee -a "$O/sweep.txt"
  done
done
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || exit $?
tail -1 $O/bench_default.log
