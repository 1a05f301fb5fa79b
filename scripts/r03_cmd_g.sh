set -u
cd ${GRAFT_REPO_ROOT}
O=gpurun_out/r03_g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_systems.py -m gpu -v -s --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?"; grep -E "passed|failed" $O/pytest.log | tail -2; grep -E "^FAILED" $O/pytest.log | head -20; grep -E "\[decisions|\[free-running" $O/pytest.log | sed 's/^tests\S* //' | cut -c1-220 | head -60
timeout -k 10 300 python bench.py --no-cpu > $O/bench_default.log 2>&1 || exit $?
tail -1 $O/bench_default.log
