#!/usr/bin/env bash
# One GPU session: parity suite, caller-path throughput, commit store attribution, forward-fma A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_iter.sh "" > gpurun_out/batch_iter.log 2>&1; echo "iter rc=$?"; grep -E "\[iter\]|\[ab\]" gpurun_out/batch_iter.log
timeout -k 10 300 python scripts/bench_callers.py > gpurun_out/callers.json 2> gpurun_out/callers.err; echo "callers rc=$?"; cat gpurun_out/callers.json
bash scripts/diag_nostore.sh
L=$PWD/differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt
DTMPC_LIBRARY=$L/libdtmpc_ffma.so timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "tube_step or full_batch or chunk or closed_loop" > gpurun_out/t_ffma.log 2>&1; echo "ffma tests rc=$? $(tail -n1 gpurun_out/t_ffma.log)"
LANES=1 PLANES=none bash scripts/ab_phase.sh "base ffma base ffma"
