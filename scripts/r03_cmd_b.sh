set -u
cd ${GRAFT_REPO_ROOT}
mkdir -p gpurun_out/r03_b
timeout -k 10 120 python -u scripts/diag_g0.py "G0=1,L=1" "G0=0,L=1" "G0=1,L=2" "G0=1,L=4" > gpurun_out/r03_b/diag_main.txt 2>&1 || exit $?
cat gpurun_out/r03_b/diag_main.txt | tail -8
DTMPC_LIBRARY=$PWD/differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt/libdtmpc_nolds.so timeout -k 10 120 python -u scripts/diag_g0.py "G0=1,L=1" "G0=0,L=1" "G0=1,L=2" "G0=1,L=4" > gpurun_out/r03_b/diag_nolds.txt 2>&1 || exit $?
cat gpurun_out/r03_b/diag_nolds.txt | tail -8
