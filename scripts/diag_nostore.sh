set -u
cd "${GRAFT_REPO_ROOT:-.}"
L=$PWD/differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt
for v in prof nostp; do
  DTMPC_TUBE_LANES=1 DTMPC_LIBRARY=$L/libdtmpc_$v.so timeout -k 10 200 python scripts/phase_prof.py --batch 65536 > gpurun_out/ph_$v.log 2>&1 || exit $?
  echo "== $v"; grep -E "commit|linesearch|backward|kernel" gpurun_out/ph_$v.log
done
LANES=1 PLANES=none bash scripts/ab_phase.sh "base nost base nost"
