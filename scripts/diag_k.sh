#!/usr/bin/env bash
# run one pytest selection (FILE, -k EXPR) on A/B variant libraries (build.py --variant NAME ...), REPEAT times each
# Usage: diag_k.sh FILE EXPR variant...   (env: REPEAT, default 1; OUT, default gpurun_out/diagk)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/diagk}
mkdir -p $O
F=$1
K=$2
shift 2
for v in "$@"; do
  for r in $(seq 1 ${REPEAT:-1}); do
    lib=$PWD/differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt/libdtmpc_$v.so
    [ "$v" = product ] && lib=$PWD/differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt/libdtmpc.so
    DTMPC_LIBRARY=$lib timeout -k 10 300 \
      python -u -m pytest $F -m gpu -q -s -rxX --timeout 240 --timeout-method thread -k "$K" > $O/${v}_$r.txt 2>&1
    rc=$?
    echo "$v run $r rc=$rc $(grep -c DIAG $O/${v}_$r.txt) diag lines; $(tail -1 $O/${v}_$r.txt)"
    [ $rc -le 1 ] || exit $rc
  done
done
