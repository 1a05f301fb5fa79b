set -u
cd ${GRAFT_REPO_ROOT}
O=gpurun_out/r03_c; mkdir -p $O
L=$PWD/differentiable-tube-mpc_amd/diff_tube_mpc_strict_pt
for lib in main nolds lds13; do
  for c in "G0=1,L=1" "G0=0,L=1" "G0=2,L=1"; do
    f=$O/${lib}_$(echo $c | tr '=,' '__').npz
    if [ $lib = main ]; then so=$L/libdtmpc.so; else so=$L/libdtmpc_$lib.so; fi
    DTMPC_LIBRARY=$so timeout -k 10 120 python -u scripts/diag_g0.py run $f "$c" > $O/log_$lib.txt 2>&1 || { cat $O/log_$lib.txt; exit 1; }
  done
done
python scripts/diag_g0.py cmp $O/nolds_G0_0_L_1.npz $O/nolds_G0_1_L_1.npz $O/main_G0_0_L_1.npz $O/main_G0_1_L_1.npz $O/lds13_G0_0_L_1.npz $O/lds13_G0_1_L_1.npz > $O/cmp.txt
python scripts/diag_g0.py cmp $O/nolds_G0_2_L_1.npz $O/main_G0_2_L_1.npz $O/lds13_G0_2_L_1.npz >> $O/cmp.txt
cat $O/cmp.txt
for c in "G0=2,L=1" "G0=2,L=2" "G0=2,L=4"; do
  f=$O/nc_$(echo $c | tr '=,' '__').npz
  DTMPC_LIBRARY=$L/libdtmpc_nc.so timeout -k 10 120 python -u scripts/diag_g0.py run $f "$c" > $O/log_nc.txt 2>&1 || { cat $O/log_nc.txt; exit 1; }
done
python scripts/diag_g0.py cmp $O/nc_G0_2_L_1.npz $O/nc_G0_2_L_2.npz $O/nc_G0_2_L_4.npz | tee -a $O/cmp.txt
