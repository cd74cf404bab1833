# r03d: veach parity with the hoisted pdf row, then A/B: M over r02 / current / branchy brute test /
# no film window; C3 over pdf row on / off.
mkdir -p gpurun_out
true
timeout -k 10 400 python -u tools/ab_value.py --kernels lib lib_bt lib_nw lib lib_bt lib_nw > gpurun_out/r03d_ab_M.log 2>&1 || exit 1
AB_CONFIG=C3 timeout -k 10 400 python -u tools/ab_value.py --kernels lib lib_pr0 lib lib_pr0 > gpurun_out/r03d_ab_C3.log 2>&1 || exit 1
echo done
