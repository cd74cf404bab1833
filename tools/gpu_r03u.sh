# r03u: same-box A/B on M: current (tiles), current without tiles, the r03q build (before the
# deterministic mode)
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab_value.py --kernels lib lib_nt lib_q lib lib_nt lib_q > gpurun_out/r03u_ab_M.log 2>&1 || exit 1
echo done
