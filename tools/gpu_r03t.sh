# r03t: GPU suite with tiled splat slots on by default (and the deterministic path outside the row
# kernels), then A/B on M (tiles on / off) and the C3 / C5 bench lines
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r03t_tests.log 2>&1 || exit 1
timeout -k 10 500 python -u tools/ab_value.py --kernels lib lib_nt lib lib_nt > gpurun_out/r03t_ab_M.log 2>&1 || exit 1
AB_CONFIG=C3 timeout -k 10 500 python -u tools/ab_value.py --kernels lib lib_nt > gpurun_out/r03t_ab_C3.log 2>&1 || exit 1
echo done
