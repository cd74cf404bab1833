# r03w: GPU suite on the shifted-weight row splat (AMVPT_SPLAT_W5), then A/B lib (W5 on) vs lib_w0 on M, C3, mesh
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03w_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/ab_value.py --kernels lib lib_w0 lib lib_w0 > gpurun_out/r03w_ab_M.log 2>&1 || exit 1
AB_CONFIG=C3 timeout -k 10 400 python -u tools/ab_value.py --kernels lib lib_w0 > gpurun_out/r03w_ab_C3.log 2>&1 || exit 1
AB_CONFIG=mesh timeout -k 10 400 python -u tools/ab_value.py lib lib_w0 > gpurun_out/r03w_ab_mesh.log 2>&1 || exit 1
echo done
