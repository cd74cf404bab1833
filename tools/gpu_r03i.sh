# r03i: GPU tests with two chunk streams, then A/B (two streams vs one) on M, C3, mesh
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r03i_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/ab_value.py lib lib_s1 lib lib_s1 > gpurun_out/r03i_ab_M.log 2>&1 || exit 1
AB_CONFIG=C3 timeout -k 10 400 python -u tools/ab_value.py lib lib_s1 > gpurun_out/r03i_ab_C3.log 2>&1 || exit 1
AB_CONFIG=mesh timeout -k 10 400 python -u tools/ab_value.py lib lib_s1 > gpurun_out/r03i_ab_mesh.log 2>&1 || exit 1
echo done
