# r03l: GPU tests with 256-bit view masks (groups up to 256 views) and the small mesh-light scene,
# then config M as a regression check
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r03l_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_value.py lib lib > gpurun_out/r03l_ab_M.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/scene_stats.py scenes/cbox_mesh.xml > gpurun_out/r03l_stats.txt 2>&1 || exit 1
echo done
