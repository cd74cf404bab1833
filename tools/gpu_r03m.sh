# r03m: GPU tests (groups up to 256 views, small mesh-light scene), mesh BVH size, then A/B:
# M fused suffix at 6 vs 5 waves/SIMD; mesh wavefront vs fused BVH suffix
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r03m_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/scene_stats.py scenes/cbox_mesh.xml > gpurun_out/r03m_stats.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_value.py --kernels lib lib_f5 lib lib_f5 > gpurun_out/r03m_ab_M.log 2>&1 || exit 1
AB_CONFIG=mesh timeout -k 10 400 python -u tools/ab_value.py lib lib_fb lib lib_fb > gpurun_out/r03m_ab_mesh.log 2>&1 || exit 1
echo done
