# r03y: GPU suite with the 4-wide BVH per-lane walks (mesh scenes), mesh A/B wide vs binary
# (AMVPT_WIDE_BVH=0), M A/B packed-f32 row reduce (lib_pk) and attribution builds (lib_a8: plain LDS
# stores for the window adds; lib_a16: no cross-lane reduce steps)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03y_tests.log 2>&1 || exit 1
AB_CONFIG=mesh timeout -k 10 400 python -u tools/ab_value.py --kernels --env AMVPT_WIDE_BVH=1 --env AMVPT_WIDE_BVH=0 --env AMVPT_WIDE_BVH=1 --env AMVPT_WIDE_BVH=0 > gpurun_out/r03y_ab_mesh.log 2>&1 || exit 1
timeout -k 10 500 python -u tools/ab_value.py --kernels lib lib_pk lib_a8 lib_a16 lib lib_pk > gpurun_out/r03y_ab_M.log 2>&1 || exit 1
echo done
