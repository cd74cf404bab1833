# r03v: restored tree: GPU suite + smoke + M bench line; mesh parity on the coherent-uniform build
# (lib_cu: AMVPT_COH_UNI=1) and the mesh A/B lib vs lib_cu
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03v_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03v_smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/r03v_bench_M.json 2> gpurun_out/r03v_bench_M.err || exit 1
AMVPT_LIB_DIR=$PWD/mitsuba3-amvpt_amd/lib_cu timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "mesh or bvh or uniform or meshes" --timeout 300 --timeout-method thread > gpurun_out/r03v_tests_cu.log 2>&1 || exit 1
AB_CONFIG=mesh timeout -k 10 400 python -u tools/ab_value.py --kernels lib lib_cu lib lib_cu > gpurun_out/r03v_ab_mesh.log 2>&1 || exit 1
echo done
