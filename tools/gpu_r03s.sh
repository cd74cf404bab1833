# r03s: GPU suite (deterministic film), tiled-slot parity (lib_t), then A/B on M: current / block
# windows (lib_w0) / tiled slots + block windows (lib_t) / tiled slots + wave windows (lib_tw)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r03s_tests.log 2>&1 || exit 1
AMVPT_LIB_DIR=$PWD/mitsuba3-amvpt_amd/lib_t timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "amvpt_mis or full_resolution or many_chunks or deterministic or sharded or adaptive" > gpurun_out/r03s_tests_t.log 2>&1 || exit 1
timeout -k 10 500 python -u tools/ab_value.py --kernels lib lib_w0 lib_t lib_tw lib lib_t > gpurun_out/r03s_ab_M.log 2>&1 || exit 1
echo done
