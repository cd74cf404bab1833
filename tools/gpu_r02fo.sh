T=r02fo
S="bash tools/gpu_step.sh $T"
$S 400 ab -- python -u tools/ab_value.py --kernels lib lib_f0 lib_f2 lib lib_f2
$S 300 tf2 -- env AMVPT_LIB_DIR=$PWD/mitsuba3-amvpt_amd/lib_f2 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread
cat gpurun_out/${T}_steps.log
