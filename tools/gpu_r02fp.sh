T=r02fp
S="bash tools/gpu_step.sh $T"
$S 400 tf0 -- env AMVPT_LIB_DIR=$PWD/mitsuba3-amvpt_amd/lib_f0 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
$S 400 ab -- python -u tools/ab_value.py --kernels lib_f0 lib lib_f0 lib
cat gpurun_out/${T}_steps.log
