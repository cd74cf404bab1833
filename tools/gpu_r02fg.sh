T=r02fg
S="bash tools/gpu_step.sh $T"
$S 600 tests -- python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or config"
$S 400 ab -- python -u tools/ab_value.py --kernels lib lib_v4w4 lib_v4w5 lib_v3w5 lib
$S 300 t4 -- env AMVPT_LIB_DIR=$PWD/mitsuba3-amvpt_amd/lib_v4w5 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "config_m or mis_g8 or veach"
cat gpurun_out/${T}_steps.log
