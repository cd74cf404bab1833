T=r02fi
S="bash tools/gpu_step.sh $T"
$S 600 tests -- python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
$S 400 ab -- python -u tools/ab_value.py --kernels lib lib_rc0 lib
cat gpurun_out/${T}_steps.log
