T=r02ff
S="bash tools/gpu_step.sh $T"
$S 900 tests -- python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or config or unbiased"
$S 400 ab -- python -u tools/ab_value.py --kernels lib lib_p0 lib_p5 lib
cat gpurun_out/${T}_steps.log
