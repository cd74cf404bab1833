T=r02fc
S="bash tools/gpu_step.sh $T"
$S 400 ab -- python -u tools/ab_value.py --kernels lib lib_w4 lib_w6 lib
cat gpurun_out/${T}_steps.log
