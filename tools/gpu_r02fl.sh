T=r02fl
S="bash tools/gpu_step.sh $T"
$S 400 ab -- python -u tools/ab_value.py --kernels lib lib_s4 lib_s6 lib_p6 lib
cat gpurun_out/${T}_steps.log
