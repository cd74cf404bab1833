T=r02fq
S="bash tools/gpu_step.sh $T"
$S 300 ab -- python -u tools/ab_value.py --kernels lib lib_s4 lib
cat gpurun_out/${T}_steps.log
bash tools/gpu_final.sh r02i
