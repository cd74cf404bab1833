T=r02fk
S="bash tools/gpu_step.sh $T"
$S 400 ab -- python -u tools/ab_value.py --kernels --env AB_TRAV=0 --env AB_TRAV=2
cat gpurun_out/${T}_steps.log
