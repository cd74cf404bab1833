T=r02fm
S="bash tools/gpu_step.sh $T"
$S 400 ab -- python -u tools/ab_value.py --kernels --env AMVPT_FUSED_BLOCKS=16 --env AMVPT_FUSED_BLOCKS=12 --env AMVPT_FUSED_BLOCKS=24 --env AMVPT_FUSED_BLOCKS=32 --env AMVPT_FUSED_BLOCKS=16
cat gpurun_out/${T}_steps.log
