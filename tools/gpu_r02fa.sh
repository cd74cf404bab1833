T=r02fa
S="bash tools/gpu_step.sh $T"
$S 900 tests -- python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
$S 400 ab -- python -u tools/ab_value.py --kernels --env AMVPT_FUSE_SUFFIX=0 --env AMVPT_FUSE_SUFFIX=1 --env AMVPT_FUSED_BLOCKS=3 --env AMVPT_FUSED_BLOCKS=8
cat gpurun_out/${T}_steps.log
