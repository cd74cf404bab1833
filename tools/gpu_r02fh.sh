T=r02fh
S="bash tools/gpu_step.sh $T"
$S 600 tests -- python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
$S 400 ab -- python -u tools/ab_value.py --kernels --env AMVPT_VIS_LEAVES=1 --env AMVPT_VIS_LEAVES=0 --env AMVPT_VIS_LEAVES=1
cat gpurun_out/${T}_steps.log
