T=r02fj
S="bash tools/gpu_step.sh $T"
$S 600 tests -- python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
cat gpurun_out/${T}_steps.log
