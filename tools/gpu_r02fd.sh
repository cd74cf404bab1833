T=r02fd
S="bash tools/gpu_step.sh $T"
$S 900 tests -- python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
$S 400 ab -- python -u tools/ab_value.py --kernels --env AB_CHUNK=8388608 --env AB_CHUNK=16777216 --env AB_CHUNK=33554432 --env AB_CHUNK=4194304
cat gpurun_out/${T}_steps.log
