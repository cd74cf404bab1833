T=r02fn
S="bash tools/gpu_step.sh $T"
$S 600 tests -- python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
$S 400 ab -- python -u tools/ab_value.py --kernels lib lib_k0 lib lib_k0
$S 300 bench -- python -u bench.py --steps 3 --warmup 1
cat gpurun_out/${T}_steps.log
