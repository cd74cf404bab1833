# r02v: parity tests, config-M A/B vs HEAD (lib_b), mesh bench with and without octant-ordered BVH copies
S="bash tools/gpu_step.sh r02v"
$S 600 tests -- python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
$S 300 ab -- python -u tools/ab_value.py --kernels lib_b lib
$S 300 mesh0 -- env AMVPT_OCT_BVH=0 python -u bench.py --config mesh --steps 2 --warmup 1 --no-cpu-baseline --rmse-lanes 0
$S 300 mesh1 -- python -u bench.py --config mesh --steps 2 --warmup 1 --no-cpu-baseline --rmse-lanes 0
cat gpurun_out/r02v_steps.log
