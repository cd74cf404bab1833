T=r02fe
S="bash tools/gpu_step.sh $T"
$S 900 tests -- python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
$S 600 bench -- python -u bench.py
$S 300 c3 -- python -u bench.py --config C3 --steps 2 --warmup 1 --no-cpu-baseline --rmse-lanes 0
$S 300 c5 -- python -u bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline --rmse-lanes 0

bash tools/gpu_step.sh r02fe 600 sq -- bash tools/pmc_sq.sh r02fe
cat gpurun_out/r02fe_steps.log
