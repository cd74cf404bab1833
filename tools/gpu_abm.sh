# parity tests, config-M A/B of library dirs, and the mesh bench on lib/
# usage: bash tools/gpu_abm.sh <tag> <libdir> [<libdir> ...]
T=$1; shift
S="bash tools/gpu_step.sh $T"
$S 600 tests -- python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
$S 300 ab -- python -u tools/ab_value.py --kernels "$@"
$S 300 mesh -- python -u bench.py --config mesh --steps 2 --warmup 1 --no-cpu-baseline --rmse-lanes 0
cat gpurun_out/${T}_steps.log
