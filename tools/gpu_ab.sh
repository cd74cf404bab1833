# GPU parity tests on lib/ + an A/B of config-M Msamples/s over library dirs (baseline first and last).
# usage: bash tools/gpu_ab.sh <tag> <libdir> [<libdir> ...]
set -u
T=$1; shift
S="bash tools/gpu_step.sh $T"
$S 600 tests -- python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
$S 600 ab -- python -u tools/ab_value.py --kernels "$@"
cat gpurun_out/${T}_steps.log
