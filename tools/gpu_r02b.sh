set -u
T=${1:-r02b}
S="bash tools/gpu_step.sh $T"
$S 900 tests -- python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
$S 300 smoke -- python -u -c "import __graft_entry__ as g; g.smoke()"
$S 400 bench -- python -u bench.py --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$S 300 trace -- rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_trace -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --rmse-lanes 0
$S 180 pmc_fetch -- rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_fetch -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0
$S 180 pmc_write -- rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_write -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0
cat gpurun_out/${T}_steps.log
