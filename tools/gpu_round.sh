# GPU round: parity tests, smoke, the default bench line, a kernel-trace profile and the
# two PMC traffic passes (FETCH_SIZE and WRITE_SIZE in separate runs).
# usage (from the repo root, via gpurun):  bash tools/gpu_round.sh <tag> [tests|bench|prof|all]
set -e
TAG=${1:-r01}
WHAT=${2:-all}
mkdir -p gpurun_out
if [ "$WHAT" = all ] || [ "$WHAT" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
fi
if [ "$WHAT" = all ] || [ "$WHAT" = bench ]; then
  timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
fi
if [ "$WHAT" = all ] || [ "$WHAT" = prof ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_trace.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_fetch -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/${TAG}_fetch.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_write -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/${TAG}_write.log 2>&1
fi
echo done
