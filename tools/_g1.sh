set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02c_tests.log 2>&1
timeout -k 10 600 python tools/ab_value.py lib_h lib_lo lib > gpurun_out/r02c_ab.log 2>&1
timeout -k 10 600 python tools/ab_value.py --kernels --env AB_CHUNK=8388608 >> gpurun_out/r02c_ab.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r02c_write -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r02c_write.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r02c_fetch -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r02c_fetch.log 2>&1
echo ok
