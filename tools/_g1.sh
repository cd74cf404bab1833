set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02b_tests.log 2>&1
timeout -k 10 600 python tools/ab_value.py lib_1s lib > gpurun_out/r02b_ab.log 2>&1
timeout -k 10 600 python tools/ab_value.py --kernels --env AB_CHUNK=8388608 --env AB_CHUNK=4194304 --env AB_CHUNK=16777216 >> gpurun_out/r02b_ab.log 2>&1
echo ok
