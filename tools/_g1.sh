set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r01y_tests.log 2>&1
timeout -k 10 600 python tools/ab_value.py lib_h lib_nt lib > gpurun_out/r01y_ab.log 2>&1
timeout -k 10 600 python tools/ab_value.py --kernels --env AMVPT_BRUTE=1 --env AMVPT_BRUTE=0 >> gpurun_out/r01y_ab.log 2>&1
echo ok
