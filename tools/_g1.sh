set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02f_tests.log 2>&1
timeout -k 10 900 python tools/ab_value.py lib_w96 lib lib_h > gpurun_out/r02f_ab.log 2>&1
timeout -k 10 900 python tools/ab_value.py --kernels --env AMVPT_WIN_RS=16 >> gpurun_out/r02f_ab.log 2>&1
echo ok
