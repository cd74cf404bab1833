# r03r: deterministic film mode + the rest of the GPU suite
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r03r_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_value.py lib > gpurun_out/r03r_ab_M.log 2>&1 || exit 1
echo done
