# r03h: veach parity with register-resident pair operands, then A/B on C3 (PAIR_REGS on / off)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "veach" -x -q --timeout 300 --timeout-method thread > gpurun_out/r03h_tests.log 2>&1 || exit 1
AB_CONFIG=C3 timeout -k 10 400 python -u tools/ab_value.py --kernels lib lib_pr lib > gpurun_out/r03h_ab_C3.log 2>&1 || exit 1
echo done
