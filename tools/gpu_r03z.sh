# r03z: GPU suite on packed row reduce + row kernels without the deterministic film path + literal default-filter coefficients, then
# A/B lib vs lib_pk (packed reduce only) on M and C3
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03z_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/ab_value.py --kernels lib lib_pk lib lib_pk > gpurun_out/r03z_ab_M.log 2>&1 || exit 1
AB_CONFIG=C3 timeout -k 10 400 python -u tools/ab_value.py --kernels lib lib_pk > gpurun_out/r03z_ab_C3.log 2>&1 || exit 1
echo done
