# r03e: GPU tests after the deferred per-view BSDF sample / whole-quilt splat instance / branchy
# brute test, then A/B: M (lib vs the r03d no-window build), C3 (deferred sample on / off).
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r03e_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/ab_value.py --kernels lib lib_nw lib lib_nw > gpurun_out/r03e_ab_M.log 2>&1 || exit 1
AB_CONFIG=C3 timeout -k 10 400 python -u tools/ab_value.py --kernels lib lib_ds0 lib lib_ds0 > gpurun_out/r03e_ab_C3.log 2>&1 || exit 1
echo done
