# r03za: GPU suite (shared row boxes in the row splat), A/B lib vs lib_ts (fused-suffix scenes on two chunk
# streams) on M, then the M bench line
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03za_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/ab_value.py --kernels lib lib_ts lib lib_ts > gpurun_out/r03za_ab_M.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/r03za_bench_M.json 2> gpurun_out/r03za_bench_M.err || exit 1
echo done
