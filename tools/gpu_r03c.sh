# r03c: GPU tests after the crop-window / branch-free walk changes, and bench M + C5.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 400 --timeout-method thread > gpurun_out/r03c_tests.log 2>&1
echo "tests rc=$?"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/r03c_bench_M.json 2> gpurun_out/r03c_bench_M.err || exit 1
timeout -k 10 300 python -u bench.py --config mesh --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03c_bench_mesh.json 2> gpurun_out/r03c_bench_mesh.err || exit 1
timeout -k 10 300 python -u bench.py --config C3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03c_bench_C3.json 2> gpurun_out/r03c_bench_C3.err || exit 1
echo done
