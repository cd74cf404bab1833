# r03q: GPU tests (render_ex now honours set_chunk_lanes / set_traversal; two-stream parity), then bench
# lines for M (CPU baseline), C3, mesh, C5
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r03q_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/r03q_bench_M.json 2> gpurun_out/r03q_bench_M.err || exit 1
timeout -k 10 300 python -u bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03q_bench_C3.json 2> gpurun_out/r03q_bench_C3.err || exit 1
timeout -k 10 300 python -u bench.py --config mesh --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03q_bench_mesh.json 2> gpurun_out/r03q_bench_mesh.err || exit 1
timeout -k 10 300 python -u bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03q_bench_C5.json 2> gpurun_out/r03q_bench_C5.err || exit 1
echo done
