# r03a: GPU tests of the ABI-8 changes (view-group lane sets, film windows, per-call options), the bench
# lines of M and C5, a splat attribution A/B (variant builds without the flush's film atomics /
# without the window's LDS adds -- wrong images, timing only), and Z-map dumps for the edge-mask gate.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03a_tests.log 2>&1
echo "tests rc=$?"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03a_smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/r03a_bench_M.json 2> gpurun_out/r03a_bench_M.err || exit 1
timeout -k 10 300 python -u bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03a_bench_C5.json 2> gpurun_out/r03a_bench_C5.err || exit 1
bash tools/ab.sh r03a_attr lib lib_a1 lib_a2 > gpurun_out/r03a_attr.log 2>&1 || exit 1
for c in "cbox_grid.xml g8 res=48 gx=4 gy=2 reuse=8" "cbox_grid.xml g8box res=48 gx=4 gy=2 reuse=8 rfilter=box" "cbox_grid.xml g4 res=48" "veach_grid.xml vg8 res=48 gx=4 gy=2 reuse=8"; do
  timeout -k 10 300 python -u tools/zmap.py $c >> gpurun_out/r03a_zmap.log 2>&1 || exit 1
done
echo done
