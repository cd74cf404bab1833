set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r06z_bench_M.json 2> gpurun_out/r06z_bench_M.err
for c in C3 mesh C5; do
  timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r06z_bench_$c.json 2> gpurun_out/r06z_bench_$c.err
done
echo done
