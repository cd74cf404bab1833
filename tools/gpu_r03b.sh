# r03b: full GPU tests (captured output of passing tests in the log: -rA), bench M and C5, splat
# attribution (filter weights / plain LDS stores), kernel trace + PMC traffic + SQ VALU of bench M
# (summaries stamped with the source revision), all into gpurun_out/r03b_*.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 400 --timeout-method thread > gpurun_out/r03b_tests.log 2>&1
echo "tests rc=$?"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/r03b_bench_M.json 2> gpurun_out/r03b_bench_M.err || exit 1
timeout -k 10 300 python -u bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03b_bench_C5.json 2> gpurun_out/r03b_bench_C5.err || exit 1
bash tools/ab.sh r03b_attr lib lib_a4 lib_a8 > gpurun_out/r03b_attr.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03b_trace -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --rmse-lanes 0 > gpurun_out/r03b_trace.log 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r03b_fetch -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0 > gpurun_out/r03b_fetch.log 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r03b_write -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0 > gpurun_out/r03b_write.log 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH --output-format csv -d gpurun_out/r03b_sqA -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0 > gpurun_out/r03b_sqA.log 2>&1 || exit 1
python3 tools/pmc_traffic.py gpurun_out/r03b_fetch gpurun_out/r03b_write gpurun_out/r03b_traffic.json M > gpurun_out/r03b_traffic.log 2>&1
python3 tools/pmc_valu.py gpurun_out/r03b_sqA gpurun_out/r03b_valu.json M > gpurun_out/r03b_valu.log 2>&1
echo done
