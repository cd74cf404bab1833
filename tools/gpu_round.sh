set -e
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01b_trace -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r01b_trace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r01b_fetch -o pmc -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r01b_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r01b_write -o pmc -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r01b_write.log 2>&1
