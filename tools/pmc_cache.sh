# L1 (TCP) / L2 (TCC) hit picture per kernel, one rocprofv3 pass (usage: bash tools/pmc_cache.sh <tag> [bench args])
set -e
TAG=$1; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/${TAG}_cache -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0 "$@" > gpurun_out/${TAG}_cache.log 2>&1 || { echo "cache pass failed"; tail -5 gpurun_out/${TAG}_cache.log; exit 1; }
echo done
