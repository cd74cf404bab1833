# Vector-memory pipeline counters (TA / TD / TCP) per kernel, two rocprofv3 passes within the per-block slot limits
# (MI355X_MICROARCH.md "rocprofv3 PMC slots": 2 TA, 2 TD, 4 TCP, 2 GRBM per pass).
# usage: bash tools/pmc_mem.sh <tag> [bench args...]
set -e
TAG=$1; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCP_LATENCY GRBM_GUI_ACTIVE GRBM_COUNT"
B="TD_TD_BUSY TD_TC_STALL TCP_READ_TAGCONFLICT_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES TCP_UTCL1_TRANSLATION_MISS TCP_TCC_READ_REQ_LATENCY GRBM_GUI_ACTIVE"
for P in A B; do
  eval CS=\$$P
  timeout -s KILL 120 rocprofv3 --pmc $CS --output-format csv -d gpurun_out/${TAG}_mem$P -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0 "$@" > gpurun_out/${TAG}_mem$P.log 2>&1 || { echo "pass $P failed"; tail -5 gpurun_out/${TAG}_mem$P.log; exit 1; }
done
echo done
