# SQ instruction-mix / stall / LDS counters per kernel, one rocprofv3 pass per counter group
# (each group within the per-block limits of MI355X_MICROARCH.md "rocprofv3 PMC slots").
# usage: bash tools/pmc_sq.sh <tag> [bench args...]
set -e
TAG=$1; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH"
B="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"
C="SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64"
for P in A B C; do
  eval CS=\$$P
  timeout -s KILL 120 rocprofv3 --pmc $CS --output-format csv -d gpurun_out/${TAG}_sq$P -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0 "$@" > gpurun_out/${TAG}_sq$P.log 2>&1 || { echo "pass $P failed"; tail -5 gpurun_out/${TAG}_sq$P.log; exit 1; }
done
echo done
