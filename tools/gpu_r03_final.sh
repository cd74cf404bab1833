# End-of-round-3 measurement set on the final kernels (one gpurun call):
#   parity suite + smoke, then per config (M, C3, mesh): the bench line, a kernel-trace profile of the
#   same bench command, FETCH_SIZE and WRITE_SIZE passes, SQ pass A (VALU / SALU / LDS counts); M also
#   SQ passes B and C.  Each step has its own time limit; the first failure ends the script.
# usage: bash tools/gpu_r03_final.sh <tag>
set -e
T=${1:-r03z}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA --timeout 400 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in M C3 mesh; do
  if [ $c = M ]; then B="--steps 10 --warmup 2"; else B="--steps 3 --warmup 1 --no-cpu-baseline --config $c"; fi
  if [ $c = M ]; then P=""; else P="--config $c"; fi
  timeout -k 10 500 python -u bench.py $B > gpurun_out/${T}_bench_$c.json 2> gpurun_out/${T}_bench_$c.err
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_trace_$c -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --rmse-lanes 0 $P > gpurun_out/${T}_trace_$c.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_fetch_$c -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0 $P > gpurun_out/${T}_fetch_$c.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_write_$c -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0 $P > gpurun_out/${T}_write_$c.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH --output-format csv -d gpurun_out/${T}_sqA_$c -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0 $P > gpurun_out/${T}_sqA_$c.log 2>&1
done
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/${T}_sqB_M -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0 > gpurun_out/${T}_sqB_M.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 --output-format csv -d gpurun_out/${T}_sqC_M -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0 > gpurun_out/${T}_sqC_M.log 2>&1
timeout -k 10 300 python -u bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_bench_C5.json 2> gpurun_out/${T}_bench_C5.err
echo final-done
