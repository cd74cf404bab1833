# End-of-round measurement set on the final kernels, in two gpurun calls:
#   bash tools/gpu_final.sh <tag> a : parity suite + smoke, then config M: the bench line, a kernel-trace
#        profile of the same bench command, FETCH_SIZE and WRITE_SIZE passes, SQ passes A, B and C
#   bash tools/gpu_final.sh <tag> b : configs C3 and mesh (bench line, kernel trace, FETCH/WRITE, SQ A) and C5
# Each step has its own time limit; the first failure ends the script.
set -e
T=${1:-r04z}
PART=${2:-a}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
one() {   # config, bench steps
  c=$1
  if [ $c = M ]; then B="--steps 10 --warmup 2"; P=""; else B="--steps 3 --warmup 1 --no-cpu-baseline --config $c"; P="--config $c"; fi
  timeout -k 10 500 python -u bench.py $B > gpurun_out/${T}_bench_$c.json 2> gpurun_out/${T}_bench_$c.err
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_trace_$c -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --rmse-lanes 0 --one-stream $P > gpurun_out/${T}_trace_$c.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_fetch_$c -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0 $P > gpurun_out/${T}_fetch_$c.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_write_$c -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0 $P > gpurun_out/${T}_write_$c.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH --output-format csv -d gpurun_out/${T}_sqA_$c -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0 $P > gpurun_out/${T}_sqA_$c.log 2>&1
}
if [ $PART = a ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
  one M
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/${T}_sqB_M -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0 > gpurun_out/${T}_sqB_M.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 --output-format csv -d gpurun_out/${T}_sqC_M -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0 > gpurun_out/${T}_sqC_M.log 2>&1
else
  one C3
  one mesh
  timeout -k 10 300 python -u bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_bench_C5.json 2> gpurun_out/${T}_bench_C5.err
fi
echo final-done
