# One call: GPU parity suite + smoke, the round's A/B set, then the final measurement set on the default build
# (bench lines, kernel-trace profiles of the same command, FETCH/WRITE and SQ passes for M, C3 and mesh; C5).
set -u
T=${1:-r04z}
S="bash tools/gpu_step.sh $T"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$S 900 tests -- python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread
$S 300 smoke -- python -u -c "import __graft_entry__ as g; g.smoke()"
# the A/B set of the call (AB=0 skips it): variant library dirs next to lib/, see profiles/<tag>_ab_*.log
if [ "${AB:-1}" = 1 ]; then
  AB_CONFIG=mesh $S 300 abmesh -- python -u tools/ab_value.py --kernels lib_r1 lib lib_v4 lib_r1 lib lib_v4
  AB_CONFIG=C3 $S 300 abC3 -- python -u tools/ab_value.py --kernels lib_d0 lib_u lib_r1 lib_v4 lib_d0 lib_u lib_r1 lib_v4
  $S 300 abM -- python -u tools/ab_value.py --kernels lib_r1 lib_v4 lib lib_r1 lib_v4 lib
fi
one() {   # config
  c=$1
  if [ $c = M ]; then B="--steps 10 --warmup 2"; P=""; else B="--steps 3 --warmup 1 --no-cpu-baseline --config $c"; P="--config $c"; fi
  $S 500 bench_$c -- python -u bench.py $B
  cp gpurun_out/${T}_bench_$c.log gpurun_out/${T}_bench_$c.json 2>/dev/null
  $S 300 trace_$c -- rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_trace_$c -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --rmse-lanes 0 --one-stream $P
  $S 300 fetch_$c -- rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_fetch_$c -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0 $P
  $S 300 write_$c -- rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_write_$c -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0 $P
  $S 200 sqA_$c -- rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH --output-format csv -d gpurun_out/${T}_sqA_$c -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0 $P
}
one M
one C3
one mesh
$S 300 bench_C5 -- python -u bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline
cat gpurun_out/${T}_steps.log
echo all-done
