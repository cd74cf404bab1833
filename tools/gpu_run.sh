# One gpurun call of round-5 work: bash tools/gpu_run.sh <tag> <steps...>
# steps: tests | smoke | bench:<config> | trace:<config> | fetch:<config> | write:<config> | sqA:<config>
# Each step runs under its own time limit (tools/gpu_step.sh); a crash / timeout ends the call.
set -e
T=$1; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
S="bash tools/gpu_step.sh $T"
for st in "$@"; do
  kind=${st%%:*}; c=${st#*:}
  if [ "$c" = M ] || [ "$c" = "$kind" ]; then P=""; else P="--config $c"; fi
  case $kind in
    tests) $S 900 tests -- python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread ;;
    testslib) $S 900 tests_$c -- env AMVPT_LIB_DIR=$GRAFT_REPO_ROOT/mitsuba3-amvpt_amd/$c python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread ;;
    smoke) $S 300 smoke -- python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) $S 500 bench_$c -- python -u bench.py --steps 5 --warmup 1 $P ;;
    quick) $S 300 quick_$c -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --rmse-lanes 0 $P ;;
    trace) $S 300 trace_$c -- rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_trace_$c -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --rmse-lanes 0 --one-stream $P ;;
    fetch) $S 300 fetch_$c -- rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_fetch_$c -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0 $P ;;
    write) $S 300 write_$c -- rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_write_$c -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0 $P ;;
    sqA) $S 200 sqA_$c -- rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH --output-format csv -d gpurun_out/${T}_sqA_$c -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --rmse-lanes 0 $P ;;
    abflags) $S 600 abflags_$c -- env AB_CONFIG=$c python -u tools/ab_value.py --kernels --env AB_FLAGS=0 --env AB_FLAGS=32 --env AB_FLAGS=0 --env AB_FLAGS=32 ;;
    abchunk) $S 600 abchunk_$c -- env AB_CONFIG=$c python -u tools/ab_value.py --kernels --env AB_CHUNK=0 --env AB_CHUNK=33554432 --env AB_CHUNK=16777216 --env AB_CHUNK=0 --env AB_CHUNK=33554432 ;;
    ablib) $S 900 ablib_$c -- env AB_CONFIG=${c%%+*} python -u tools/ab_value.py --kernels $(echo ${c#*+} | tr '+' ' ') ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
  if [ -f gpurun_out/${T}.stop ]; then echo "stopped after $st"; break; fi
done
cat gpurun_out/${T}_steps.log
