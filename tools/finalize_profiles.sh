# Copy one gpu_all.sh call's outputs (gpurun_out/<tag>_*) into profiles/: bench lines (the JSON line of each
# bench log), kernel-trace summaries, PMC traffic / VALU summaries and SQ counters, A/B logs, test log, smoke.
set -e
T=${1:-r04z}
G=gpurun_out
P=profiles
for c in M C3 mesh C5; do
  [ -f $G/${T}_bench_$c.log ] && grep '^{' $G/${T}_bench_$c.log | tail -1 > $P/${T}_bench_$c.json
done
for c in M C3 mesh C5; do
  [ -f $G/${T}_trace_$c/run_kernel_stats.csv ] && cp $G/${T}_trace_$c/run_kernel_stats.csv $P/${T}_kernel_stats_$c.csv
  sfx=$([ $c = M ] && echo "" || echo "_$c")
  if [ -f $G/${T}_fetch_$c/pmc_counter_collection.csv ] && [ -f $G/${T}_write_$c/pmc_counter_collection.csv ]; then
    python3 tools/pmc_traffic.py $G/${T}_fetch_$c $G/${T}_write_$c $P/${T}_traffic$sfx.json $c > /dev/null
  fi
  if [ -f $G/${T}_sqA_$c/pmc_counter_collection.csv ]; then
    python3 tools/pmc_valu.py $G/${T}_sqA_$c $P/${T}_valu$sfx.json $c > /dev/null
    python3 tools/pmc_summary.py $G/${T}_sqA_$c > $P/${T}_sq_counters$sfx.txt
  fi
done
for c in M C3 mesh C5; do
  [ -f $G/${T}_quick_$c.log ] && grep '^{' $G/${T}_quick_$c.log | tail -1 > $P/${T}_quick_$c.json
  [ -f $G/${T}_ab$c.log ] && grep '^{' $G/${T}_ab$c.log > $P/${T}_ab_$c.log || true
done
[ -f $G/${T}_tests.log ] && cp $G/${T}_tests.log $P/${T}_gpu_tests.txt
[ -f $G/${T}_smoke.log ] && cp $G/${T}_smoke.log $P/${T}_smoke.txt
cp $G/${T}_steps.log $P/${T}_steps.log
ls $P | grep "^$T"
