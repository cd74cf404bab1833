# End-of-round measurement set: parity tests + smoke + the default bench line + kernel trace + PMC
# traffic (tools/gpu_round.sh), SQ instruction counts (tools/pmc_sq.sh), and the other configs' lines.
# usage: bash tools/gpu_final.sh <tag>
T=$1
bash tools/gpu_round.sh $T all || exit 1
bash tools/pmc_sq.sh $T || exit 1
for c in C3 C5 mesh; do
  timeout -k 10 400 python -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_bench_$c.json 2> gpurun_out/${T}_bench_$c.err || exit 1
done
echo final-done
