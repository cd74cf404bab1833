# A/B variant builds (Makefile LIB=lib_x ...): stage times of one bench run per library dir.
# usage: bash tools/ab.sh <tag> <libdir> [<libdir> ...]   (dirs relative to mitsuba3-amvpt_amd/)
set -e
TAG=$1; shift
mkdir -p gpurun_out
for L in "$@"; do
  AMVPT_LIB_DIR=$PWD/mitsuba3-amvpt_amd/$L timeout -k 10 120 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_$L.json 2> gpurun_out/${TAG}_$L.err
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_$L.json')); print('$L', d['value'], d['roofline']['stage_ms'])"
done
