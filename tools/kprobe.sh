# Register / scratch usage of ONE kernel instance without building the whole library (seconds):
#   bash tools/kprobe.sh '<explicit instantiation>' [EXTRA hipcc flags]
# e.g. bash tools/kprobe.sh 'template __global__ void k_splat_multi<8, 4, true>(KParams, const DView *, Bufs);'
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
printf '#define AMVPT_KERNEL_PROBE 1\n#include "%s/mitsuba3-amvpt_amd/csrc/amvpt_render.hip"\nnamespace amvpt {\n%s\n}\n' "$R" "$1" > $T/probe.hip
shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize --cuda-device-only -S -o $T/probe.s $T/probe.hip "$@" 2>&1 | grep -v warning | grep -v "^ *[0-9]* |" | grep -v "^\s*\^" | grep -v "generated" || true
grep -E "^\s+\.(name|vgpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count|private_segment_fixed_size|group_segment_fixed_size):" $T/probe.s | grep -v "\.name:\s*$" 
cp $T/probe.s /tmp/kprobe.s
rm -rf $T
