# Copy the A/B results of gpu_run.sh calls (gpurun_out/<tag>_ablib_<cfg>+<variants>.log and
# <tag>_abflags_<cfg>.log) into profiles/<tag>_ab_<cfg>.log: the variant JSON lines, headed by the variant list.
#   bash tools/collect_ab.sh r05      (every tag starting with r05)
set -e
pre=${1:-r05}
cd "$(dirname "$0")/.."
for f in gpurun_out/${pre}*_ablib_*.log gpurun_out/${pre}*_abflags_*.log; do
  [ -f "$f" ] || continue
  b=$(basename "$f" .log)
  tag=${b%%_ab*}
  rest=${b#*_ab}            # lib_<cfg>+<variants> or flags_<cfg>
  kind=${rest%%_*}          # lib | flags
  spec=${rest#*_}
  cfg=${spec%%+*}
  out=profiles/${tag}_ab_${cfg}.log
  [ "$kind" = flags ] && out=profiles/${tag}_ab_flags_${cfg}.log
  {
    if [ "$kind" = lib ]; then echo "# config $cfg, variant libraries (in run order): ${spec#*+}" | tr '+' ' ';
    else echo "# config $cfg, amvpt_render_opts.flags A/B (AB_FLAGS)"; fi
    grep '^{' "$f" || true
  } > "$out"
done
ls profiles | grep "^${pre}.*_ab_" || true
