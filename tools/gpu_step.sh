# Run GPU steps in order, each under its own time limit; stop at the first step that
# crashed, faulted or timed out (exit 124/134/137/139 or a signal), continue after plain
# failures (exit 1, e.g. a failing assertion) so one call still yields every report.
#   bash tools/gpu_step.sh <tag> <seconds> <name> -- <cmd...>   (one step; appends to gpurun_out/<tag>_steps.log)
TAG=$1; SECS=$2; NAME=$3; shift 4
mkdir -p gpurun_out
if [ -f gpurun_out/${TAG}.stop ]; then echo "skip $NAME (earlier crash)" >> gpurun_out/${TAG}_steps.log; exit 0; fi
echo "start $NAME $(date +%T)" >> gpurun_out/${TAG}_steps.log
timeout -k 10 "$SECS" "$@" > gpurun_out/${TAG}_${NAME}.log 2>&1
rc=$?
echo "end $NAME rc=$rc $(date +%T)" >> gpurun_out/${TAG}_steps.log
case $rc in
  0|1|2|5) exit 0 ;;
  *) touch gpurun_out/${TAG}.stop; exit 0 ;;
esac
