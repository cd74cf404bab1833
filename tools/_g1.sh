set -e
mkdir -p gpurun_out
timeout -k 10 900 python tools/ab_value.py --kernels lib lib_a1 lib_a2 lib_a4 > gpurun_out/r02g_ab.log 2>&1
echo ok
