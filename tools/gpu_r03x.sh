# r03x: attribution of the config-M splat (measurement-only builds, wrong images): lib_a1 skips the LDS
# window adds, lib_a2 the flush's film atomics, lib_a4 the filter weights
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/ab_value.py --kernels lib lib_a1 lib_a2 lib_a4 lib > gpurun_out/r03x_ab_attr_M.log 2>&1 || exit 1
echo done
