# r03k: suffix-walk occupancy A/B on mesh (launch bounds 1 / 6 / 8 waves per SIMD)
mkdir -p gpurun_out
AB_CONFIG=mesh timeout -k 10 500 python -u tools/ab_value.py --kernels lib lib_w6 lib_w8 lib lib_w6 lib_w8 > gpurun_out/r03k_ab_mesh.log 2>&1 || exit 1
echo done
