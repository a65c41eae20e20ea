# 32-row march tiles (lib_r32, VR_MARCH_ROWS=32) vs 16-row (lib): parity, bench, views
set -o pipefail
O=gpurun_out/ab_r32; mkdir -p $O
export TMPDIR=/tmp
B=$PWD/volumetric-renderer_amd/lib_r32/libvr_amd.so
VR_AMD_LIB=$B timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_b16.log 2>&1 &&
for r in 1 2; do for L in lib lib_r32; do
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_${L}_$r.json 2> $O/bench_${L}_$r.err || exit $?
done; done &&
for L in lib lib_r32; do
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 200 python tools/view_sweep.py > $O/views_${L}.txt 2>&1 || exit $?
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 200 python tools/view_sweep.py --shading 1 --ert 1e-5 > $O/views_shaded_${L}.txt 2>&1 || exit $?
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 200 python tools/view_sweep.py --n 1024 --dtype uint8 --size 2048x2048 > $O/views_u8_${L}.txt 2>&1 || exit $?
done
