# plain f32 layout (lib_plain, VR_F32_PLAIN=1) vs z-pair (lib): parity, bench, views
set -o pipefail
O=gpurun_out/ab5; mkdir -p $O
PL=$PWD/volumetric-renderer_amd/lib_plain/libvr_amd.so
VR_AMD_LIB=$PL timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_plain.log 2>&1 &&
for r in 1 2; do for L in lib lib_plain; do
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_${L}_$r.json 2> $O/bench_${L}_$r.err || exit $?
done; done &&
for L in lib lib_plain; do
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 200 python tools/view_sweep.py > $O/views_${L}.txt 2>&1 || exit $?
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 200 python tools/view_sweep.py --shading 1 --ert 1e-5 > $O/views_shaded_${L}.txt 2>&1 || exit $?
done
