# launch tuner (lib) vs static policy (lib_notune, VR_TUNE=0): GPU tests with the tuner, C3 bench x2, views
set -o pipefail
O=gpurun_out/ab_tune; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_lib.log 2>&1 || exit $?
for r in 1 2; do for L in lib lib_notune; do
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_${L}_$r.json 2> $O/bench_${L}_$r.err || exit $?
done; done
for L in lib lib_notune; do
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 200 python tools/view_sweep.py --reps 40 > $O/views_${L}.txt 2>&1 || exit $?
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 200 python tools/view_sweep.py --reps 40 --shading 1 --ert 1e-5 > $O/views_shaded_${L}.txt 2>&1 || exit $?
done
