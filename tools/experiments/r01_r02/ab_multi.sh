# A/B of experiment builds: parity (first variant), C3 bench x2 alternating, unshaded + shaded view sweeps
# usage: bash tools/experiments/r01_r02/ab_multi.sh <tag> lib lib_a [lib_b ...]
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
VR_AMD_LIB=$PWD/volumetric-renderer_amd/$2/libvr_amd.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_$2.log 2>&1 || exit $?
for r in 1 2; do for L in "$@"; do
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_${L}_$r.json 2> $O/bench_${L}_$r.err || exit $?
done; done
for L in "$@"; do
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 200 python tools/view_sweep.py > $O/views_${L}.txt 2>&1 || exit $?
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 200 python tools/view_sweep.py --shading 1 --ert 1e-5 > $O/views_shaded_${L}.txt 2>&1 || exit $?
done
