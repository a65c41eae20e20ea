# banded vr_render (lib) vs single launch + one pageable copy (lib_old): host-output fps
set -o pipefail
O=gpurun_out/ab_host; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 &&
for r in 1 2; do for L in lib lib_old; do
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_${L}_$r.json 2> $O/bench_${L}_$r.err || exit $?
done; done
