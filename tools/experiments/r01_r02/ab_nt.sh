# non-temporal difference-field loads (lib_nt, VR_GRAD_NT=1) vs lib: parity, C3 bench, shaded views
set -o pipefail
O=gpurun_out/ab_nt; mkdir -p $O
export TMPDIR=/tmp
B=$PWD/volumetric-renderer_amd/lib_nt/libvr_amd.so
VR_AMD_LIB=$B timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_nt.log 2>&1 &&
for r in 1 2; do for L in lib lib_nt; do
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-variants > $O/bench_${L}_$r.json 2> $O/bench_${L}_$r.err || exit $?
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-variants --frames-in-flight 1 > $O/bench1_${L}_$r.json 2> $O/bench1_${L}_$r.err || exit $?
done; done &&
for L in lib lib_nt; do
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 200 python tools/view_sweep.py --shading 1 --ert 1e-5 > $O/views_shaded_${L}.txt 2>&1 || exit $?
done
