# timing bound: C3 without the difference-field loads (lib_nog, wrong gradient) vs lib
set -o pipefail
O=gpurun_out/ab_nog; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do for L in lib lib_nog; do
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-variants > $O/bench_${L}_$r.json 2> $O/bench_${L}_$r.err || exit $?
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-variants --frames-in-flight 1 > $O/bench1_${L}_$r.json 2> $O/bench1_${L}_$r.err || exit $?
done; done
