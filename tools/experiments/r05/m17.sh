# the slab-march experiment: tools/experiments/r05_pruned/slab_march.patch applied (builds lib_exp / lib_stats as the line below says)
# build: make -C volumetric-renderer_amd EXTRA=-DVR_EXPERIMENTS LIBDIR=lib_exp BUILDDIR=build_exp (lib_* must travel for the call)
# round 5: slab march (VR_SLAB=1: rays of a tile advance through LDS-staged slabs) -- parity
# files on it first, then against the shipped kernels in the same library, alternating
set -o pipefail
O=gpurun_out/r05_m17; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/volumetric-renderer_amd/lib_exp/libvr_amd.so
VR_SLAB=1 VR_AMD_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_slab.log 2>&1; rc=$?; tail -4 $O/pytest_slab.log; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1; do
    for cfg in c3 c3_ref; do
      if [ $v = 1 ]; then export VR_SLAB=1; else unset VR_SLAB; fi
      VR_AMD_LIB=$L timeout -k 10 150 python -u bench.py --config $cfg --no-variants --no-cpu-baseline --steps 40 --warmup 10 > $O/b_${v}_${cfg}_$r.json 2> $O/b_${v}_${cfg}_$r.err || exit 1
      python -c "import json,sys; d=json.load(open('$O/b_${v}_${cfg}_$r.json')); print('slab=$v', '$cfg', $r, d['value'], d['ms_per_step'], d['roofline']['kernel'][:60])"
    done
  done
done
