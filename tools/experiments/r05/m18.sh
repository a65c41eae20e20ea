# the slab-march experiment: tools/experiments/r05_pruned/slab_march.patch applied (builds lib_exp / lib_stats as the line below says)
# build: lib_exp (EXTRA=-DVR_EXPERIMENTS), lib_stats (EXTRA="-DVR_EXPERIMENTS -DVR_SLAB_STATS"); lib_* must travel
# round 5: slab march with batched staging loads -- counters, parity, A/B against the shipped kernels
set -o pipefail
O=gpurun_out/r05_m18c; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/volumetric-renderer_amd/lib_exp/libvr_amd.so
VR_AMD_LIB=$PWD/volumetric-renderer_amd/lib_stats/libvr_amd.so timeout -k 10 200 python -u tools/experiments/r05/slab_stats.py c3 c3_ref c3_default > $O/stats.jsonl 2> $O/stats.err; rc=$?; cat $O/stats.jsonl; [ $rc = 0 ] || { tail -5 $O/stats.err; exit $rc; }
VR_SLAB=1 VR_AMD_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_slab.log 2>&1; rc=$?; tail -2 $O/pytest_slab.log; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1; do
    for cfg in c3 c3_ref; do
      if [ $v = 1 ]; then export VR_SLAB=1; else unset VR_SLAB; fi
      VR_AMD_LIB=$L timeout -k 10 150 python -u bench.py --config $cfg --no-variants --no-cpu-baseline --steps 40 --warmup 10 > $O/b_${v}_${cfg}_$r.json 2> $O/b_${v}_${cfg}_$r.err || exit 1
      python -c "import json,sys; d=json.load(open('$O/b_${v}_${cfg}_$r.json')); print('slab=$v', '$cfg', $r, d['value'], d['ms_per_step'])"
    done
  done
done
