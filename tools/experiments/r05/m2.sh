# round 5, second GPU call: the queue A/B (tile order 5 against 4),
# the f32 lane-sharing build (VR_F32_SHARE) and the once-per-voxel binary16 field
# (VR_FIELD_PLAIN) against the default build on C3, alternating builds, two rounds; then the
# parity files on both experiment builds
set -o pipefail
O=gpurun_out/r05_m2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/experiments/r04/queue_ab.py 2 default,fill,diag > $O/queue_ab.jsonl 2> $O/queue_ab.err || exit 1
echo "queue done"
for r in 1 2; do
  for b in lib lib_f32share lib_fplain; do
    for cfg in c3 c3_default c3_ref; do
      [ $b = lib_fplain ] && [ $cfg = c3_ref ] && continue
      VR_AMD_LIB=$PWD/volumetric-renderer_amd/$b/libvr_amd.so timeout -k 10 150 python -u bench.py --config $cfg --no-variants --no-cpu-baseline --steps 40 --warmup 10 > $O/b_${b}_${cfg}_$r.json 2> $O/b_${b}_${cfg}_$r.err || exit 1
      python -c "import json,sys; d=json.load(open('$O/b_${b}_${cfg}_$r.json')); print('$b', '$cfg', $r, d['value'], d['ms_per_step'], d['roofline']['kernel'])"
    done
  done
done
for b in lib_fplain lib_f32share; do
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$b/libvr_amd.so timeout -k 10 240 python -u -m pytest tests/test_gpu_random.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_$b.log 2>&1; rc=$?; echo "$b rc=$rc"; tail -2 $O/pytest_$b.log; [ $rc -le 1 ] || exit $rc
done
