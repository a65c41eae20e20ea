# round 4: f32 z-pair cross-lane sharing A/B on C3 (headline, reference semantics, default
# camera), alternating builds, 2 rounds; then the parity files on the share build
set -o pipefail
O=gpurun_out/r04_e3; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for b in lib lib_f32share; do
    for cfg in c3 c3_ref c3_default; do
      VR_AMD_LIB=$PWD/volumetric-renderer_amd/$b/libvr_amd.so timeout -k 10 240 python -u bench.py --config $cfg --no-variants --no-cpu-baseline --steps 40 --warmup 10 > $O/b_${b}_${cfg}_$r.json 2> $O/b_${b}_${cfg}_$r.err || exit 1
      python -c "import json,sys; d=json.load(open('$O/b_${b}_${cfg}_$r.json')); print('$b', '$cfg', $r, d['value'], d['ms_per_step'])"
    done
  done
done
VR_AMD_LIB=$PWD/volumetric-renderer_amd/lib_f32share/libvr_amd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_random.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_f32share.log 2>&1; echo "f32share rc=$?"; tail -2 $O/pytest_f32share.log
