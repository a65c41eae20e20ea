# build: make -C volumetric-renderer_amd EXTRA=-DVR_DEFER_SHADE=0 LIBDIR=lib_d0 BUILDDIR=build_d0 (lib_* must travel for the call)
# round 5: deferred shading off (VR_DEFER_SHADE=0: the headline kernel 80 -> 65 VGPRs, 6 -> 7
# waves per SIMD, no spills) against the default, alternating, 3 rounds; C3 (3 in flight),
# C3 default camera, C3 serial frames (frames_in_flight 1)
set -o pipefail
O=gpurun_out/r05_m12; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for b in lib lib_d0; do
    for cfg in c3 c3_default; do
      VR_AMD_LIB=$PWD/volumetric-renderer_amd/$b/libvr_amd.so timeout -k 10 150 python -u bench.py --config $cfg --no-variants --no-cpu-baseline --steps 40 --warmup 10 > $O/b_${b}_${cfg}_$r.json 2> $O/b_${b}_${cfg}_$r.err || exit 1
      python -c "import json,sys; d=json.load(open('$O/b_${b}_${cfg}_$r.json')); print('$b', '$cfg', $r, d['value'], d['ms_per_step'])"
    done
  done
done
for b in lib lib_d0; do
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$b/libvr_amd.so timeout -k 10 200 python -u bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline > $O/full_${b}.json 2> $O/full_${b}.err || exit 1
  python - $O/full_${b}.json $b <<'PY'
import json,sys
d=json.load(open(sys.argv[1])); v=d.get('variants',{})
print(sys.argv[2], 'c3', d['value'], {k:(x.get('value') if isinstance(x,dict) else x) for k,x in v.items()})
PY
done
