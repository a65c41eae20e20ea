# build: lib = the single-exit loop (tools/experiments/r05_pruned/single_exit_loop.patch applied), lib_base = the shipped build copied aside (lib_* must travel for the call)
# round 5: the pipelined march with one exit per loop iteration (the next stage's loads no
# longer wait behind the field loads; half-field kernel at a 6-wave floor) = lib, against the
# previous build (lib_base = the 03073e13 code), alternating, 2 rounds; then the parity files
set -o pipefail
O=gpurun_out/r05_m14; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for b in lib_base lib; do
    for cfg in c3 c3_ref c3_default c4 c2; do
      VR_AMD_LIB=$PWD/volumetric-renderer_amd/$b/libvr_amd.so timeout -k 10 150 python -u bench.py --config $cfg --no-variants --no-cpu-baseline --steps 40 --warmup 10 > $O/b_${b}_${cfg}_$r.json 2> $O/b_${b}_${cfg}_$r.err || exit 1
      python -c "import json,sys; d=json.load(open('$O/b_${b}_${cfg}_$r.json')); print('$b', '$cfg', $r, d['value'], d['ms_per_step'])"
    done
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_random.py tests/test_gpu_golden.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; exit $rc
