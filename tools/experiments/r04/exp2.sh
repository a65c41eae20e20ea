# u8 cross-lane sharing A/B (C4: 1024^3 u8 @ 2048^2), alternating builds, 2 rounds, then the
# GPU suite on the share builds (bit-identity) -- round 4
set -o pipefail
O=gpurun_out/r04_e2; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for b in lib lib_share1 lib_share2; do
    VR_AMD_LIB=$PWD/volumetric-renderer_amd/$b/libvr_amd.so timeout -k 10 240 python -u tools/experiments/r04/u8_ab.py $b >> $O/u8_ab.jsonl 2>> $O/u8_ab.err || exit 1
  done
done
cat $O/u8_ab.jsonl
for b in lib_share1 lib_share2; do
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$b/libvr_amd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_random.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_$b.log 2>&1; echo "$b rc=$?"; tail -2 $O/pytest_$b.log
done
