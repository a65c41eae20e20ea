# A/B old (divergent-exit PIPE loop) vs new (uniform loop): rank shares with 3 frames in flight
set -o pipefail
O=gpurun_out/ab4; mkdir -p $O
for r in 1 2; do for L in lib_old lib; do
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 200 python tools/inflight_sweep.py --streams 1,3 --frames 150 > $O/${L}_shaded_$r.txt 2>&1 || exit $?
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 200 python tools/inflight_sweep.py --streams 3 --frames 150 --shading 0 --ert 0 > $O/${L}_ref_$r.txt 2>&1 || exit $?
done; done
