# round 5, fourth GPU call: brick geometries whose rows / slices are one 64-B sector
# (TCP_TOTAL_CACHE_ACCESSES is counted per lane-quad and sector: td_mask, profiles/r05/m3):
# f32 GeomWide 7x7x8 cells (8-element z-pair rows = 64 B) and 8-bit 7x7x8 (8-B rows, 64-B
# slices), against the default 8^3 / 7x8x8, alternating, two rounds; TCP counters on C3/C4;
# then the parity files on the geometry build
set -o pipefail
O=gpurun_out/r05_m4; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for b in lib lib_g77; do
    for cfg in c3 c3_ref c3_default c4 c2; do
      VR_AMD_LIB=$PWD/volumetric-renderer_amd/$b/libvr_amd.so timeout -k 10 150 python -u bench.py --config $cfg --no-variants --no-cpu-baseline --steps 40 --warmup 10 > $O/b_${b}_${cfg}_$r.json 2> $O/b_${b}_${cfg}_$r.err || exit 1
      python -c "import json,sys; d=json.load(open('$O/b_${b}_${cfg}_$r.json')); print('$b', '$cfg', $r, d['value'], d['ms_per_step'], d['config']['volume_resident_bytes'])"
    done
  done
done
for b in lib lib_g77; do
  for cfg in c3 c4; do
    VR_AMD_LIB=$PWD/volumetric-renderer_amd/$b/libvr_amd.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TD_TD_BUSY_sum TD_TC_STALL_sum -d $O/pmc_${b}_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --no-variants --no-cpu-baseline --steps 10 --warmup 3 > $O/pmc_${b}_$cfg.log 2>&1 || exit 1
    VR_AMD_LIB=$PWD/volumetric-renderer_amd/$b/libvr_amd.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_RD FETCH_SIZE -d $O/pmc2_${b}_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --no-variants --no-cpu-baseline --steps 10 --warmup 3 > $O/pmc2_${b}_$cfg.log 2>&1 || exit 1
  done
done
VR_AMD_LIB=$PWD/volumetric-renderer_amd/lib_g77/libvr_amd.so timeout -k 10 240 python -u -m pytest tests/test_gpu_random.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_g77.log 2>&1; rc=$?; echo "g77 rc=$rc"; tail -2 $O/pytest_g77.log; exit $rc
