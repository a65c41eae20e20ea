# build: make -C volumetric-renderer_amd EXTRA=-DVR_EXPERIMENTS LIBDIR=lib_exp BUILDDIR=build_exp (lib_* must travel for the call)
# round 5: contiguous frame regions per XCD (VR_XCD_REGIONS: tiles in Hilbert order cut into 8
# runs of equal measured duration, each run sorted longest first on its XCD) against tile
# order 4's interleaved super-tiles; alternating, 2 rounds; then L2 hit/miss counters on C3
set -o pipefail
O=gpurun_out/r05_m15; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/volumetric-renderer_amd/lib_exp/libvr_amd.so
for r in 1 2; do
  for v in 0 1; do
    for cfg in c3 c3_ref c3_default c4; do
      if [ $v = 1 ]; then export VR_XCD_REGIONS=1; else unset VR_XCD_REGIONS; fi
      VR_AMD_LIB=$L timeout -k 10 150 python -u bench.py --config $cfg --no-variants --no-cpu-baseline --steps 40 --warmup 10 > $O/b_${v}_${cfg}_$r.json 2> $O/b_${v}_${cfg}_$r.err || exit 1
      python -c "import json,sys; d=json.load(open('$O/b_${v}_${cfg}_$r.json')); print('regions=$v', '$cfg', $r, d['value'], d['ms_per_step'])"
    done
  done
done
unset VR_XCD_REGIONS
for v in 0 1; do
  if [ $v = 1 ]; then export VR_XCD_REGIONS=1; else unset VR_XCD_REGIONS; fi
  VR_AMD_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TD_TD_BUSY_sum TD_TC_STALL_sum -d $O/pmc_${v} -o run --output-format csv -- python3 bench.py --config c3 --no-variants --no-cpu-baseline --steps 10 --warmup 3 > $O/pmc_${v}.log 2>&1 || exit 1
done
