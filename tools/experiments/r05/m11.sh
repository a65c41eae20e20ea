# build: make -C volumetric-renderer_amd EXTRA=-DVR_EXPERIMENTS LIBDIR=lib_exp BUILDDIR=build_exp (and let lib_exp travel: drop lib_* from .gpurunignore for the call)
# round 5, occupancy cap: dynamic LDS per march workgroup (VR_MARCH_LDS_PAD, experiment build
# lib_exp) caps the workgroups resident on a CU -- 6 (no pad), 5, 4, 3 -- fewer waves sharing
# the CU's L1.  C3 (3 in flight and serial), C3 reference semantics, C4; alternating, 2 rounds
set -o pipefail
O=gpurun_out/r05_m11; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/volumetric-renderer_amd/lib_exp/libvr_amd.so
for r in 1 2; do
  for pad in 0 21744 27744 39744; do
    for cfg in c3 c3_ref c4; do
      VR_MARCH_LDS_PAD=$pad VR_AMD_LIB=$L timeout -k 10 150 python -u bench.py --config $cfg --no-variants --no-cpu-baseline --steps 40 --warmup 10 > $O/b_${pad}_${cfg}_$r.json 2> $O/b_${pad}_${cfg}_$r.err || exit 1
      python -c "import json,sys; d=json.load(open('$O/b_${pad}_${cfg}_$r.json')); print('$pad', '$cfg', $r, d['value'], d['ms_per_step'], d['roofline'].get('serial_kernel_ms'))"
    done
  done
done
for pad in 0 27744; do
  VR_MARCH_LDS_PAD=$pad VR_AMD_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TD_TD_BUSY_sum TD_TC_STALL_sum -d $O/pmc_${pad} -o run --output-format csv -- python3 bench.py --config c3 --no-variants --no-cpu-baseline --steps 10 --warmup 3 > $O/pmc_${pad}.log 2>&1 || exit 1
done
