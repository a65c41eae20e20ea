# the slab-march experiment: tools/experiments/r05_pruned/slab_march.patch applied (builds lib_exp / lib_stats as the line below says)
# build: lib_exp (EXTRA=-DVR_EXPERIMENTS); lib_* must travel
# round 5: where the slab march's time goes -- SQ counters, slab vs shipped kernel, c3_ref and c3
set -o pipefail
O=gpurun_out/r05_m19b; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/volumetric-renderer_amd/lib_exp/libvr_amd.so
for v in 0 1; do
  for cfg in c3_ref; do
    if [ $v = 1 ]; then export VR_SLAB=1; else unset VR_SLAB; fi
    VR_AMD_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_SALU -d $O/pmc1_${v}_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --no-variants --no-cpu-baseline --steps 10 --warmup 3 > $O/pmc1_${v}_$cfg.log 2>&1 || exit 1
    VR_AMD_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS TD_TD_BUSY_sum TD_TC_STALL_sum -d $O/pmc2_${v}_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --no-variants --no-cpu-baseline --steps 10 --warmup 3 > $O/pmc2_${v}_$cfg.log 2>&1 || exit 1
  done
done
