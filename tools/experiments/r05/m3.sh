# round 5, third GPU call: the 8-bit lane-sharing A/B on C4, alternating
# builds, TD/TCP/SQ counters per build; td_mask (what TCP_TOTAL_CACHE_ACCESSES counts); the
# parity files on the share builds
set -o pipefail
O=gpurun_out/r05_m3; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for b in lib lib_share1 lib_share2; do
    VR_AMD_LIB=$PWD/volumetric-renderer_amd/$b/libvr_amd.so timeout -k 10 200 python -u tools/experiments/r04/u8_ab.py $b >> $O/u8_ab.jsonl 2>> $O/u8_ab.err || exit 1
  done
done
cat $O/u8_ab.jsonl
for b in lib lib_share1 lib_share2; do
  i=0
  for G in "TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum" "SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
    i=$((i+1))
    VR_AMD_LIB=$PWD/volumetric-renderer_amd/$b/libvr_amd.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $G -d $O/pmc_$b/p$i -o run --output-format csv -- python3 bench.py --config c4 --no-variants --no-cpu-baseline --steps 10 --warmup 3 > $O/pmc_${b}_p$i.log 2>&1 || exit 1
  done
done
for b in lib lib_share1 lib_share2; do python tools/pmc_report.py $O/pmc_$b > $O/pmc_$b.txt 2>&1; done
timeout -k 10 120 ./tools/experiments/r04/td_mask > $O/td_mask.json 2>&1 || exit 1
i=0
for G in "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" "TD_TD_BUSY_sum TD_TC_STALL_sum" "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $G -d $O/td_pmc/p$i -o run --output-format csv -- ./tools/experiments/r04/td_mask > $O/td_pmc_p$i.log 2>&1 || exit 1
done
python tools/experiments/r04/td_pmc.py $O/td_pmc $O/td_mask.json > $O/td_pmc.json
for b in lib_share1 lib_share2; do
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$b/libvr_amd.so timeout -k 10 240 python -u -m pytest tests/test_gpu_random.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_$b.log 2>&1; rc=$?; echo "$b rc=$rc"; tail -2 $O/pytest_$b.log; [ $rc -le 1 ] || exit $rc
done
