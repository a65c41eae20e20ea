# round 5, third GPU call: the whole GPU suite on the current default build; the 8-bit
# lane-sharing A/B on C4 (VR_U8_SHARE 1/2 against the default, alternating, two rounds) with
# TD/TCP/SQ counters per build and the parity files on the share builds; td_mask (what
# TCP_TOTAL_CACHE_ACCESSES counts); FETCH/WRITE bytes of the once-per-voxel field build
# (VR_FIELD_PLAIN) on C3; unprofiled bench lines of C2/C4/C5 on the default build
set -o pipefail
O=gpurun_out/r05_m3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for b in lib lib_share1 lib_share2; do
    VR_AMD_LIB=$PWD/volumetric-renderer_amd/$b/libvr_amd.so timeout -k 10 200 python -u tools/experiments/r04/u8_ab.py $b >> $O/u8_ab.jsonl 2>> $O/u8_ab.err || exit 1
  done
done
echo "u8 A/B done"
for b in lib lib_share1 lib_share2; do
  i=0
  for G in "TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum" "SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
    i=$((i+1))
    VR_AMD_LIB=$PWD/volumetric-renderer_amd/$b/libvr_amd.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $G -d $O/pmc_$b/p$i -o run --output-format csv -- python3 bench.py --config c4 --no-variants --no-cpu-baseline --steps 10 --warmup 3 > $O/pmc_${b}_p$i.log 2>&1 || exit 1
  done
done
for b in lib lib_share1 lib_share2; do python tools/pmc_report.py $O/pmc_$b > $O/pmc_$b.txt 2>&1; done
echo "u8 counters done"
timeout -k 10 120 ./tools/experiments/r04/td_mask > $O/td_mask.json 2>&1 || exit 1
i=0
for G in "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" "TD_TD_BUSY_sum TD_TC_STALL_sum" "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $G -d $O/td_pmc/p$i -o run --output-format csv -- ./tools/experiments/r04/td_mask > $O/td_pmc_p$i.log 2>&1 || exit 1
done
python tools/experiments/r04/td_pmc.py $O/td_pmc $O/td_mask.json > $O/td_pmc.json
echo "td_mask done"
for ctr in FETCH_SIZE WRITE_SIZE; do
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/lib_fplain/libvr_amd.so timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d $O/fplain_pmc_$ctr -o run --output-format csv -- python3 bench.py --config c3 --no-variants --no-cpu-baseline --steps 10 --warmup 3 > $O/fplain_pmc_$ctr.log 2>&1 || exit 1
done
for cfg in c2 c4 c5; do
  timeout -k 10 300 python -u bench.py --config $cfg --no-variants --no-cpu-baseline --steps 100 --warmup 20 > $O/bench_$cfg.json 2> $O/bench_$cfg.err || exit 1
  python -c "import json; d=json.load(open('$O/bench_$cfg.json')); print('$cfg', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
for b in lib_share1 lib_share2; do
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$b/libvr_amd.so timeout -k 10 240 python -u -m pytest tests/test_gpu_random.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_$b.log 2>&1; rc=$?; echo "$b rc=$rc"; tail -2 $O/pytest_$b.log; [ $rc -le 1 ] || exit $rc
done
