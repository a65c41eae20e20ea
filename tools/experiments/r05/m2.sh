# round 5, second GPU call: the round-4 A/Bs that never ran, part 1:
# td_mask timings + TD/TCP counters, the default-camera workgroup timeline (WG_TIMES build),
# the queue A/B (tile order 5 against 4), and the f32 lane-sharing A/B (exp3) with its parity
set -o pipefail
O=gpurun_out/r05_m2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./tools/experiments/r04/td_mask > $O/td_mask.json 2>&1 || exit 1
i=0
for G in "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" "TD_TD_BUSY_sum TD_TC_STALL_sum" "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $G -d $O/td_pmc/p$i -o run --output-format csv -- ./tools/experiments/r04/td_mask > $O/td_pmc_p$i.log 2>&1 || exit 1
done
python tools/experiments/r04/td_pmc.py $O/td_pmc $O/td_mask.json > $O/td_pmc.json
echo "td done"
VR_AMD_LIB=$PWD/volumetric-renderer_amd/lib_wgt/libvr_amd.so timeout -k 10 200 python -u tools/experiments/r04/default_timeline.py $O/timeline > $O/timeline.log 2>&1 || exit 1
echo "timeline done"
timeout -k 10 400 python -u tools/experiments/r04/queue_ab.py 2 default,fill,diag > $O/queue_ab.jsonl 2> $O/queue_ab.err || exit 1
echo "queue done"
for r in 1 2; do
  for b in lib lib_f32share; do
    for cfg in c3 c3_ref c3_default; do
      VR_AMD_LIB=$PWD/volumetric-renderer_amd/$b/libvr_amd.so timeout -k 10 180 python -u bench.py --config $cfg --no-variants --no-cpu-baseline --steps 40 --warmup 10 > $O/b_${b}_${cfg}_$r.json 2> $O/b_${b}_${cfg}_$r.err || exit 1
      python -c "import json,sys; d=json.load(open('$O/b_${b}_${cfg}_$r.json')); print('$b', '$cfg', $r, d['value'], d['ms_per_step'])"
    done
  done
done
VR_AMD_LIB=$PWD/volumetric-renderer_amd/lib_f32share/libvr_amd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_random.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_f32share.log 2>&1; rc=$?; echo "f32share rc=$rc"; tail -2 $O/pytest_f32share.log; exit $rc
