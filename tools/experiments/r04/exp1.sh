# round 4: GPU suite, td_mask timing + PMC, default-camera timeline (WG_TIMES build), queue A/B
set -o pipefail
O=gpurun_out/r04_e1c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 ./tools/experiments/r04/td_mask > $O/td_mask.json 2>&1 && cat $O/td_mask.json || exit 1
i=0
for G in "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" "TD_TD_BUSY_sum TD_TC_STALL_sum" "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $G -d $O/td_pmc/p$i -o run --output-format csv -- ./tools/experiments/r04/td_mask > $O/td_pmc_p$i.log 2>&1 || exit 1
done
python tools/experiments/r04/td_pmc.py $O/td_pmc $O/td_mask.json > $O/td_pmc.json && cat $O/td_pmc.json | head -80
VR_AMD_LIB=$PWD/volumetric-renderer_amd/lib_wgt/libvr_amd.so timeout -k 10 300 python -u tools/experiments/r04/default_timeline.py $O/timeline > $O/timeline.log 2>&1 && cat $O/timeline.log | cut -c1-600
timeout -k 10 600 python -u tools/experiments/r04/queue_ab.py 2 default,fill,diag > $O/queue_ab.jsonl 2> $O/queue_ab.err && cat $O/queue_ab.jsonl
