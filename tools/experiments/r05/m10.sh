# round 5: tile order 6 (CU strips: co-resident workgroups on neighbouring tiles) -- the
# placement parity test, then the A/B against order 4 (views fill/default/diag, shaded and not,
# serial and 3 in flight, two rounds), the C3 bench with tile order 6 forced through the knob,
# and the gather counters of the headline kernel under order 6 (L1 hit rate, TD stall)
set -o pipefail
O=gpurun_out/r05_m10; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "placement or tile_order or work_placement" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_placement.log 2>&1; rc=$?; tail -2 $O/pytest_placement.log; [ $rc -eq 0 ] || exit 1
ORDERS=4,6 timeout -k 10 500 python -u tools/experiments/r05/order_ab.py 2 fill,default,diag > $O/order_ab.jsonl 2> $O/order_ab.err || exit 1
echo "order A/B done"
bash tools/pmc_passes.sh r05_m10/ta6 tools/pmc_sets_ta.txt --frames 10 --tile-order 6 || exit $?
python tools/gather_report.py gpurun_out/r05_m10/ta6 "F32H, true" > $O/gather_report_order6.json 2>&1; head -30 $O/gather_report_order6.json
