# round 5, measurement of the pruned sources: the GPU suite (verbose), the round measurement
# (bench + rocprofv3 kernel trace + FETCH_SIZE/WRITE_SIZE for every config), the one-GPU
# rehearsal of the multi-device path under bench.py (2, 3 and 8 members on device 0, copy
# exchange), and unprofiled bench lines of C2/C4/C5.
set -o pipefail
O=gpurun_out/r05_m5; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -le 1 ] || exit $rc
bash tools/measure_round.sh r05_final "c3 c3_default c3_ref c2 c4 c5" || exit $?
for m in 2 3 8; do
  timeout -k 10 200 python -u bench.py --members-on-one-gpu $m --no-variants --no-cpu-baseline --steps 40 --warmup 10 > $O/bench_members$m.json 2> $O/bench_members$m.err || exit 1
  python -c "import json; d=json.load(open('$O/bench_members$m.json')); print('members', $m, d['value'], d['ms_per_step'], d['frame_check'], [ (r['rank'], r['kernel_ms'], r['render_span_ms'], r['gather_span_ms']) for r in d['per_rank']])"
done
for cfg in c2 c4 c5; do
  timeout -k 10 300 python -u bench.py --config $cfg --no-variants --no-cpu-baseline --steps 100 --warmup 20 > $O/bench_$cfg.json 2> $O/bench_$cfg.err || exit 1
  python -c "import json; d=json.load(open('$O/bench_$cfg.json')); print('$cfg', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic_status'])"
done
