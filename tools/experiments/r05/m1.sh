# round 5, first GPU call: the whole GPU suite on the current sources, then the round
# measurement (bench, rocprof kernel trace, FETCH_SIZE/WRITE_SIZE for every config).  Test
# failures (pytest status 1) do not stop the measurement; a crash, fault or time limit does.
set -o pipefail
O=gpurun_out/r05_suite; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
[ $rc -le 1 ] || exit $rc
bash tools/measure_round.sh r05_m1 "c3 c3_default c3_ref c2 c4 c5"
