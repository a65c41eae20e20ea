# round 5, first GPU call: the whole GPU suite on the round-4 sources, then the round
# measurement (bench, rocprof kernel trace, FETCH_SIZE/WRITE_SIZE for every config)
set -o pipefail
O=gpurun_out/r05_suite; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/measure_round.sh r05_m1 "c3 c3_default c3_ref c2 c4 c5"
