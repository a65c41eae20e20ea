set -o pipefail
O=gpurun_out/r04_e1c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 ./tools/experiments/r04/td_mask > $O/td_mask.json 2>&1 && cat $O/td_mask.json
VR_AMD_LIB=$PWD/volumetric-renderer_amd/lib_wgt/libvr_amd.so timeout -k 10 300 python -u tools/experiments/r04/default_timeline.py $O/timeline > $O/timeline.log 2>&1 && cat $O/timeline.log | cut -c1-600
timeout -k 10 600 python -u tools/experiments/r04/queue_ab.py 2 default,fill,diag > $O/queue_ab.jsonl 2> $O/queue_ab.err && cat $O/queue_ab.jsonl
