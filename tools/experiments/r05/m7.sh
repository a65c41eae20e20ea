# round 5: the final headline kernel's gather-pipeline counters (TA / TCP / TD / SQ, one
# rocprofv3 --pmc pass per group: tools/pmc_sets_ta.txt) on the C3 frame (serial frames,
# tools/prof_run.py), and the one-process-per-GPU bench path rehearsed with two gloo ranks on
# the one GPU (VR_DIST_BACKEND=gloo, host-staged gathers: frame_check of the assembled frame)
set -o pipefail
O=gpurun_out/r05_m7; mkdir -p $O
export TMPDIR=/tmp
bash tools/pmc_passes.sh r05_m7/ta tools/pmc_sets_ta.txt --frames 10 || exit $?
python tools/gather_report.py gpurun_out/r05_m7/ta "F32H, true" > $O/gather_report.json 2>&1; head -40 $O/gather_report.json
VR_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-variants --no-cpu-baseline > $O/bench_gloo2.json 2> $O/bench_gloo2.err || exit 1
python -c "import json; d=json.load(open('$O/bench_gloo2.json')); print('gloo x2', d['n_gpus'], d['value'], d['frame_check'], d['config']['parallelism'])"
