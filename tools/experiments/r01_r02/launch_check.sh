# bench.py under torch.distributed.run: N=1, and an N=2 gloo rehearsal on the one GPU
set -o pipefail
O=gpurun_out/launch; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 5 > $O/n1.json 2> $O/n1.err &&
VR_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline > $O/n2_gloo.json 2> $O/n2_gloo.err
