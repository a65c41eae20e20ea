# parity + bench + unshaded single-lane/pipelined view sweeps of the current build
set -o pipefail
O=gpurun_out/ab3; mkdir -p $O
V="timeout -k 10 200 python tools/view_sweep.py"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err &&
$V --shading 1 --ert 1e-5 > $O/f32_shaded.txt 2>&1 &&
VR_PIPELINE=0 $V > $O/f32_nopipe.txt 2>&1 &&
VR_PIPELINE=1 $V > $O/f32_pipe.txt 2>&1 &&
VR_PIPELINE=0 $V --dtype uint8 --n 256 --size 1024x1024 > $O/u8_nopipe.txt 2>&1 &&
VR_PIPELINE=1 $V --dtype uint8 --n 256 --size 1024x1024 > $O/u8_pipe.txt 2>&1
