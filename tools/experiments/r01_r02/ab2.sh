# unshaded full-frame march: single-lane vs pipelined (VR_PIPELINE) over the sweep views
set -o pipefail
O=gpurun_out/ab2; mkdir -p $O
V="timeout -k 10 200 python tools/view_sweep.py"
VR_PIPELINE=0 $V > $O/f32_nopipe.txt 2>&1 &&
VR_PIPELINE=1 $V > $O/f32_pipe.txt 2>&1 &&
VR_PIPELINE=0 $V --dtype uint8 --n 256 --size 1024x1024 > $O/u8_nopipe.txt 2>&1 &&
VR_PIPELINE=1 $V --dtype uint8 --n 256 --size 1024x1024 > $O/u8_pipe.txt 2>&1 &&
VR_PIPELINE=0 $V --dtype uint8 --n 1024 --size 2048x2048 > $O/u8big_nopipe.txt 2>&1 &&
VR_PIPELINE=1 $V --dtype uint8 --n 1024 --size 2048x2048 > $O/u8big_pipe.txt 2>&1
