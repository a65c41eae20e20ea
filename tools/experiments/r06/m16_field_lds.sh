#!/bin/bash
# Round 6: the difference-field build staged through LDS -- the tests whose frames read the field
# (bit-exact against the oracle), then the build's duration under rocprofv3 (kernel trace).
set -o pipefail
O=gpurun_out/m16
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_round4.py tests/test_gpu_round6.py tests/test_gpu_inputs.py \
    "tests/test_gpu_fullsize.py::test_c3_512_f32_1080p_whole_frame" > $O/pytest.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/trace.log 2>&1
