# HBM read traffic of the u8 configurations (C2 view of C4 geometry, C4): FETCH_SIZE passes
set -o pipefail
O=gpurun_out/pmc_u8; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/prof_run.py --n 1024 --dtype uint8 --size 2048x2048 --shading 0 --ert 0 --frames 10 > $O/c4_time.json 2> $O/c4_time.err &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/c4_fetch -o run --output-format csv -- python3 tools/prof_run.py --n 1024 --dtype uint8 --size 2048x2048 --shading 0 --ert 0 --frames 10 > $O/c4_fetch.log 2>&1 &&
timeout -k 10 120 python3 tools/prof_run.py --n 256 --dtype uint8 --size 1024x1024 --shading 0 --ert 0 --frames 10 > $O/c2_time.json 2> $O/c2_time.err &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/c2_fetch -o run --output-format csv -- python3 tools/prof_run.py --n 256 --dtype uint8 --size 1024x1024 --shading 0 --ert 0 --frames 10 > $O/c2_fetch.log 2>&1
