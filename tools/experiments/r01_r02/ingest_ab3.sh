set -o pipefail
O=gpurun_out/ingest3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 &&
VR_AMD_LIB=$PWD/volumetric-renderer_amd/lib_old/libvr_amd.so timeout -k 10 300 python tools/ingest_bench.py > $O/ingest_old.txt 2>&1 &&
timeout -k 10 300 python tools/ingest_bench.py > $O/ingest_new.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 tools/ingest_bench.py --reps 2 > $O/trace.log 2>&1
