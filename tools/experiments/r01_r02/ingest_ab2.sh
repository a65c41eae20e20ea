# per-brick workgroup brick/grad-field kernels (this build) vs per-element (lib_old)
set -o pipefail
O=gpurun_out/ingest2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 &&
VR_AMD_LIB=$PWD/volumetric-renderer_amd/lib_old/libvr_amd.so timeout -k 10 300 python tools/ingest_bench.py > $O/ingest_old.txt 2>&1 &&
timeout -k 10 300 python tools/ingest_bench.py > $O/ingest_new.txt 2>&1
