# parallel raw read + chunked min/max (lib) vs serial (lib_old): ingest bench
set -o pipefail
O=gpurun_out/ingest4; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/ingest_bench.py > $O/ingest_new.txt 2>&1 &&
VR_AMD_LIB=$PWD/volumetric-renderer_amd/lib_old/libvr_amd.so timeout -k 10 300 python tools/ingest_bench.py > $O/ingest_old.txt 2>&1
