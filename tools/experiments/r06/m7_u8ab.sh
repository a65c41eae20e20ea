#!/bin/bash
# round 6, VERDICT r5 item 4: the u8 march at C4 (1024^3 u8 @ 2048^2, fill view, reference
# semantics as bench.py's c4) in the plain 7x8x8 layout (policy) against yz-quads (one 8-B load
# per sample): gather-path counters (TD/TA/TCP/SQ) and DRAM bytes, one rocprofv3 pass per group
set -u
cd "$GRAFT_REPO_ROOT"
ARGS="--n 1024 --dtype uint8 --size 2048x2048 --cam fill --shading 0 --ert 0 --frames 10"
for L in 0 1; do
  PASS_TIMEOUT=120 bash tools/pmc_passes.sh r06/u8ab/layout$L tools/pmc_sets_u8ab.txt $ARGS --knob u8_layout=$L
  rc=$?; [ $rc -ne 0 ] && exit $rc
done
for L in 0 1; do
  python tools/pmc_report.py gpurun_out/r06/u8ab/layout$L march_kernel > gpurun_out/r06/u8ab/report_layout$L.json
  python tools/gather_report.py gpurun_out/r06/u8ab/layout$L march_kernel > gpurun_out/r06/u8ab/gather_layout$L.json || true
done
