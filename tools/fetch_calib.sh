#!/bin/bash
# FETCH_SIZE calibration passes (tools/fetch_calib.hip, built by __graft_entry__.build into tools/bin).
O=gpurun_out/${1:-r02_calib}; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- tools/bin/fetch_calib > $O/fetch.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $O/rdreq -o run --output-format csv -- tools/bin/fetch_calib > $O/rdreq.log 2>&1
