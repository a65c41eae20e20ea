#!/bin/bash
# Fresh-process arms of tools/experiments/r01_r02/ramp.py (K W preburn timing tile_order), alternating, two rounds.
O=gpurun_out/${1:-r02_ramp5}; mkdir -p $O
for r in 1 2; do
  for arm in "mm 0 20 5 0 1 4" "march1 0 20 5 300 1 4" "march3 0 20 5 300 1 4" "mm 0 20 50 0 1 4" "mm 100 20 50 0 1 4" "mm 1000 20 50 0 1 4"; do
    set -- $arm; B=$1; S=$2; shift 2
    RAMP_SLEEP=$S RAMP_BURN=$B timeout -k 10 200 python -u tools/experiments/r01_r02/ramp.py "$@" >> $O/out.jsonl 2>> $O/err.txt || exit 1
  done
done
