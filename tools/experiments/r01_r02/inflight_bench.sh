#!/bin/bash
# C3 bench line with 2, 3, 4 frames in flight (alternating, 2 rounds).  GPU box.
O=gpurun_out/r02_fif; mkdir -p $O
for r in 1 2; do for f in 2 3 4; do
  timeout -k 10 300 python bench.py --no-variants --no-cpu-baseline --steps 100 --frames-in-flight $f > $O/b.json 2> $O/b.err || exit 1
  python -c "import json; d=json.load(open('$O/b.json')); print('$r', 'fif=$f', d['value'], d['ms_per_step'])" | tee -a $O/out.txt
done; done
