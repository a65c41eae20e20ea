#!/bin/bash
# Headline bench at the driver's K=20/W=5 against longer timed regions, alternating on one box.
O=gpurun_out/r02_steps; mkdir -p $O
for r in 1 2; do for kw in "20 5" "50 10" "200 10"; do set -- $kw
  timeout -k 10 300 python bench.py --no-variants --no-cpu-baseline --steps $1 --warmup $2 > $O/b.json 2> $O/b.err || exit 1
  python -c "import json; d=json.load(open('$O/b.json')); print('$r', 'K=$1 W=$2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" | tee -a $O/out.txt
done; done
