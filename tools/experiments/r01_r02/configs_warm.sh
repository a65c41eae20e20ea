#!/bin/bash
# C2/C4/C5 bench lines with a long warm-up (the cold-device ramp), no CPU baseline.
O=gpurun_out/${1:-r02_configs_warm}; mkdir -p $O
for c in c2 c4 c5; do
  timeout -k 10 600 python bench.py --config $c --steps 100 --warmup 50 --no-cpu-baseline > $O/$c.json 2> $O/$c.err || exit 1
  python -c "import json; d=json.load(open('$O/$c.json')); r=d['roofline']; print('$c', d['value'], d['ms_per_step'], 'frac', r['frac'], 'serial', d['variants'].get('serial_frames',{}).get('ms_per_step'))" | tee -a $O/out.txt
done
