#!/bin/bash
# Cold-start ramp vs hardware queue count: ramp.py arms and the headline-first bench (--no-variants).
O=gpurun_out/${1:-r02_rampq}; mkdir -p $O
for r in 1 2; do for q in 4 8; do
  for arm in "20 5 0 1 4" "20 50 0 1 4"; do
    GPU_MAX_HW_QUEUES=$q RAMP_BURN=mm timeout -k 10 200 python -u tools/experiments/r01_r02/ramp.py $arm > $O/o.json 2>> $O/err.txt || exit 1
    python -c "import json; d=json.load(open('$O/o.json')); print('q=$q ramp', d['K'], d['W'], d['ms_per_step'])" | tee -a $O/out.txt
  done
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --no-variants --no-cpu-baseline --steps 20 --warmup 5 > $O/b.json 2>> $O/err.txt || exit 1
  python -c "import json; d=json.load(open('$O/b.json')); print('q=$q bench --no-variants K=20 W=5', d['value'], d['ms_per_step'])" | tee -a $O/out.txt
done; done
