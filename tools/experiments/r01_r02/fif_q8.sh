#!/bin/bash
# Frames in flight under 8 hardware queues (bench.py raises GPU_MAX_HW_QUEUES), driver flags, alternating.
O=gpurun_out/${1:-r02_fif_q8}; mkdir -p $O
for r in 1 2 3; do for f in 3 4 5 2; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --frames-in-flight $f > $O/b.json 2>> $O/err || exit 1
  python -c "import json; d=json.load(open('$O/b.json')); v=d['variants']; print('$r fif=$f', d['value'], d['ms_per_step'], 'default', v['default_camera']['ms_per_step'], 'ref', v['reference_semantics_no_shading_no_ert']['ms_per_step'], 'skip', v['c3_skip_empty']['ms_per_step'])" | tee -a $O/out.txt
done; done
