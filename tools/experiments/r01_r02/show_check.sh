#!/bin/bash
# Summarise a gpu_check.sh run (local side).
O=gpurun_out/$1
cat $O/rc.txt; tail -1 $O/tests.log
python3 -c "
import json; d=json.load(open('$O/bench.json'))
print('C3 value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'kernel_ms', d['roofline']['kernel_ms'])
print('ref-sem', d['variants'])" 2>/dev/null
for f in $O/views_*.txt; do echo "== $f"; grep -v '^{' $f | grep -v amdgpu.ids; done
