#!/bin/bash
# bench.py A/B (two bench scripts at the repo root), driver flags, alternating, 3 rounds.
A=$1; B=$2; O=gpurun_out/${3:-r02_benchab}; mkdir -p $O
for r in 1 2 3; do for S in $A $B; do
  timeout -k 10 400 python $S --steps 20 --warmup 5 --no-cpu-baseline > $O/b.json 2>> $O/err || exit 1
  python - $O/b.json $r $S <<'PY' | tee -a $O/out.txt
import json, sys
d = json.load(open(sys.argv[1])); v = d["variants"]
print(sys.argv[2], sys.argv[3].ljust(14), "C3", d["value"], d["ms_per_step"], "serial", v["serial_frames"]["ms_per_step"],
      "default", v["default_camera"]["ms_per_step"], "ref", v["reference_semantics_no_shading_no_ert"]["ms_per_step"],
      "skip", v["c3_skip_empty"]["ms_per_step"])
PY
done; done
