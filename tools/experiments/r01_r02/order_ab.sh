#!/bin/bash
# Default tile order A/B on the full bench (variants first, headline last), alternating.
O=gpurun_out/${1:-r02_order}; mkdir -p $O
for r in 1 2; do for T in 4 1 3; do
  VR_TILE_ORDER_DEFAULT=$T timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/b$T.json 2> $O/b.err || exit 1
  python - $O/b$T.json $r $T <<'PY' | tee -a $O/out.txt
import json, sys
d = json.load(open(sys.argv[1])); v = d["variants"]
print(sys.argv[2], "order", sys.argv[3], "C3", d["value"], d["ms_per_step"], "serial", v["serial_frames"]["ms_per_step"],
      "default", v["default_camera"]["ms_per_step"], "ref", v["reference_semantics_no_shading_no_ert"]["ms_per_step"],
      "skip", v["c3_skip_empty"]["ms_per_step"])
PY
done; done
