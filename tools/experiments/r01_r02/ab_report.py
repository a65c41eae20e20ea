"""Summarise tools/experiments/r01_r02/ab_multi.sh output: python tools/experiments/r01_r02/ab_report.py <dir> lib lib_a ..."""
import glob
import json
import os
import sys

d, libs = sys.argv[1], sys.argv[2:]
print("== bench C3: value (3 in flight) | serial | reference semantics")
for L in libs:
    for f in sorted(glob.glob(os.path.join(d, f"bench_{L}_[0-9].json"))):
        j = json.loads([l for l in open(f) if l.startswith("{")][0])
        v = j["variants"]
        print(f"{L:10s} {j['value']:8.1f} {v['serial_frames']['value']:8.1f} "
              f"{v['reference_semantics_no_shading_no_ert']['value']:8.1f}")
for kind in ("views", "views_shaded"):
    print(f"== {kind} kernel_ms: " + " ".join(libs))
    rows = {}
    for L in libs:
        for line in open(os.path.join(d, f"{kind}_{L}.txt")):
            if line.startswith("{") or "amdgpu.ids" in line or not line.strip():
                continue
            name, js = line.split(" ", 1)
            rows.setdefault(name, []).append(json.loads(js)["kernel_ms"])
    for name, vals in rows.items():
        print(f"{name:14s} " + " ".join(f"{x:.4f}" for x in vals))
