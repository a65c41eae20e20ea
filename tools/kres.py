"""Kernel resource usage (VGPRs, occupancy, spills, LDS) from `make -C volumetric-renderer_amd asm`
(build/asm/resource-usage.txt), one line per kernel; optional substring filters.
Usage: python tools/kres.py [filter ...]"""
import re
import subprocess
import sys

path = "volumetric-renderer_amd/build/asm/resource-usage.txt"
if len(sys.argv) > 1 and sys.argv[1].endswith(".txt"):
    path = sys.argv.pop(1)
cur, rows = None, {}
for line in open(path):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:(?: \S+)?     ([^:]+): (\S+)", line)
    if m and cur:
        rows[cur][m.group(1)] = m.group(2)
names = list(rows)
dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
for n, d in zip(names, dem):
    if all(f in d for f in sys.argv[1:]) and rows[n].get("VGPRs"):
        r = rows[n]
        print(f"{r.get('VGPRs'):>4} vgpr {r.get('Occupancy [waves/SIMD]'):>2} waves "
              f"spill {r.get('VGPRs Spill')} scratch {r.get('ScratchSize [bytes/lane]')}  {d[:150]}")
