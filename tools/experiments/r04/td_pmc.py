"""Per-case PMC of td_mask (tools/experiments/r04/td_mask.hip): for each pass directory under
<dir>/p*/ (rocprofv3 --pmc ... -o run --output-format csv), the timed (last) dispatch of every
case's kernel, its counters divided by the wave-level loads of one launch.
Usage: python td_pmc.py <dir> <td_mask.json>  -> JSON on stdout"""
import csv
import glob
import json
import os
import re
import sys


def main():
    d, tj = sys.argv[1], sys.argv[2]
    cases = json.load(open(tj))
    loads = cases["wave_loads"]
    per = {}  # (width, stride, pattern) -> {counter: value of the last dispatch}
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        last = {}
        for r in csv.DictReader(open(f)):
            m = re.search(r"td_kernel<(\d+), (\d+), (\d+)>", r["Kernel_Name"])
            if not m:
                continue
            key = tuple(int(x) for x in m.groups())
            did = int(r.get("Dispatch_Id", 0) or 0)
            slot = last.setdefault((key, r["Counter_Name"]), [-1, 0.0])
            if did > slot[0]:
                slot[0], slot[1] = did, 0.0
            if did == slot[0]:
                slot[1] += float(r["Counter_Value"])
        for (key, name), (_, v) in last.items():
            per.setdefault(key, {})[name] = v
    out = []
    for c in cases["cases"]:
        key = (c["width"], c["stride"], c["pattern"])
        ctr = per.get(key, {})
        e = dict(c)
        for name, v in sorted(ctr.items()):
            e[name + "_per_wave_load"] = round(v / loads, 4) if "BUSY" not in name and "STALL" not in name else v
        out.append(e)
    json.dump({"wave_loads": loads, "cases": out}, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
