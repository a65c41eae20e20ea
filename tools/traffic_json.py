"""Turn tools/measure_round.sh PMC passes into profiles/pmc_traffic.json (read by bench.py).

HBM bytes per launch of the timed march kernel = 2 x FETCH_SIZE x 1024 (gfx950: FETCH_SIZE
reads 1/2 of the bytes of 128-B requests, MI355X_MICROARCH.md §HBM) + WRITE_SIZE x 1024.
Usage: python tools/traffic_json.py gpurun_out/<tag> [out.json]
"""
import csv
import glob
import json
import os
import sys


def mean_counter(d, name):
    vals = []
    for f in glob.glob(os.path.join(d, "run_counter_collection.csv")) + glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "march_kernel<" in k:
                targs = [t.strip() for t in k.split("march_kernel<", 1)[1].split(">", 1)[0].split(",")]
                if targs[2] == "true":  # <VT, SHADE, COUNT, SKIP>: the counting kernel is not timed
                    continue
                if r["Counter_Name"] == name:
                    vals.append(float(r["Counter_Value"]))
    return sum(vals) / len(vals) if vals else None


def main():
    src = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_traffic.json"
    res = {}
    for cfg in ("c3", "c3_ref"):
        f = mean_counter(os.path.join(src, f"pmc_{cfg}_FETCH_SIZE"), "FETCH_SIZE")
        w = mean_counter(os.path.join(src, f"pmc_{cfg}_WRITE_SIZE"), "WRITE_SIZE")
        if f is None:
            continue
        res[cfg] = dict(n_gpus=1, fetch_size_kb=f, write_size_kb=w,
                        hbm_bytes_per_launch=2 * f * 1024 + (w or 0) * 1024,
                        method="rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate runs of "
                               "tools/prof_run.py (10 frames), mean over dispatches of the timed "
                               "march kernel; FETCH_SIZE x2 gfx950 correction",
                        source=src)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
