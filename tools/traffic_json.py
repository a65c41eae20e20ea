"""Turn tools/measure_round.sh PMC passes into profiles/pmc_traffic.json (read by bench.py).

HBM bytes per frame launch of the timed march kernel = 2 x FETCH_SIZE x 1024 (gfx950:
FETCH_SIZE reads 1/2 of the bytes of 128-B requests, MI355X_MICROARCH.md §HBM) + WRITE_SIZE x
1024, averaged over the dispatches of the configuration's frame kernel (the counting kernel
that bench.py launches once for its work counters is excluded).  The passes run bench.py
itself (--config X --no-variants), so the launches are the benchmark's own.
Usage: python tools/traffic_json.py gpurun_out/<tag> [out.json]
"""
import collections
import csv
import glob
import json
import os
import sys

def template_args(name, head):
    """Top-level template arguments of the first `head<...>` in a demangled kernel name
    (nested <> kept whole: "march_kernel<vr::Quad8<unsigned char>, false, ...>")."""
    s = name.split(head, 1)[1]
    args, depth, cur = [], 0, ""
    for ch in s:
        if ch == "<":
            depth += 1
        elif ch == ">":
            if depth == 0:
                break
            depth -= 1
        if ch == "," and depth == 0:
            args.append(cur.strip())
            cur = ""
        else:
            cur += ch
    args.append(cur.strip())
    return args


CONFIGS = ("c3", "c3_ref", "c3_default", "c2", "c4", "c5")


def frame_kernel(name):
    """True for a march launch that renders a frame (not the COUNT instantiation)."""
    for k in ("march_kernel<", "march_pair_kernel<", "march_lds_kernel<"):
        if k in name:
            targs = template_args(name, k)
            return not (k == "march_kernel<" and targs[2] == "true")  # <VT, SHADE, COUNT, ...>
    return False


def counter(d, name):
    vals, kernels = [], collections.Counter()
    for f in glob.glob(os.path.join(d, "run_counter_collection.csv")) + glob.glob(
            os.path.join(d, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if frame_kernel(r["Kernel_Name"]) and r["Counter_Name"] == name:
                vals.append(float(r["Counter_Value"]))
                kernels[r["Kernel_Name"]] += 1
    if not vals:
        return None, None, 0
    return sum(vals) / len(vals), kernels.most_common(1)[0][0], len(vals)


def bench_line(log):
    """The bench.py JSON line in a pass's log (stdout of the profiled bench.py run)."""
    if not os.path.exists(log):
        return None
    for line in open(log, errors="replace"):
        if line.startswith('{"metric"'):
            return json.loads(line)
    return None


def main():
    src = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_traffic.json"
    res = json.load(open(out)) if os.path.exists(out) else {}
    for cfg in CONFIGS:
        f, kern, n = counter(os.path.join(src, f"pmc_{cfg}_FETCH_SIZE"), "FETCH_SIZE")
        w, _, _ = counter(os.path.join(src, f"pmc_{cfg}_WRITE_SIZE"), "WRITE_SIZE")
        if f is None:
            continue
        # the key bench.py checks before using the entry: the kernel sources and volume layout
        # the profiled run reported (its own JSON line)
        b = bench_line(os.path.join(src, f"pmc_{cfg}_FETCH_SIZE.log")) or {}
        rf = b.get("roofline", {})
        if rf.get("kernel") and rf["kernel"] != kern:
            print(f"{cfg}: profiled kernel {kern} != bench's {rf['kernel']}", file=sys.stderr)
        res[cfg] = dict(n_gpus=1, kernel=kern, code_hash=rf.get("kernel_code_hash"),
                        layout=rf.get("volume_layout"), dispatches=n, fetch_size_kb=f, write_size_kb=w,
                        hbm_bytes_per_launch=2 * f * 1024 + (w or 0) * 1024,
                        method="rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate runs of "
                               f"bench.py --config {cfg} --no-variants, mean over the frame "
                               "kernel's dispatches; FETCH_SIZE x2 gfx950 correction",
                        source=os.path.relpath(src, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
                        if os.path.isabs(src) else src)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
