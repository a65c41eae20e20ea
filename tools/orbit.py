"""The bench's orbit variant alone (bench.orbit: the reference's camera drag, default memory
budget) on the C3 volume, printed as JSON; --budget unlimited|default|<bytes>.
    python tools/orbit.py [--frames 360] [--budget default]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=360)
    ap.add_argument("--budget", default="default")
    ap.add_argument("--config", default="c3")
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    rp = bench.setup_pass(cfg, 0)
    if a.budget != "default":
        bench.BUDGET_DEFAULT = (2 ** 64 - 1) if a.budget == "unlimited" else int(a.budget)
    frame = torch.empty((cfg["H"], cfg["W"]), dtype=torch.int32, device="cuda")
    out = bench.orbit(rp, cfg, frame.data_ptr(), a.frames)
    out["budget"] = a.budget
    print(json.dumps(out))
    rp.close()


if __name__ == "__main__":
    main()
