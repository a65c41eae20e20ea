"""Does what ran before change a variant's time?  python tools/experiments/r01_r02/seq.py <pre> ; pre in
none | fill1 (one shaded fill frame: builds the difference field) | serial (bench's serial
variant) | fillpipe (40+20 pipelined fill frames).  Then the default-camera variant as bench
runs it (K=20 after 40 warm-up frames), twice."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402

pre = sys.argv[1]
torch.cuda.set_device(0)
cfg = bench.CONFIGS["c3"]
rp = bench.setup_pass(cfg, 0)
if pre == "fill1":
    bench.run_variant(rp, cfg, 1, 0, 0, 1, 1)
elif pre == "serial":
    bench.run_variant(rp, cfg, 10, 5, 0, 1, 1)
elif pre == "fillpipe":
    bench.run_variant(rp, cfg, 20, 40, 0, 1, 3)
out = []
for _ in range(2):
    V = bench.run_variant(rp, bench.CONFIGS["c3_default"], 20, 40, 0, 1, 3)
    out.append(round(V["secs"] / 20 * 1e3, 4))
print(json.dumps(dict(pre=pre, default_ms=out, kernel=rp.kernel_name(
    bench.vr_amd.default_params(shading=1)))), flush=True)
