"""Where the fixed cost of a short timed region goes (K=20 W=5 vs K=200): one arm per fresh
process, C3, 3 frames in flight; per-frame end times relative to the start of the timed region.
  python tools/experiments/r01_r02/ramp.py K W [preburn_ms] [timing]
preburn_ms > 0: keep the GPU busy with a torch matmul loop that long before the warm-up (clock
ramp test); timing=1: the library's per-launch HIP event timing on, as bench.py runs it."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from bench import synth, vr_amd, vr_dist  # noqa: E402
import torch  # noqa: E402


def main():
    K, W = int(sys.argv[1]), int(sys.argv[2])
    preburn = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
    timing = len(sys.argv) > 4 and sys.argv[4] == "1"
    order = int(sys.argv[5]) if len(sys.argv) > 5 else 4
    torch.cuda.set_device(0)
    cfg = bench.CONFIGS["c3"]
    rp = bench.setup_pass(cfg, 0)
    inflight = 3
    cam = synth.camera(cfg["cam"]).to_vr_camera()
    p = vr_amd.default_params(shading=cfg["shading"], ert_eps=cfg["ert"], frames_in_flight=inflight)
    p.tile_order = order
    H, Wd = cfg["H"], cfg["W"]
    slots = [vr_dist.Slot(torch.empty((H + 16, Wd), dtype=torch.int32, device="cuda"), None, None,
                          torch.cuda.Stream()) for _ in range(inflight)]
    pipe = vr_dist.FramePipeline(
        slots, 0, 1, None,
        render=lambda sl: rp.render_device(cam, p, sl.shard.data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1,
                                           sl.stream.cuda_stream),
        assemble=None)
    burn = os.environ.get("RAMP_BURN", "mm")
    if preburn and burn == "mem":  # HBM-bound: 1 GiB copies
        a = torch.empty(1 << 28, device="cuda")
        b = torch.empty_like(a)
        torch.cuda.synchronize()
        t = time.perf_counter()
        while (time.perf_counter() - t) * 1e3 < preburn:
            for _ in range(4):
                b.copy_(a)
            torch.cuda.synchronize()
        del a, b
    elif preburn and burn == "march1":  # serial frames on one stream, no host waits between
        t = time.perf_counter()
        while (time.perf_counter() - t) * 1e3 < preburn:
            for _ in range(20):
                rp.render_device(cam, p, slots[0].shard.data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1,
                                 torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
    elif preburn and burn == "march3":  # the pipelined frames themselves (= a longer warm-up)
        t = time.perf_counter()
        while (time.perf_counter() - t) * 1e3 < preburn:
            for _ in range(30):
                pipe.step()
            torch.cuda.synchronize()
    elif preburn and burn == "march":  # the march itself, serial frames, before the warm-up
        t = time.perf_counter()
        while (time.perf_counter() - t) * 1e3 < preburn:
            rp.render_device(cam, p, slots[0].shard.data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1,
                             torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
    elif preburn:
        a = torch.randn(4096, 4096, device="cuda")
        torch.cuda.synchronize()
        t = time.perf_counter()
        while (time.perf_counter() - t) * 1e3 < preburn:
            for _ in range(8):
                a = torch.tanh(a @ a * 1e-3)
            torch.cuda.synchronize()
    for _ in range(W):
        pipe.step()
    torch.cuda.synchronize()
    if os.environ.get("RAMP_SLEEP"):
        time.sleep(float(os.environ["RAMP_SLEEP"]) / 1e3)
    rp.timing_reset()
    rp.timing_enable(timing)
    torch.cuda.synchronize()
    start = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    start.record(torch.cuda.current_stream())
    for sl in slots:
        sl.stream.wait_event(start)
    ends = []
    for k in range(K):
        sl = slots[pipe.k % inflight]
        pipe.step()
        e = torch.cuda.Event(enable_timing=True)
        e.record(sl.stream)
        ends.append(e)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    rp.timing_enable(False)
    kms, nl = rp.timing_read()
    fin = [round(start.elapsed_time(e), 3) for e in ends]
    print(json.dumps(dict(K=K, W=W, preburn_ms=preburn, burn=burn, sleep=os.environ.get('RAMP_SLEEP'), timing=timing, order=order,
                          ms_per_step=round((t1 - t0) * 1e3 / K, 4), frame_end_ms=fin,
                          kernel_ms=round(kms / max(nl, 1), 4))), flush=True)


if __name__ == "__main__":
    main()
