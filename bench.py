"""Benchmark of the MI355X ray-march (BASELINE.json metric: Gsamples/s + fps, 512^3 NRRD @ 1080p;
achieved HBM GB/s vs peak).

A step = one frame of the hot path: every rank ray-marches its row blocks of the 1920x1080
frame (HIP kernel through the C ABI) and, for N > 1, the row shards are gathered to rank 0
over RCCL (torch.distributed "nccl") and assembled there.  The volume is resident in HBM
before timing starts (generated on device); timing brackets exactly K steps with a barrier +
device synchronize on both sides and takes the max over ranks.

Workload (configs[2] of BASELINE.json, the configuration the metric is quoted on):
  512^3 f32 synthetic volume (sum of 32 Gaussians + 0.05 value noise, seed 2024),
  1920x1080, camera r = 1.6 (frame-filling), TF-2 (demo ramp), gradient Phong shading +
  early-ray termination (eps 1e-5).  The reference-semantics variant (no shading, no ERT) is
  timed as well and reported under "variants".

Usage: python bench.py [--gpus N] [--steps K] [--warmup W].
  N > 1 under torch.distributed.run (WORLD_SIZE set): one process per GPU, the library's RCCL
        frame path (vr_dist.h); WORLD_SIZE must equal N.
  N > 1 without WORLD_SIZE: bench.py starts `python -m torch.distributed.run --nproc-per-node N
        --master-addr 127.0.0.1` on itself as a child process, before anything touches the GPU,
        and exits with its status (the per-process RCCL path INTEGRATION.md recommends).
        --multi-device-context instead drives the N devices from ONE process through
        vr_create_mask (the drop-in boundary's own multi-GPU form).
  --members-on-one-gpu M (rehearsal): one process, a multi-device context of M members all on
        device 0 (vr_debug_create_members, copy exchange): the multi-device machinery on one GPU.
  Either way a run that cannot use exactly N GPUs fails (exit 2) naming what is missing.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for sub in ("volumetric-renderer_amd", "tools", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, sub))

# Hardware queues: the process's environment is used as it is (HIP's default and the GPU
# boxes' setting is 4) and recorded in the JSON line.  `--hw-queues Q` sets GPU_MAX_HW_QUEUES
# for this process before the HIP runtime starts (an explicit experiment; never the default).
def _early_flag(name):
    for i, a in enumerate(sys.argv):
        if a == name and i + 1 < len(sys.argv):
            return sys.argv[i + 1]
        if a.startswith(name + "="):
            return a.split("=", 1)[1]
    return None


if _early_flag("--hw-queues") is not None:
    os.environ["GPU_MAX_HW_QUEUES"] = str(int(_early_flag("--hw-queues")))
HW_QUEUES = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import synth  # noqa: E402
import vr_amd  # noqa: E402
import vr_dist  # noqa: E402

BACKEND = "nccl"
GATHER = "native"  # N > 1 over RCCL: "native" (vr_dist.h) or "torch" (torch.distributed.gather)
# Every timed run (the headline and each variant) warms up for max(--warmup, STEADY_WARMUP)
# frames right before its timed region: a device idle for >= 100 ms renders its first ~50
# pipelined frames 10-15% slower (profiles/r02/warm_state/), so a fixed warm-up makes each
# number independent of what ran before it.  The frames actually run are recorded.
STEADY_WARMUP = 120
BUDGET_DEFAULT = 2 ** 64 - 2  # vr.h VR_MEMORY_BUDGET_DEFAULT (ABI 8; 5x the bricks since ABI 9)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "Gsamples/sec + fps, 512³ NRRD @ 1080p; achieved HBM GB/s vs peak"

CONFIGS = {
    # name: volume dims, dtype, viewport, camera, tf, shading, ert
    "c3": dict(dims=(512, 512, 512), dtype=np.float32, W=1920, H=1080, cam="fill", tf="tf2",
               shading=1, ert=1e-5, seed=2024,
               workload="C3: 512^3 f32 synthetic NRRD-equivalent volume, 1920x1080, "
                        "gradient Phong + early-ray termination, camera r=1.6"),
    "c3_ref": dict(dims=(512, 512, 512), dtype=np.float32, W=1920, H=1080, cam="fill", tf="tf2",
                   shading=0, ert=0.0, seed=2024,
                   workload="C3 reference semantics: no shading, no ERT (volume.frag as written)"),
    # benchmarks use r=1.6 (frame-filling) plus the reference's default camera
    # (camera.cpp:7-13: r=3, 17% of the 1080p frame covered)
    "c3_default": dict(dims=(512, 512, 512), dtype=np.float32, W=1920, H=1080, cam="default",
                       tf="tf2", shading=1, ert=1e-5, seed=2024,
                       workload="C3 at the reference's default camera (r=3), gradient Phong + ERT"),
    "c2": dict(dims=(256, 256, 256), dtype=np.uint8, W=1024, H=1024, cam="fill", tf="tf2",
               shading=0, ert=0.0, seed=1234, source="ct_head",
               workload="C2: 256^3 u8 synthetic CT head, 1024x1024, trilinear + 1D TF"),
    "c4": dict(dims=(1024, 1024, 1024), dtype=np.uint8, W=2048, H=2048, cam="fill", tf="tf2",
               shading=0, ert=0.0, seed=7, workload="C4: 1024^3 u8, 2048x2048"),
    "c1": dict(dims=(64, 64, 64), dtype=np.float32, W=256, H=256, cam="fill", tf="tf2",
               shading=0, ert=0.0, seed=1, workload="C1: 64^3 f32, 256x256 (the CPU plumbing case)"),
    "c5": dict(dims=(2048, 2048, 2048), dtype=np.uint8, W=4096, H=4096, cam="fill", tf="tf2",
               shading=0, ert=0.0, seed=11,
               workload="C5: 2048^3 u8 bricked (plain 7x8x8-cell bricks, 12.4 GB resident in HBM), "
                        "4096x4096"),
}


def algorithmic_bytes(stats, voxel_bytes, pixels, out_bytes=4):
    """8 x sizeof(voxel) per executed density sample, + 48 x sizeof(voxel) per
    shaded sample (6 extra trilinear footprints), + 4 B per written pixel."""
    return (stats["samples"] * 8 * voxel_bytes + stats["shaded_samples"] * 48 * voxel_bytes
            + pixels * out_bytes)


def setup_pass(cfg, device, device_mask=None, members=None):
    rp = vr_amd.OffscreenPass(cfg["W"], cfg["H"], device=device, device_mask=device_mask,
                              members=members)
    if cfg.get("source") == "ct_head":
        # host-generated u8 CT head through the Dataset path (volume_dataset_changed)
        rp.volume_dataset_changed(synth.dataset(synth.ct_head(cfg["dims"][0], cfg["seed"])))
    else:
        rp.generate_volume(cfg["dims"], cfg["dtype"], seed=cfg["seed"])
    rp.transfer_function_changed(synth.TFS[cfg["tf"]]())
    return rp


_DIST = {}


def set_gather(kind):
    global GATHER
    GATHER = kind


def _all_ok(ok: bool) -> bool:
    """True on every rank iff `ok` holds on every rank (one MIN all-reduce)."""
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device="cuda")
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return bool(flag.item())


def dist_frames(rp, rank, world, row_block, inflight):
    """One RCCL communicator per frames-in-flight setting (vr_dist_create), id from rank 0
    broadcast over the torch.distributed process group.  Every rank checks that RCCL loads
    and that its communicator came up, and the ranks agree on both, so a failure on any rank
    sends all of them to the torch.distributed path together (never a rank left waiting in a
    collective the others skipped)."""
    key = (row_block, inflight)
    if key not in _DIST:
        err = None
        try:
            uid = vr_amd.dist_unique_id()  # every rank: proves RCCL loads here
        except RuntimeError as e:
            uid, err = bytes(vr_amd.DIST_ID_BYTES), e
        if not _all_ok(err is None):
            raise RuntimeError(f"RCCL unavailable on some rank ({err or 'another rank'})")
        t = torch.tensor(list(uid), dtype=torch.uint8, device="cuda")
        dist.broadcast(t, 0)
        df = None
        try:
            df = vr_amd.DistFrames(rp, bytes(t.cpu().tolist()), world, rank, row_block, inflight)
        except RuntimeError as e:
            err = e
        if not _all_ok(df is not None):
            if df is not None:
                df.close()
            raise RuntimeError(f"vr_dist_create failed on some rank ({err or 'another rank'})")
        _DIST[key] = df
    return _DIST[key]


class NativeFrames:
    """FramePipeline's interface over vr_amd.DistFrames (include/vr/vr_dist.h)."""

    def __init__(self, frames, cam, p, rank, H, W):
        self.frames, self.cam, self.p, self.rank = frames, cam, p, rank
        self.stream = torch.cuda.Stream()
        self.last = vr_dist.Slot(None, frame=torch.empty((H, W), dtype=torch.int32, device="cuda")
                                 if rank == 0 else None)

    def step(self):
        self.frames.render(self.cam, self.p, self.last.frame.data_ptr() if self.rank == 0 else 0,
                           self.stream.cuda_stream)

    def drain(self):
        self.frames.synchronize()
        self.stream.synchronize()


class GroupFrames:
    """Frames of a multi-device context (vr_create_mask): each vr_render_device call renders
    the whole frame across the context's devices into one frame buffer on the caller's stream
    (the library keeps `frames_in_flight` frames in flight across the devices)."""

    def __init__(self, rp, cam, p, H, W):
        self.rp, self.cam, self.p = rp, cam, p
        self.stream = torch.cuda.Stream()
        self.last = vr_dist.Slot(None, frame=torch.empty((H, W), dtype=torch.int32, device="cuda"))

    def step(self):
        self.rp.render_device(self.cam, self.p, self.last.frame.data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1,
                              self.stream.cuda_stream)

    def drain(self):
        self.stream.synchronize()


def run_variant(rp, cfg, steps, warmup, rank, world, inflight, row_block=8, group=False):
    """Time `steps` frames; returns a dict: secs (max over ranks), kms (this rank's average
    kernel ms), frame (frame work counters), mine (this rank's), shard_px, check (N > 1:
    assembled frame == single-rank frame) and per_rank timings.  For N > 1 a frame is: render
    this rank's row blocks -> RCCL gather to rank 0 -> de-interleave on rank 0.  `inflight`
    frames are in flight (vr_dist.FramePipeline): frame i's work goes to stream i mod
    inflight, so consecutive frames overlap on the device and a frame's gather overlaps the
    next frames' renders; inflight = 1 is the serial frame loop.  group: rp is a multi-device
    context (one process, vr_create_mask) that splits and gathers every frame itself."""
    W, H = cfg["W"], cfg["H"]
    cam = synth.camera(cfg["cam"]).to_vr_camera()
    p = vr_amd.default_params(shading=cfg["shading"], ert_eps=cfg["ert"],
                              skip_empty=cfg.get("skip_empty", 0), frames_in_flight=inflight,
                              exact_gradient=cfg.get("exact_gradient", 0))
    sr = vr_amd.shard_rows(H, row_block, world)
    if BACKEND != "nccl":
        inflight = 1  # host-staged gloo rehearsal: serial
    slots = []
    for _ in range(0 if group else inflight):
        gbuf = frame = None
        if world > 1 and rank == 0:
            # RCCL gathers straight into the rank-major buffer the assembly kernel reads
            gbuf = torch.empty((world, sr, W), dtype=torch.int32, device="cuda")
            frame = torch.empty((H, W), dtype=torch.int32, device="cuda")
        slots.append(vr_dist.Slot(torch.empty((sr, W), dtype=torch.int32, device="cuda"), gbuf,
                                  frame, torch.cuda.Stream()))

    my_stats = rp.count_work(cam, p, row_block, rank, world)
    sdev = "cuda" if BACKEND == "nccl" else "cpu"
    keys = ("rays", "samples", "shaded_samples", "steps", "skipped_samples")
    tot = torch.tensor([my_stats[k] for k in keys], dtype=torch.float64, device=sdev)
    if world > 1:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    frame_stats = dict(zip(keys, [int(x) for x in tot.tolist()]))

    pipe = None
    if group:
        pipe = GroupFrames(rp, cam, p, H, W)
    elif world > 1 and BACKEND == "nccl" and GATHER == "native":
        # the whole frame in the library: render -> ncclGather -> assemble, stream-ordered
        try:
            pipe = NativeFrames(dist_frames(rp, rank, world, row_block, inflight), cam, p, rank, H, W)
        except RuntimeError as e:  # raised on every rank together (dist_frames)
            print(f"bench: native RCCL frame path unavailable ({e}); using torch.distributed.gather",
                  file=sys.stderr, flush=True)
            set_gather("torch")
    if pipe is None:
        pipe = vr_dist.FramePipeline(
            slots, rank, world, dist,
            render=lambda sl: rp.render_device(cam, p, sl.shard.data_ptr(), vr_amd.OUT_RGBA8,
                                               row_block, rank, world, sl.stream.cuda_stream),
            assemble=lambda sl: rp.assemble_rows(sl.gbuf.data_ptr(), sl.frame.data_ptr(),
                                                 vr_amd.OUT_RGBA8, row_block, world,
                                                 sl.stream.cuda_stream),
            host_staging=(BACKEND != "nccl"))

    for _ in range(warmup):
        pipe.step()
    pipe.drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    rp.timing_reset()
    rp.timing_enable(True)
    native = isinstance(pipe, NativeFrames)
    if native:
        pipe.frames.timing_read()  # clears the warm-up record
        pipe.frames.timing_enable(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        pipe.step()
    pipe.drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    rp.timing_enable(False)
    kms, nl = rp.timing_read()
    rend_ms = gath_ms = float("nan")
    if native:
        pipe.frames.timing_enable(False)
        r, g, n = pipe.frames.timing_read()
        rend_ms, gath_ms = r / max(n, 1), g / max(n, 1)
    el = torch.tensor([t1 - t0], dtype=torch.float64, device=sdev)
    # per-rank diagnostics (straggler localisation): this rank's own loop time, its render
    # kernel's average duration and, on the native RCCL path, the render and ncclGather
    # spans timed by HIP events on their streams
    mine = torch.tensor([rank, t1 - t0, kms / max(nl, 1), rend_ms, gath_ms], dtype=torch.float64,
                        device=sdev)
    per_rank = [mine]
    if world > 1:
        per_rank = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(per_rank, mine)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    per_rank = [dict(rank=int(v[0]), loop_ms_per_frame=round(float(v[1]) / steps * 1e3, 4),
                     kernel_ms=round(float(v[2]), 4),
                     render_span_ms=None if np.isnan(float(v[3])) else round(float(v[3]), 4),
                     gather_span_ms=None if np.isnan(float(v[4])) else round(float(v[4]), 4))
                for v in (t.cpu() for t in per_rank)]
    if group:
        # one process drives every device: one entry per device of the context, from its own
        # HIP events (vr_debug_timing_member), so a slow frame names its straggler
        loop = round((t1 - t0) / steps * 1e3, 4)
        per_rank = []
        for m in range(rp.n_members):
            t = rp.timing_member(m)
            n = max(t["frames"], 1)
            per_rank.append(dict(rank=m, device=t["device"], loop_ms_per_frame=loop,
                                 kernel_ms=round(t["kernel_ms"] / n, 4),
                                 render_span_ms=round(t["render_ms"] / n, 4),
                                 gather_span_ms=round(t["gather_ms"] / n, 4),
                                 assemble_span_ms=round(t["assemble_ms"] / n, 4) if m == 0 else None,
                                 frames=t["frames"]))
    check = None
    if world > 1 and rank == 0:
        # the assembled frame must equal this device's single-rank render of the whole frame
        full = torch.empty((vr_amd.shard_rows(H, row_block, 1), W), dtype=torch.int32, device="cuda")
        rp.render_device(cam, p, full.data_ptr(), vr_amd.OUT_RGBA8, row_block, 0, 1,
                         torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        check = bool(torch.equal(full[:H], pipe.last.frame))
    return dict(secs=float(el.item()), kms=kms / max(nl, 1), frame=frame_stats, mine=my_stats,
                shard_px=sr * W, check=check, per_rank=per_rank, warmup_frames=warmup,
                last_frame=pipe.last.frame if group else None,
                last_frame_ptr=slots[0].shard.data_ptr() if slots else pipe.last.frame.data_ptr(),
                keep=slots)


def orbit_cameras(n=360):
    """A camera drag like the reference's (main_window.cpp:284-289 -> Camera::rotate,
    camera.cpp:15-29): every frame rotate((4, 1)) -- 1 degree of yaw, 0.25 degree of pitch at the
    0.25 sensitivity -- while the radius swings 1.6 -> 3.0 -> 1.6 (zoom), so the path crosses the
    frame-filling, oblique, side and default-radius view classes."""
    cam = vr_amd.make_camera(radius=1.6)
    out = []
    for i in range(n):
        cam.rotate(4.0, 1.0)
        cam.set_radius(1.6 + 1.4 * (1.0 - np.cos(2.0 * np.pi * i / n)) / 2.0)
        out.append(cam.to_vr_camera())
    return out


def orbit(rp, cfg, frame_ptr, n=360):
    """The renderer under a moving camera: the orbit path (orbit_cameras),
    default memory budget, derived structures freed first.  Two laps of serial frames, each timed
    on the host (enqueue + device synchronize: every build, eviction and kernel switch on the
    path lands in its frame): the first lap builds what the views want, the second runs on what
    the first left.  Reported per lap: p50 / p99 / max frame ms and the library's derived-
    structure history (builds, evictions, downgrades).  The frame time also varies with the
    view's own work (samples per frame move 3-4x along the path), so two stability figures sit
    beside p99 / p50: each frame's time over the same camera's second-lap time (spikes from
    builds and evictions; p99 and the frames above 1.5x), and ns per executed sample (p99 /
    p50).  Then the same path with 3 frames in flight (ms per frame over the path), twice: from
    freed structures (builds included) and on what that pass built."""
    cams = orbit_cameras(n)
    p1 = vr_amd.default_params(shading=cfg["shading"], ert_eps=cfg["ert"])
    p3 = vr_amd.default_params(shading=cfg["shading"], ert_eps=cfg["ert"], frames_in_flight=3)
    stream = torch.cuda.current_stream().cuda_stream
    hist = ("builds", "evictions", "downgrades")

    def history():
        m = rp.memory_report()
        return {k: m[k] for k in hist + ("derived_bytes", "budget_bytes")}

    def fresh():
        rp.set_memory_budget(0)
        rp.set_memory_budget(BUDGET_DEFAULT)
        torch.cuda.synchronize()

    def lap():
        h0 = history()
        t = []
        for cam in cams:
            t0 = time.perf_counter()
            rp.render_device(cam, p1, frame_ptr, vr_amd.OUT_RGBA8, 8, 0, 1, stream)
            torch.cuda.synchronize()
            t.append((time.perf_counter() - t0) * 1e3)
        h1 = history()
        t = np.array(t)
        return t, dict(p50_ms=round(float(np.percentile(t, 50)), 4),
                       p99_ms=round(float(np.percentile(t, 99)), 4), max_ms=round(float(t.max()), 4),
                       mean_ms=round(float(t.mean()), 4),
                       p99_over_p50=round(float(np.percentile(t, 99) / np.percentile(t, 50)), 3),
                       slowest_frames=[int(i) for i in np.argsort(-t)[:5]],
                       **{k: h1[k] - h0[k] for k in hist})

    fresh()
    t1, lap1 = lap()
    t2, lap2 = lap()
    mem = history()
    samples = np.array([rp.count_work(c, p1, 8)["samples"] for c in cams], dtype=np.float64)
    ratio = t1 / t2
    nsps = t2 * 1e6 / np.maximum(samples, 1.0)
    stability = dict(
        first_lap_over_steady_p99=round(float(np.percentile(ratio, 99)), 3),
        first_lap_frames_above_1p5x_steady=int((ratio > 1.5).sum()),
        second_lap_over_first_lap_steady_p99=round(float(np.percentile(t2 / np.minimum(t1, t2), 99)), 3),
        ns_per_sample_p50=round(float(np.percentile(nsps, 50)), 4),
        ns_per_sample_p99=round(float(np.percentile(nsps, 99)), 4),
        ns_per_sample_p99_over_p50=round(float(np.percentile(nsps, 99) / np.percentile(nsps, 50)), 3),
        samples_per_frame_min_max=[int(samples.min()), int(samples.max())])
    # frames in flight over the same path (fresh structures)
    fresh()
    hp = history()
    streams = [torch.cuda.Stream() for _ in range(3)]
    bufs = [torch.empty((cfg["H"], cfg["W"]), dtype=torch.int32, device="cuda") for _ in streams]

    def inflight():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i, cam in enumerate(cams):
            rp.render_device(cam, p3, bufs[i % 3].data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1,
                             streams[i % 3].cuda_stream)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    pip = inflight()  # builds the structures on the way, as the first lap
    h3 = history()
    pip2 = inflight()  # on what the first pass built
    return dict(path=f"{n} frames of Camera::rotate((4, 1)) with the radius 1.6 -> 3.0 -> 1.6, C3 "
                     "volume and params, default memory budget, derived structures freed first",
                first_lap=lap1, second_lap=lap2, stability=stability,
                frames_in_flight_3=dict(ms_per_frame=round(pip, 4),
                                        gsamples_per_s=round(float(samples.sum()) / (pip * 1e-3 * n) / 1e9, 3),
                                        **{k: h3[k] - hp[k] for k in hist}),
                frames_in_flight_3_steady=dict(
                    ms_per_frame=round(pip2, 4),
                    gsamples_per_s=round(float(samples.sum()) / (pip2 * 1e-3 * n) / 1e9, 3)),
                memory_after=mem)


def host_cores():
    """(threads, description): the host CPUs this process can actually use: nproc (the
    affinity mask), capped by the cgroup CPU quota when one is set.  On the MI355X boxes nproc
    is 256 but the quota is 16 CPUs; 256 OpenMP threads in that quota measured 0.17 against
    0.43 Gsamples/s at 16 (time-sliced), so the quota is the core count that runs."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    desc = f"nproc={n}, os.cpu_count()={os.cpu_count()}, cgroup cpu quota=" + (
        f"{quota:g} CPUs" if quota else "none")
    use = max(1, min(n, int(quota))) if quota else n
    return use, desc


def cpu_baseline(rp, cfg, budget_s=12.0, nthreads=None):
    """The CPU oracle (oracle/oracle.c, OpenMP over rows) on a bounded row sample of the same
    frame, on all host cores (nproc)."""
    import pyoracle
    ncores, cores_desc = host_cores()
    if nthreads is None:
        nthreads = ncores
    vol = rp.read_volume()
    _, (vmin, vmax), _ = rp.volume_info()
    cam = synth.camera(cfg["cam"]).to_vr_camera()
    p = vr_amd.default_params(shading=cfg["shading"], ert_eps=cfg["ert"])
    sc = pyoracle.Scene.from_params(vol, vmin, vmax, synth.TFS[cfg["tf"]](), cam, cfg["W"], cfg["H"], p)
    H = cfg["H"]
    buf = np.empty((H, cfg["W"], 4), np.float32)
    # calibrate on rows spread over the frame, then size the sample to ~budget_s of CPU work
    probe = list(range(H // 32, H, H // 16))
    t0 = time.perf_counter()
    sc.render_rows(probe, buf, nthreads)
    per_row = (time.perf_counter() - t0) / len(probe)
    nrows = int(max(16, min(H, budget_s / max(per_row, 1e-6))))
    stride = max(1, H // nrows)
    rows = list(range(stride // 2, H, stride))
    # a whole frame can take well under a second on a many-core host: repeat the sample until
    # ~budget_s of CPU work has been timed, so the rate is not a sub-second measurement
    t, samples, reps = 0.0, 0, 0
    while t < budget_s * 0.8 or reps == 0:
        t0 = time.perf_counter()
        _, st = sc.render_rows(rows, buf, nthreads)
        t += time.perf_counter() - t0
        samples += st["samples"]
        reps += 1
    return dict(value=round(samples / t / 1e9, 4), unit="Gsamples/s", cores=nthreads, kind="port",
                ms_per_frame=round(t / reps / len(rows) * H * 1e3, 2),
                sample=f"{len(rows)} of {H} frame rows (every {stride}th row) x {reps} repeats, same "
                       f"volume/camera/TF/params; {samples} samples in {t:.2f} s (oracle/oracle.c, "
                       f"OpenMP x{nthreads}; {cores_desc})")


def cpu_baseline_other(name, device, budget_s, nthreads):
    """the CPU baseline of C1 and C2 as well (their own volumes and frames)."""
    cfg = CONFIGS[name]
    rp = setup_pass(cfg, device)
    try:
        r = cpu_baseline(rp, cfg, budget_s, nthreads)
    finally:
        rp.close()
    r["workload"] = cfg["workload"]
    return r


def load_traffic(cfg_name, world, kernel, layout):
    """Measured HBM bytes per frame (rocprofv3 PMC, profiles/pmc_traffic.json written by
    tools/traffic_json.py from tools/measure_round.sh) for this config: (bytes, source, status).
    The entry counts only if it was measured on the kernel this run launches, in the same
    device code (vr_amd.kernel_code_hash) and the same volume layout; otherwise bytes is
    None and status says why ("stale: ...")."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None, None, "missing: no profiles/pmc_traffic.json"
    try:
        e = json.load(open(path)).get(cfg_name)
    except Exception as ex:
        return None, None, f"unreadable: {ex}"
    if not e:
        return None, None, f"missing: no entry for {cfg_name}"
    want = dict(n_gpus=world, kernel=kernel, code_hash=vr_amd.kernel_code_hash(), layout=layout)
    for k, v in want.items():
        if e.get(k) != v:
            return None, e.get("source"), f"stale: {k} {e.get(k)!r} != this run's {v!r}"
    return float(e["hbm_bytes_per_launch"]), e.get("source"), "ok"


def fail_exit(msg):
    print(f"bench: {msg}", file=sys.stderr, flush=True)
    sys.exit(2)


def volume_layout(rp):
    """The resident layout a PMC traffic entry is keyed on: storage type + bricked bytes."""
    _, _, st = rp.volume_info()
    return f"st{st}:{rp.volume_bytes()}"


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def gpu_fds(pid="self"):
    """The GPU device files a process holds open (/dev/kfd, /dev/dri/*): the HIP runtime opens
    them when it initialises, so a parent that holds none has not touched the GPU."""
    d = f"/proc/{pid}/fd"
    out = []
    for fd in os.listdir(d):
        try:
            t = os.readlink(os.path.join(d, fd))
        except OSError:
            continue
        if t == "/dev/kfd" or t.startswith("/dev/dri/"):
            out.append(t)
    return sorted(out)


def launch_ranks(n: int, rehearsal: bool = False) -> int:
    """--gpus N > 1 without WORLD_SIZE: run this script under torch.distributed.run, one process
    per GPU, as a child, and return its exit status.  The child's rank 0 prints the JSON line on
    the stdout this process hands down.  The parent must not have initialised the GPU (it only
    counted devices, which does not): it checks that it holds no GPU device file before it
    spawns, refuses (exit 2) otherwise, and hands the check's result to the ranks, which report
    it in the JSON line (`launch`).  rehearsal: the N ranks share the visible device(s) and
    gather through gloo (VR_DIST_BACKEND=gloo), the driver's exact launch path on one GPU."""
    import subprocess
    held = gpu_fds()
    if held:
        fail_exit(f"the launching process holds GPU device files {held} before spawning the "
                  "ranks: something initialised HIP in the parent")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env["VR_BENCH_LAUNCH"] = json.dumps(dict(path="bench.py launch_ranks -> torch.distributed.run",
                                             parent_pid=os.getpid(), parent_gpu_fds=held,
                                             rehearsal=rehearsal))
    if rehearsal:
        env["VR_DIST_BACKEND"] = "gloo"
    print(f"bench: --gpus {n} without WORLD_SIZE: launching {' '.join(cmd)} (parent holds no GPU "
          f"device file{'; rehearsal: gloo ranks sharing the visible GPU' if rehearsal else ''})",
          file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-variants", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    # 3 frames in flight on the box's 4 hardware queues: C3 318.9-326.4 Gsamples/s against
    # 309.6-312.2 with 4 and 317.8-322.3 with 6 (profiles/r03/frames_in_flight/)
    ap.add_argument("--frames-in-flight", type=int, default=3,
                    help="frames in flight on separate streams (1 = serial frame loop)")
    ap.add_argument("--serial-gather", action="store_true",
                    help="= --frames-in-flight 1: each frame's gather waited for before the next render")
    ap.add_argument("--gather", default="native", choices=("native", "torch"),
                    help="N > 1: the library's RCCL frame path (vr_dist.h) or torch.distributed.gather")
    ap.add_argument("--hw-queues", type=int, default=None,
                    help="GPU_MAX_HW_QUEUES for this process (set before HIP starts; default: the "
                         "environment's, HIP default 4)")
    ap.add_argument("--multi-device-context", action="store_true",
                    help="without WORLD_SIZE: drive the N GPUs from one process through "
                         "vr_create_mask (default for N > 1: one process per GPU, launched here)")
    ap.add_argument("--members-on-one-gpu", type=int, default=0,
                    help="rehearsal: a multi-device context of M members all on device 0 "
                         "(vr_debug_create_members, copy exchange); --gpus must be 1")
    ap.add_argument("--rehearse-launch", action="store_true",
                    help="rehearsal: --gpus N > 1 through the driver's launch path (launch_ranks, "
                         "torch.distributed.run) with N gloo ranks sharing the visible GPU(s)")
    args = ap.parse_args()
    if args.gpus < 1:
        fail_exit("--gpus must be >= 1")
    if args.members_on_one_gpu and (args.gpus != 1 or os.environ.get("WORLD_SIZE")):
        fail_exit("--members-on-one-gpu needs --gpus 1 and no torch.distributed launch")
    if args.rehearse_launch and (args.gpus < 2 or args.multi_device_context or args.members_on_one_gpu):
        fail_exit("--rehearse-launch needs --gpus N >= 2 and the per-process path")
    if (os.environ.get("WORLD_SIZE") is None and args.gpus > 1 and not args.multi_device_context):
        ndev = torch.cuda.device_count()  # counts devices without initialising HIP
        if args.rehearse_launch:
            if ndev < 1:
                fail_exit(f"--rehearse-launch needs a HIP device; device 0 is not present ({ndev} visible)")
        elif ndev < args.gpus:
            fail_exit(f"--gpus {args.gpus} needs {args.gpus} HIP devices; device {ndev} is not "
                      f"present ({ndev} visible)")
        sys.exit(launch_ranks(args.gpus, rehearsal=args.rehearse_launch))

    # stdout carries exactly one line, the JSON result (rank 0).  Libraries print banners to
    # fd 1 on their own (RCCL writes its version block when a communicator is created), so fd
    # 1 points at stderr for the whole run and is restored only for the result line.
    sys.stdout.flush()
    result_fd = os.dup(1)
    os.dup2(2, 1)

    # How the N GPUs are driven.  torch.distributed.run sets WORLD_SIZE: one process per GPU,
    # and the launch must match --gpus.  Without it (and with --multi-device-context), --gpus N
    # is ONE process over N devices (vr_create_mask).  Either way exactly N devices must be
    # there.
    world_env = os.environ.get("WORLD_SIZE")
    world = int(world_env) if world_env is not None else 1
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world_env is not None and world != args.gpus:
        fail_exit(f"--gpus {args.gpus} but torch.distributed.run started WORLD_SIZE={world} "
                  "ranks; they must agree")
    group = world_env is None and (args.gpus > 1 or args.multi_device_context
                                   or args.members_on_one_gpu > 0)
    members = [0] * args.members_on_one_gpu if args.members_on_one_gpu else None
    ndev = torch.cuda.device_count()
    global BACKEND, GATHER
    # VR_DIST_BACKEND=gloo rehearses the N > 1 path with ranks sharing devices (host-staged
    # gathers); the real multi-GPU run uses "nccl" (RCCL over xGMI), one device per rank.
    BACKEND = os.environ.get("VR_DIST_BACKEND", "nccl")
    GATHER = args.gather
    if group:
        if ndev < args.gpus:
            fail_exit(f"--gpus {args.gpus} needs {args.gpus} HIP devices in this process; device "
                      f"{ndev} is not present ({ndev} visible)")
        device = 0
    else:
        if world == 1 and ndev < 1:
            fail_exit(f"--gpus 1 needs a HIP device; device 0 is not present ({ndev} visible)")
        if BACKEND == "nccl" and world > 1 and ndev <= local_rank:
            fail_exit(f"rank {rank} (LOCAL_RANK {local_rank}) has no device: device {local_rank} is "
                      f"not present ({ndev} visible)")
        device = local_rank % max(1, ndev)
    torch.cuda.set_device(device)
    if world > 1:
        if BACKEND == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(BACKEND)
    n_gpus = args.gpus if group else world

    cfg = CONFIGS[args.config]
    rp = setup_pass(cfg, device, device_mask=((1 << args.gpus) - 1) if group and not members else None,
                    members=members)
    if group and rp.device_mask != (1 << args.gpus) - 1:
        fail_exit(f"multi-device context spans mask {rp.device_mask:#x}, not {args.gpus} devices")
    vbytes = np.dtype(cfg["dtype"]).itemsize

    inflight = 1 if args.serial_gather else max(1, min(8 if group else 16, args.frames_in_flight))
    if BACKEND != "nccl":
        inflight = 1
    warm = max(args.warmup, STEADY_WARMUP)

    # also the reference-equivalent sample count (volume.frag as written: no
    # ERT, every in-slab step sampled) of the same frame, per second of this configuration
    ref_cam = synth.camera(cfg["cam"]).to_vr_camera()
    ref_stats = rp.count_work(ref_cam, vr_amd.default_params(), 8, rank, world)
    ref_samples = torch.tensor([ref_stats["samples"]], dtype=torch.float64,
                               device="cuda" if BACKEND == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(ref_samples, op=dist.ReduceOp.SUM)
    ref_samples = int(ref_samples.item())

    def frame_check(last_frame, vcfg, p):
        """Multi-device context: the assembled frame == a one-device context's frame, bytes."""
        one = setup_pass(vcfg, device)
        try:
            full = torch.empty((vcfg["H"], vcfg["W"]), dtype=torch.int32, device="cuda")
            one.render_device(synth.camera(vcfg["cam"]).to_vr_camera(), p, full.data_ptr(),
                              vr_amd.OUT_RGBA8, 16, 0, 1, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            return bool(torch.equal(full, last_frame))
        finally:
            one.close()

    # The headline first: W (at least STEADY_WARMUP) untimed frames, then exactly K timed ones.
    R = run_variant(rp, cfg, args.steps, warm, rank, world, inflight, group=group)
    if group and rank == 0:
        R["check"] = frame_check(R["last_frame"], cfg, vr_amd.default_params(
            shading=cfg["shading"], ert_eps=cfg["ert"], frames_in_flight=inflight))
    secs, kms, fstats = R["secs"], R["kms"], R["frame"]
    frame_s = secs / args.steps
    value = fstats["samples"] * args.steps / secs / 1e9
    fps = args.steps / secs
    gather_bytes = algorithmic_bytes(fstats, vbytes, cfg["W"] * cfg["H"])
    # the kernel the launch policy picked for the headline's view (vr_kernel_name reads the
    # last frame's view), and the PMC bytes measured for that kernel
    kernel = rp.kernel_name(vr_amd.default_params(shading=cfg["shading"]))
    layout = volume_layout(rp)
    traffic, traffic_src, traffic_status = load_traffic(args.config, n_gpus, kernel, layout)
    # compulsory traffic of a frame: every voxel once at the source dtype + the framebuffer
    compulsory = int(np.prod(cfg["dims"])) * vbytes + cfg["W"] * cfg["H"] * 4

    variants = {}
    serial_kms = None
    if not args.no_variants and inflight > 1:
        # the serial form too (one frame at a time; for N > 1 each frame's
        # gather waited for before the next render).  Its kernels run alone on the device,
        # so their HIP-event durations are the kernel's own.
        ns = max(5, args.steps // 2)
        V = run_variant(rp, cfg, ns, warm, rank, world, 1, group=group)
        serial_kms = V["kms"]
        variants["serial_frames"] = dict(
            value=round(V["frame"]["samples"] * ns / V["secs"] / 1e9, 3), unit="Gsamples/s",
            ms_per_step=round(V["secs"] / ns * 1e3, 4), fps=round(ns / V["secs"], 2),
            kernel_ms=round(V["kms"], 4), frame_check=V["check"], warmup_frames=V["warmup_frames"])
    if not args.no_variants and args.config == "c3":
        # the reference's default camera (benchmarks at r=1.6 plus the default)
        dcfg = CONFIGS["c3_default"]
        V = run_variant(rp, dcfg, args.steps, warm, rank, world, inflight, group=group)
        # the launch policy picks the kernel per view (vr_api.hip use_pipeline): match the PMC
        # bytes of the kernel this view ran
        dkernel = rp.kernel_name(vr_amd.default_params(shading=dcfg["shading"]))
        dtr, _, dstatus = load_traffic("c3_default", n_gpus, dkernel, layout)
        dms = V["secs"] / args.steps
        variants["default_camera"] = dict(
            workload=dcfg["workload"], camera=synth.CAMERAS[dcfg["cam"]],
            value=round(V["frame"]["samples"] * args.steps / V["secs"] / 1e9, 3), unit="Gsamples/s",
            ms_per_step=round(dms * 1e3, 4), fps=round(args.steps / V["secs"], 2),
            samples_per_frame=V["frame"]["samples"], rays_per_frame=V["frame"]["rays"],
            kernel=dkernel, hbm_bytes_per_frame=dtr, traffic_status=dstatus,
            hbm_frac=round(dtr / dms / 1e9 / HBM_PEAK_GBS, 4) if dtr else None,
            traffic_over_compulsory=round(dtr / compulsory, 3) if dtr else None,
            warmup_frames=V["warmup_frames"])
        vcfg = CONFIGS["c3_ref"]
        V = run_variant(rp, vcfg, args.steps, warm, rank, world, inflight, group=group)
        rkernel = rp.kernel_name(vr_amd.default_params(shading=0))
        rtr, _, rstatus = load_traffic("c3_ref", n_gpus, rkernel, layout)
        rms = V["secs"] / args.steps
        variants["reference_semantics_no_shading_no_ert"] = dict(
            value=round(V["frame"]["samples"] * args.steps / V["secs"] / 1e9, 3), unit="Gsamples/s",
            ms_per_step=round(rms * 1e3, 4),
            fps=round(args.steps / V["secs"], 2), samples_per_frame=V["frame"]["samples"],
            kernel_ms=round(V["kms"], 4), hbm_bytes_per_frame=rtr, traffic_status=rstatus,
            hbm_frac=round(rtr / rms / 1e9 / HBM_PEAK_GBS, 4) if rtr else None,
            warmup_frames=V["warmup_frames"])
        # opt-in empty-space skipping (bit-identical frames): executed samples drop, so it is
        # reported as fps and as reference-equivalent samples/s, never as the headline value
        scfg = dict(CONFIGS["c3"], skip_empty=1)
        V = run_variant(rp, scfg, args.steps, warm, rank, world, inflight, group=group)
        f3 = V["frame"]
        variants["c3_skip_empty"] = dict(
            fps=round(args.steps / V["secs"], 2), ms_per_step=round(V["secs"] / args.steps * 1e3, 4),
            kernel_ms=round(V["kms"], 4),
            executed_gsamples_per_s=round(f3["samples"] * args.steps / V["secs"] / 1e9, 3),
            reference_equivalent_gsamples_per_s=round(
                (f3["samples"] + f3["skipped_samples"]) * args.steps / V["secs"] / 1e9, 3),
            samples_per_frame=f3["samples"], skipped_samples_per_frame=f3["skipped_samples"],
            warmup_frames=V["warmup_frames"])
        # exact f32 central differences (vr_params.exact_gradient = 1): every frame bit-identical
        # to the f32 oracle; the headline's default reads the binary16 difference field
        ecfg = dict(CONFIGS["c3"], exact_gradient=1)
        V = run_variant(rp, ecfg, args.steps, warm, rank, world, inflight, group=group)
        variants["c3_exact_gradient"] = dict(
            value=round(V["frame"]["samples"] * args.steps / V["secs"] / 1e9, 3), unit="Gsamples/s",
            ms_per_step=round(V["secs"] / args.steps * 1e3, 4), fps=round(args.steps / V["secs"], 2),
            kernel_ms=round(V["kms"], 4),
            kernel=rp.kernel_name(vr_amd.default_params(shading=1, exact_gradient=1)),
            note="vr_params.exact_gradient = 1: f32 differences (6 field loads per shaded sample), "
                 "bit-identical to the f32 oracle",
            warmup_frames=V["warmup_frames"])

    if not args.no_variants and args.config == "c3" and world == 1 and not group:
        # A camera crossing view classes: after frames of the fill view (the
        # difference field), the reference's default camera needs the stencil copy (~0.76 GB for
        # 512^3).  Built lazily, inside its first frame; or ahead by vr_prepare.  Serial frames,
        # host-timed, derived structures freed before each arm (budget 0, then the default).
        fcam = synth.camera(cfg["cam"]).to_vr_camera()
        dcam = synth.camera("default").to_vr_camera()
        vp = vr_amd.default_params(shading=cfg["shading"], ert_eps=cfg["ert"])

        def fresh_fill():
            rp.set_memory_budget(0)
            rp.set_memory_budget(BUDGET_DEFAULT)
            for _ in range(3):
                rp.render_device(fcam, vp, R["last_frame_ptr"], vr_amd.OUT_RGBA8, 8, 0, 1)
            torch.cuda.synchronize()

        def one_frame(cam):
            t0 = time.perf_counter()
            rp.render_device(cam, vp, R["last_frame_ptr"], vr_amd.OUT_RGBA8, 8, 0, 1)
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) * 1e3

        fresh_fill()
        lazy = one_frame(dcam)
        built = rp.memory_report()
        steady = sorted(one_frame(dcam) for _ in range(20))[10]
        fresh_fill()
        t0 = time.perf_counter()
        rp.prepare(dcam, vp)
        prep = (time.perf_counter() - t0) * 1e3
        prepared = one_frame(dcam)
        variants["view_switch"] = dict(
            path="fill view (r = 1.6, difference field) -> the reference's default camera (stencil copy)",
            first_frame_lazy_ms=round(lazy, 3), first_frame_after_prepare_ms=round(prepared, 3),
            prepare_ms=round(prep, 3), steady_serial_frame_ms=round(steady, 3),
            derived_bytes_after_switch=built["derived_bytes"],
            budget_bytes=built["budget_bytes"],
            stencil_copy_bytes=built["stencil_copy_bytes"], field_bytes=built["field_bytes"],
            note="host-timed serial frames around vr_render_device; vr_prepare builds the copy "
                 "outside the frame (vr.h ABI 7)")

    if not args.no_variants and args.config == "c3" and world == 1 and not group:
        variants["orbit"] = orbit(rp, cfg, R["last_frame_ptr"])

    if not args.no_variants and world == 1 and not group:
        # PCIe-inclusive: vr_render into (pageable) host memory, the drop-in record() path.
        # The frame's RGBA8 bytes cross PCIe inside the timed region; row bands copy while
        # the later bands render (vr_api.hip vr_render).  Never the headline value.
        hcam = synth.camera(cfg["cam"]).to_vr_camera()
        hp = vr_amd.default_params(shading=cfg["shading"], ert_eps=cfg["ert"])
        hbuf = np.empty((cfg["H"], cfg["W"], 4), dtype=np.uint8)
        for _ in range(min(warm, 30)):
            rp.render(hcam, hp, vr_amd.OUT_RGBA8, out=hbuf)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            rp.render(hcam, hp, vr_amd.OUT_RGBA8, out=hbuf)
        sh = time.perf_counter() - t0
        variants["host_output_pcie"] = dict(
            fps=round(args.steps / sh, 2), ms_per_step=round(sh / args.steps * 1e3, 4),
            gsamples_per_s=round(fstats["samples"] * args.steps / sh / 1e9, 3),
            frame_bytes=int(hbuf.nbytes),
            path="vr_render -> pageable host RGBA8 each frame (synchronous, as OffscreenPass::record + readback)")

    # the CPU baseline last: its OpenMP threads (in this process) would compete with the
    # launching thread of the GPU runs
    cpu = None
    small = int(np.prod(cfg["dims"])) <= 512 ** 3  # the oracle needs the volume as host floats
    if rank == 0 and n_gpus == 1 and not args.no_cpu_baseline and small:
        cpu = cpu_baseline(rp, cfg, args.cpu_budget)
        nproc = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
        if nproc and nproc != cpu["cores"]:
            # the same sample with one thread per nproc CPU, for the record (quota-throttled)
            allc = cpu_baseline(rp, cfg, min(4.0, args.cpu_budget), nproc)
            cpu["all_nproc_threads"] = dict(value=allc["value"], cores=nproc, sample=allc["sample"])
        # C1-C3 on the host cores, C1/C2 on smaller budgets
        cpu["other_configs"] = {n: cpu_baseline_other(n, device, min(4.0, args.cpu_budget), cpu["cores"])
                                for n in ("c1", "c2")}

    mrep = rp.memory_report()
    memory = dict(volume_bytes=mrep["volume_bytes"], derived_bytes=mrep["derived_bytes"],
                  field_bytes=mrep["field_bytes"], budget_bytes=mrep["budget_bytes"],
                  devices=rp.n_members)
    if rank == 0:
        if group and members:
            parallelism = (f"REHEARSAL: image 8-row blocks cyclic x{len(members)} members all on "
                           "device 0 in one process (vr_debug_create_members) + copy exchange")
        elif group:
            parallelism = (f"image 8-row blocks cyclic x{n_gpus} devices in one process "
                           "(vr_create_mask) + RCCL ncclGather (ncclCommInitAll), stream-ordered")
        elif world > 1:
            parallelism = f"image 8-row blocks cyclic x{world} processes" + (
                " + gloo host-staged gather (rehearsal, ranks share devices)" if BACKEND != "nccl"
                else " + RCCL ncclGather (vr_dist.h, stream-ordered)" if GATHER == "native"
                else " + RCCL gather (torch.distributed)")
        else:
            parallelism = "one device"
        # Roofline: the kernel is bound by HBM by the SURVEY's classification (a gather, no
        # MFMA).  `achieved` is the MEASURED DRAM traffic of one frame (rocprofv3 PMC
        # FETCH_SIZE x2 + WRITE_SIZE, same kernel sources/config/camera/layout,
        # profiles/pmc_traffic.json) over this run's frame period, so frac = traffic /
        # ms_per_step / 8 TB/s.  The SURVEY 8d gather model (8 x sizeof(voxel) per sample + 48 x
        # sizeof(voxel) per shaded sample + 4 B/pixel) counts L1/L2 hits as well and is reported
        # apart as gather_bytes_frac, which can exceed 1.
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Gsamples/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(frame_s * 1e3, 4),
            "fps": round(fps, 2),
            "reference_equivalent_gsamples_per_s": round(ref_samples * args.steps / secs / 1e9, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (generated on device; no dataset download)",
            "config": {
                "workload": cfg["workload"],
                "volume": f"{cfg['dims'][0]}x{cfg['dims'][1]}x{cfg['dims'][2]} {np.dtype(cfg['dtype']).name}",
                "viewport": f"{cfg['W']}x{cfg['H']}",
                "camera": synth.CAMERAS[cfg["cam"]],
                "tf": cfg["tf"], "shading": cfg["shading"], "ert_eps": cfg["ert"],
                "exact_gradient": cfg.get("exact_gradient", 0),
                "gradient": ("binary16 difference field scaled by 2^k (vr_params.exact_gradient = 0; "
                             "bit-identical to the oracle restating that rounding; C3 within RMSE "
                             "1.8e-6 of the exact frame)" if cfg["shading"] and cfg["dtype"] == np.float32
                             else None),
                "parallelism": parallelism + f", {inflight} frames in flight",
                "frames_in_flight": inflight,
                "hw_queues": HW_QUEUES,
                "warmup_frames_run": R["warmup_frames"],
                "samples_per_frame": fstats["samples"],
                "reference_equivalent_samples_per_frame": ref_samples,
                "shaded_samples_per_frame": fstats["shaded_samples"],
                "rays_per_frame": fstats["rays"],
                "volume_resident_bytes": rp.volume_bytes(),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": kernel,
                "achieved": round(traffic / frame_s / 1e9, 1) if traffic else None,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(traffic / frame_s / 1e9 / HBM_PEAK_GBS, 4) if traffic else None,
                "traffic": traffic,
                "traffic_status": traffic_status,
                "kernel_code_hash": vr_amd.kernel_code_hash(),
                "volume_layout": layout,
                "traffic_source": (f"profiles/pmc_traffic.json ({traffic_src}): rocprofv3 --pmc "
                                   "FETCH_SIZE x2 + WRITE_SIZE per frame launch") if traffic else None,
                "basis": "measured HBM bytes per frame / this run's ms_per_step / 8000 GB/s",
                "compulsory_bytes": compulsory,
                "compulsory_basis": "every voxel once at the source dtype + the RGBA8 framebuffer",
                "traffic_over_compulsory": round(traffic / compulsory, 3) if traffic else None,
                "kernel_ms": round(kms, 4),
                "serial_kernel_ms": round(serial_kms, 4) if serial_kms else None,
                "gather_bytes_per_frame": int(gather_bytes),
                "gather_bytes_frac": (round(gather_bytes / (serial_kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                                      if serial_kms else None),
                "gather_bytes_model": "SURVEY.md 8d: 8*sizeof(voxel)/sample + 48*sizeof(voxel)/shaded "
                                      "sample + 4 B/pixel, over the kernel-alone (serial) duration; "
                                      "counts L1/L2 hits, so it can exceed 1 (not HBM traffic)",
            },
            "cpu_baseline": cpu,
            # device memory of the context after the run, per device (a multi-device context
            # replicates the volume and its derived structures on every device): bricks,
            # derived structures (difference field, alternative copies, skip-empty) and the
            # budget that caps them (vr.h VR_MEMORY_BUDGET_DEFAULT: 5x the bricks)
            "memory_per_device": memory,
            "frame_check": R["check"],  # N > 1: assembled frame == single-GPU frame, bit for bit
            "per_rank": R["per_rank"],
            # N > 1 started by this script (launch_ranks): the launch path and the parent's
            # GPU-file check; null when the driver's launcher started the ranks itself
            "launch": json.loads(os.environ["VR_BENCH_LAUNCH"]) if os.environ.get("VR_BENCH_LAUNCH") else None,
            "variants": variants,
        }
        sys.stdout.flush()
        os.dup2(result_fd, 1)
        print(json.dumps(out), flush=True)
        os.dup2(2, 1)
    for d in _DIST.values():
        d.close()
    rp.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
