"""GPU: randomized API sequences against the oracle (state transitions, not single frames).

Each seed drives one context through a random sequence of the boundary's calls -- a new
volume (four element types, some integer-valued floats that are stored narrow), a new TF, a
slicing box, a resize (some frames of >= 256 rows: vr_render's row bands), a synchronous host
frame, and bursts of 2-4 frames in flight on different streams whose views need different
derived structures (alternative brick copies, the binary16 or f32 difference field, skip-empty
ranges).  A frame in flight must equal the same frame rendered serially afterwards, bit for
bit, and every serial frame must equal the oracle bit for bit (restating the binary16 field
where the kernel read it).  (Volumes here are small, so builds finish before the next frames
start: the timing-sensitive ordering cases have their own tests in test_gpu_parity.py,
test_field_precision_switch_orders_other_streams and test_builds_on_other_streams_are_chained.)"""
import numpy as np
import pytest

import pyoracle
import synth
import vr_amd

pytestmark = pytest.mark.gpu

CAMS = [(1.6, None), (1.6, (40.0, 25.0)), (1.6, (360.0, 0.0)), (2.0, (180.0, 140.0)),
        (3.0, None), (1.3, (-120.0, 80.0))]


@pytest.fixture(scope="module", params=[None, 0x1], ids=["device", "mask"])
def rp(request, gpu):
    """A one-device context, and a vr_create_mask context over device 0 (the multi-device
    path: member contexts, frame workers, the group's own streams)."""
    r = vr_amd.OffscreenPass(64, 48, device_mask=request.param)
    yield r
    r.close()


def new_volume(rng):
    dims = tuple(int(x) for x in rng.integers(20, 72, size=3))
    base = synth.gaussians_numpy(dims[::-1], seed=int(rng.integers(0, 10000)))
    kind = int(rng.integers(0, 4))
    if kind == 0:
        return base
    if kind == 1:  # integer-valued floats: stored as 8-bit (the reference importer's path)
        return np.rint(base / base.max() * 255.0).astype(np.float32)
    if kind == 2:
        return np.rint(base / base.max() * 30000.0 - 2000.0).astype(np.int16)
    return (base * 7.0 - 1.0).astype(np.float64)


def random_params(rng, inflight):
    return vr_amd.default_params(shading=int(rng.random() < 0.6),
                                 ert_eps=float(rng.choice([0.0, 1e-5])),
                                 skip_empty=int(rng.random() < 0.3),
                                 exact_gradient=int(rng.random() < 0.4),
                                 frames_in_flight=inflight)


def oracle_frame(rp, state, cam, p):
    """The serial frame and its oracle restatement (bit for bit)."""
    img = rp.render(cam, p, vr_amd.OUT_RGBA32F)
    half = "F32H" in rp.kernel_name(p)
    vol, ds, tf, (smin, smax) = state["vol"], state["ds"], state["tf"], state["slice"]
    W, H = rp.size
    sc = pyoracle.Scene.from_params(vol.astype(np.float32), ds.vmin, ds.vmax, tf, cam, W, H, p,
                                    smin, smax, grad_f16=half)
    ref, _ = sc.render()
    bad = int((img.view(np.uint32) != ref.astype(np.float32).view(np.uint32)).any(axis=-1).sum())
    return img, bad, rp.kernel_name(p)


@pytest.mark.parametrize("seed", range(64))
def test_random_call_sequence(rp, seed):
    import torch
    rng = np.random.default_rng(7000 + seed)
    state = {}
    vol = new_volume(rng)
    state.update(vol=vol, ds=synth.dataset(vol), tf=synth.tf_band(0.15, 0.9),
                 slice=((0.0, 0.0, 0.0), (1.0, 1.0, 1.0)))
    rp.volume_dataset_changed(state["ds"])
    rp.transfer_function_changed(state["tf"])
    rp.slicing_changed(*state["slice"])
    rp.framebuffer_size_changed(160, 120)
    streams = [torch.cuda.Stream() for _ in range(4)]
    log = []
    for step in range(20):
        op = rng.choice(["volume", "tf", "slice", "resize", "host", "burst", "burst"])
        log.append(str(op))
        if op == "volume":
            vol = new_volume(rng)
            state.update(vol=vol, ds=synth.dataset(vol))
            rp.volume_dataset_changed(state["ds"])
        elif op == "tf":
            state["tf"] = [synth.tf1, synth.tf2, synth.tf_color,
                           lambda: synth.tf_band(0.2, 0.95)][int(rng.integers(0, 4))]()
            rp.transfer_function_changed(state["tf"])
        elif op == "slice":
            if rng.random() < 0.5:
                a = rng.uniform(0.0, 0.4, size=3)
                b = rng.uniform(0.6, 1.0, size=3)
                state["slice"] = (tuple(float(x) for x in a), tuple(float(x) for x in b))
            else:
                state["slice"] = ((0.0, 0.0, 0.0), (1.0, 1.0, 1.0))
            rp.slicing_changed(*state["slice"])
        elif op == "resize":
            W, H = ((int(rng.integers(200, 321)), int(rng.integers(256, 300))) if rng.random() < 0.4
                    else (int(rng.integers(40, 200)), int(rng.integers(30, 160))))
            rp.framebuffer_size_changed(W, H)
        elif op == "host":
            r, rot = CAMS[int(rng.integers(0, len(CAMS)))]
            cam = vr_amd.make_camera(radius=r, rotate=rot).to_vr_camera()
            _, bad, kname = oracle_frame(rp, state, cam, random_params(rng, 1))
            assert bad == 0, f"seed {seed} step {step} ({' '.join(log)}): {bad} pixels, {kname}"
        else:  # a burst of frames in flight on different streams, different views and params
            n = int(rng.integers(2, 5))
            W, H = rp.size
            frames = []
            for i in range(n):
                r, rot = CAMS[int(rng.integers(0, len(CAMS)))]
                cam = vr_amd.make_camera(radius=r, rotate=rot).to_vr_camera()
                p = random_params(rng, n)
                out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
                rp.render_device(cam, p, out.data_ptr(), vr_amd.OUT_RGBA32F, 16, 0, 1,
                                 streams[i].cuda_stream)
                frames.append((cam, p, out))
            torch.cuda.synchronize()
            for i, (cam, p, out) in enumerate(frames):
                got = out.cpu().numpy()
                serial, bad, kname = oracle_frame(rp, state, cam, p)
                assert bad == 0, f"seed {seed} step {step} frame {i} serial: {bad} pixels, {kname}"
                diff = int((got.view(np.uint32) != serial.view(np.uint32)).any(axis=-1).sum())
                assert diff == 0, (f"seed {seed} step {step} ({' '.join(log)}) frame {i} of {n} in "
                                   f"flight: {diff} pixels differ from the serial frame, {kname}")
    rp.slicing_changed((0.0, 0.0, 0.0), (1.0, 1.0, 1.0))
