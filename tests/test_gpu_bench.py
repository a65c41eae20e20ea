"""GPU: bench.py keeps the driver's contract -- one JSON line on stdout with BASELINE.json's
metric, the whole-job value, the roofline object for the timed kernel and the config's
workload name (a short run: 4 steps, no CPU baseline, no variants)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_prints_one_contract_line(gpu):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "4", "--warmup", "2",
                        "--no-cpu-baseline", "--no-variants"],
                       cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert d["metric"] == base["metric"]
    assert d["unit"] == "Gsamples/s" and d["higher_is_better"] is True
    assert d["n_gpus"] == 1 and d["steps"] == 4 and d["warmup"] == 2
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["fps"] > 0
    assert d["dtype"] == "f32" and d["vs_baseline"] is None
    assert d["config"]["workload"].startswith("C3:")
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert "march" in rf["kernel"] and rf["kernel_ms"] > 0
    if rf["traffic"] is not None:  # PMC bytes measured on this kernel (profiles/pmc_traffic.json)
        assert rf["achieved"] > 0 and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
        # frac is measured bytes over this run's frame period: never above the HBM peak
        assert abs(rf["achieved"] - rf["traffic"] / (d["ms_per_step"] * 1e-3) / 1e9) < 0.01 * rf["achieved"]
        assert rf["frac"] <= 1.0
    assert rf["traffic_status"] == "ok" or rf["traffic"] is None
    assert rf["compulsory_bytes"] == 512 ** 3 * 4 + 1920 * 1080 * 4
    assert d["config"]["hw_queues"] >= 1 and d["config"]["warmup_frames_run"] >= d["warmup"]
    assert d["per_rank"][0]["rank"] == 0
    # the value is executed samples of the whole frame per second
    spf = d["config"]["samples_per_frame"]
    assert abs(d["value"] - spf * d["steps"] / (d["ms_per_step"] * 1e-3 * d["steps"]) / 1e9) < 0.01 * d["value"]


def test_bench_multi_device_context_path(gpu):
    """The single-process multi-GPU path (vr_create_mask) of bench.py, forced at N = 1 on the
    one-GPU box: one contract line, n_gpus 1, and the assembled frame equals a one-device
    context's frame (frame_check)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "4", "--warmup", "2",
                        "--no-cpu-baseline", "--no-variants", "--multi-device-context"],
                       cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["frame_check"] is True
    assert "vr_create_mask" in d["config"]["parallelism"]
    assert d["value"] > 0


def test_bench_member_rehearsal_on_one_gpu(gpu):
    """--members-on-one-gpu 2: the multi-device context with two members on device 0 (copy
    exchange) under bench.py's frame loop; the assembled frame equals a one-device frame and
    the per-member rows name both members."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "6", "--warmup", "2",
                        "--no-cpu-baseline", "--no-variants", "--members-on-one-gpu", "2"],
                       cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["frame_check"] is True
    assert "REHEARSAL" in d["config"]["parallelism"]
    pr = d["per_rank"]
    assert [x["rank"] for x in pr] == [0, 1] and all(x["device"] == 0 for x in pr)
    assert all(x["frames"] > 0 and x["kernel_ms"] > 0 for x in pr)


def test_bench_rehearses_the_driver_launch_path(gpu):
    """--gpus 2 --rehearse-launch: the driver's exact multi-GPU command path on one MI355X
    (bench.py -> launch_ranks -> torch.distributed.run -> 2 ranks), the ranks sharing the GPU
    and gathering through gloo.  One contract line with n_gpus 2, the assembled frame equal to
    rank 0's own whole-frame render, one per_rank row per rank, and the launching parent held
    no GPU device file when it spawned the ranks."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rehearse-launch",
                        "--steps", "3", "--warmup", "0", "--no-cpu-baseline", "--no-variants"],
                       cwd=ROOT, capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["frame_check"] is True
    assert sorted(x["rank"] for x in d["per_rank"]) == [0, 1]
    ln = d["launch"]
    assert ln["rehearsal"] is True and ln["parent_gpu_fds"] == [] and "launch_ranks" in ln["path"]
    assert "rehearsal" in d["config"]["parallelism"]


def test_device_count_opens_no_gpu_file_and_init_does(gpu):
    """The launching parent counts devices with torch.cuda.device_count(): on this image that
    opens no GPU device file (bench.gpu_fds), whereas initialising HIP does -- so the detector
    launch_ranks relies on sees a real initialisation."""
    code = ("import sys; sys.path.insert(0, %r); import bench, torch; n = torch.cuda.device_count(); "
            "before = bench.gpu_fds(); torch.cuda.init(); torch.empty(1, device='cuda'); "
            "print(n, len(before), len(bench.gpu_fds()))" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    n, before, after = (int(x) for x in r.stdout.split()[-3:])
    assert n >= 1 and before == 0 and after > 0
