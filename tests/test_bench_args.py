"""CPU (and GPU box): bench.py refuses to run on other than exactly --gpus N GPUs, before any
GPU work, with exit status 2 and a message naming what is missing (a driver run with
`--gpus 8` on a box that cannot supply 8 devices must not silently measure fewer)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, **env_over):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_over)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args, "--steps", "1",
                           "--warmup", "0", "--no-variants", "--no-cpu-baseline"],
                          cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)


def test_more_gpus_than_devices_fails_naming_the_device():
    import torch
    n = torch.cuda.device_count()  # 0 here; 1 on the one-GPU box
    r = _bench(["--gpus", str(n + 1)])
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert f"device {n} is not present" in r.stderr, r.stderr[-2000:]
    assert r.stdout.strip() == ""


def test_launcher_world_size_must_match_gpus():
    r = _bench(["--gpus", "2"], WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "WORLD_SIZE=1" in r.stderr and "must agree" in r.stderr


def test_multi_device_context_needs_the_devices_too():
    import torch
    n = torch.cuda.device_count()
    r = _bench(["--gpus", str(n + 1), "--multi-device-context"])
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert f"device {n} is not present" in r.stderr, r.stderr[-2000:]


def test_member_rehearsal_is_one_gpu_only():
    r = _bench(["--gpus", "2", "--members-on-one-gpu", "2"])
    assert r.returncode == 2 and "--members-on-one-gpu needs --gpus 1" in r.stderr


def test_launch_rehearsal_needs_two_ranks_and_a_device():
    r = _bench(["--gpus", "1", "--rehearse-launch"])
    assert r.returncode == 2 and "--rehearse-launch needs --gpus N >= 2" in r.stderr
    import torch
    if torch.cuda.device_count() == 0:
        r = _bench(["--gpus", "2", "--rehearse-launch"])
        assert r.returncode == 2 and "--rehearse-launch needs a HIP device" in r.stderr, r.stderr[-2000:]


def test_gpu_fds_sees_no_device_file_in_a_cpu_process():
    import bench
    assert bench.gpu_fds() == []
