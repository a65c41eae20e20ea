"""Host cost per call of the per-frame torch.distributed gather on a world-size-1 RCCL group
(the only RCCL group one GPU can hold), and of a render_device ctypes call."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for sub in ("volumetric-renderer_amd", "tools"):
    sys.path.insert(0, os.path.join(ROOT, sub))
import torch, torch.distributed as dist
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29533")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
x = torch.ones(135 * 1920, dtype=torch.int32, device="cuda")
g = torch.empty((1, 135 * 1920), dtype=torch.int32, device="cuda")
s = torch.cuda.Stream()
for n in (10, 1000):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ws = []
    with torch.cuda.stream(s):
        for _ in range(n):
            ws.append(dist.gather(x, [g[0]], dst=0, async_op=True))
        for w in ws:
            w.wait()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"gather x{n}: host {1e6*(t1-t0)/n:.1f} us/call, incl. device {1e6*(t2-t0)/n:.1f} us/call", flush=True)
dist.destroy_process_group()
