"""CPU, world size 2 and 3 (gloo): the multi-GPU frame schedule of vr_dist.cpp, run on host
threads.

vr_dist_render enqueues every frame through vr::sched::FrameSchedule (csrc/vr_frame_schedule.h)
on HIP streams and events, with ncclGather as the collective.  lib/libvr_sched_host.so runs the
SAME FrameSchedule::issue with a host executor (csrc/vr_sched_host.cpp): one worker thread per
stream, events completed in stream order, hipStreamWaitEvent semantics.  Here each rank drives
it with the CPU oracle rendering its row blocks (random delays shuffle the timing),
torch.distributed.gather over gloo standing in for ncclGather, and numpy assembly into ONE
frame buffer reused by every frame (as rank 0's frame_dev is).  Checked: every frame the caller
consumes equals the single-process oracle frame bit for bit, and the op log honours the
schedule's ordering (gathers in frame order after their render, a slot re-rendered only after
its previous frame was assembled/gathered, assembly of frame i+1 after the caller consumed
frame i; rank r > 0's caller stream is not ordered after its frames)."""
import ctypes as C
import os
import socket
import threading
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "volumetric-renderer_amd", "lib", "libvr_sched_host.so")
OPS = ("render", "gather", "assemble", "consume")
CB = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_uint64)


def _lib():
    lib = C.CDLL(LIB)
    lib.vr_sched_host_create.restype = C.c_void_p
    lib.vr_sched_host_create.argtypes = [C.c_int, C.c_int, CB, C.c_void_p]
    lib.vr_sched_host_frame.argtypes = [C.c_void_p]
    lib.vr_sched_host_synchronize.argtypes = [C.c_void_p]
    lib.vr_sched_host_destroy.argtypes = [C.c_void_p]
    return lib


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scene(W, H, k):
    import pyoracle
    import synth
    import vr_amd
    vol = synth.gaussians_numpy((16, 14, 12), seed=5)
    cam = vr_amd.make_camera(radius=2.0, rotate=(40.0 + 53.0 * k, 20.0 - 17.0 * k)).to_vr_camera()
    return pyoracle.Scene.from_params(vol, float(vol.min()), float(vol.max()), synth.tf_color(),
                                      cam, W, H, vr_amd.default_params(shading=1))


def _worker(rank, world, port, W, H, rb, inflight, nframes, q):
    import sys
    for sub in ("volumetric-renderer_amd", "oracle", "tools"):
        sys.path.insert(0, os.path.join(ROOT, sub))
    import vr_dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rows = vr_dist.shard_global_rows(H, rb, rank, world)
        sr = len(rows)
        shards = [torch.zeros((sr, W, 4), dtype=torch.float32) for _ in range(inflight)]
        gbufs = [torch.zeros((world, sr, W, 4), dtype=torch.float32) if rank == 0 else None
                 for _ in range(inflight)]
        frame_buf = np.full((H, W, 4), np.nan, np.float32)  # rank 0's frame_dev, reused
        consumed, log, errors = [], [], []
        lock = threading.Lock()
        rng = np.random.default_rng(100 + rank)
        delays = rng.uniform(0.0, 0.02, size=(nframes, 4))

        def op_fn(_user, op, slot, frame):
            t0 = time.monotonic_ns()
            try:
                if op == 0:  # render this rank's row blocks of frame `frame` into the slot shard
                    time.sleep(delays[frame, 0])
                    img, _ = _scene(W, H, frame).render_rows(rows[rows >= 0], nthreads=1)
                    sh = np.zeros((sr, W, 4), np.float32)
                    sh[rows >= 0] = img[rows[rows >= 0]]
                    shards[slot].copy_(torch.from_numpy(sh))
                elif op == 1:  # the collective: gather the slot's shard to rank 0 (ncclGather)
                    time.sleep(delays[frame, 1])
                    views = [gbufs[slot][r] for r in range(world)] if rank == 0 else None
                    dist.gather(shards[slot], views, dst=0)
                elif op == 2:  # rank 0: de-interleave into the single frame buffer
                    time.sleep(delays[frame, 2])
                    frame_buf[:] = vr_dist.assemble_numpy(gbufs[slot].numpy(), H, rb, world)
                elif op == 3:  # the caller's use of the finished frame
                    if rank == 0:
                        consumed.append((frame, frame_buf.copy()))
                    time.sleep(delays[frame, 3])
            except Exception as e:  # reported by the test, never across the C boundary
                errors.append(repr(e))
                return -5
            with lock:
                log.append((op, slot, frame, t0, time.monotonic_ns()))
            return 0

        cb = CB(op_fn)
        lib = _lib()
        h = lib.vr_sched_host_create(rank, inflight, cb, None)
        assert h
        for _ in range(nframes):
            assert lib.vr_sched_host_frame(h) == 0
        rc = lib.vr_sched_host_synchronize(h)
        lib.vr_sched_host_destroy(h)
        q.put((rank, rc, errors, log, consumed))
    finally:
        dist.destroy_process_group()


def _check_order(rank, log, inflight, nframes, consume=True):
    ev = {(OPS[op], fr): (t0, t1) for op, _, fr, t0, t1 in log}
    for i in range(nframes):
        assert ev[("gather", i)][0] >= ev[("render", i)][1], ("gather before render", i)
        if i:
            assert ev[("gather", i)][0] >= ev[("gather", i - 1)][1], ("gathers out of order", i)
        if rank == 0:
            assert ev[("assemble", i)][0] >= ev[("gather", i)][1], ("assemble before gather", i)
            assert ev[("consume", i)][0] >= ev[("assemble", i)][1], ("consume before assemble", i)
            if i:  # the caller's reading of frame i-1 precedes frame i's write
                assert ev[("assemble", i)][0] >= ev[("consume", i - 1)][1], ("frame overwritten", i)
        else:
            # rank r > 0 only enqueues its shard: its caller's stream is not ordered after the
            # frame (vr_frame_schedule.h, round 6; vr_dist_synchronize waits for it)
            assert ("assemble", i) not in ev
            if not consume:  # a multi-device context's other members: nothing consumes their frames
                assert ("consume", i) not in ev
        if i >= inflight:  # slot reuse: frame i renders only after frame i-F freed the slot
            freed = ev[("assemble" if rank == 0 else "gather", i - inflight)][1]
            assert ev[("render", i)][0] >= freed, ("slot reused early", i)


@pytest.mark.parametrize("world,rb,inflight,nframes", [(2, 8, 3, 7), (2, 4, 1, 3), (3, 16, 2, 5)])
def test_host_schedule_frames_and_order(world, rb, inflight, nframes):
    W, H = 36, 41
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, H, rb, inflight, nframes, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, rc, errors, log, consumed = q.get(timeout=180)
        res[rank] = (rc, errors, log, consumed)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, (rc, errors, log, consumed) in res.items():
        assert rc == 0 and not errors, (rank, rc, errors)
        _check_order(rank, log, inflight, nframes)
    consumed = res[0][3]
    assert [f for f, _ in consumed] == list(range(nframes))
    for k, img in consumed:
        full, _ = _scene(W, H, k).render()
        assert np.array_equal(img, full), k


@pytest.mark.parametrize("rank,inflight", [(0, 1), (0, 3), (1, 1), (1, 3), (2, 8)])
def test_schedule_edges_per_frame(rank, inflight):
    """The host cost of a frame is mostly its cross-stream edges (an event record ~2.4 us and a
    stream wait ~3.7 us against pending events on MI355X, tools/host_cost.cpp): the schedule
    issues 2 records + 2 waits per frame on rank 0 (the first F frames skip the slot-reuse wait)
    and 1 + 1 on the other ranks (the first frame has no previous gather to follow)."""
    lib = _lib()
    lib.vr_sched_host_edges.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    cb = CB(lambda _u, _op, _slot, _frame: 0)
    h = lib.vr_sched_host_create(rank, inflight, cb, None)
    n = 12
    for _ in range(n):
        assert lib.vr_sched_host_frame(h) == 0
    assert lib.vr_sched_host_synchronize(h) == 0
    rec, wai = C.c_uint64(), C.c_uint64()
    assert lib.vr_sched_host_edges(h, C.byref(rec), C.byref(wai)) == 0
    lib.vr_sched_host_destroy(h)
    if rank == 0:
        assert (rec.value, wai.value) == (2 * n, n + (n - inflight))
    else:
        assert (rec.value, wai.value) == (n, (n - 1) if inflight > 1 else 0)


def test_host_schedule_propagates_callback_errors():
    """A failing op (here the render of frame 1) surfaces from synchronize; records and waits
    still run, so the other streams drain instead of deadlocking."""
    lib = _lib()

    def op_fn(_u, op, _slot, frame):
        return -5 if (op == 0 and frame == 1) else 0

    cb = CB(op_fn)
    h = lib.vr_sched_host_create(0, 2, cb, None)
    for _ in range(4):
        assert lib.vr_sched_host_frame(h) == 0
    assert lib.vr_sched_host_synchronize(h) == -5
    lib.vr_sched_host_destroy(h)
    assert not lib.vr_sched_host_create(0, 0, cb, None)


GCB = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_uint64)


def _glib():
    lib = C.CDLL(LIB)
    lib.vr_group_host_create.restype = C.c_void_p
    lib.vr_group_host_create.argtypes = [C.c_int, C.c_int, GCB, C.c_void_p]
    lib.vr_group_host_frame.argtypes = [C.c_void_p]
    lib.vr_group_host_synchronize.argtypes = [C.c_void_p]
    lib.vr_group_host_destroy.argtypes = [C.c_void_p]
    return lib


@pytest.mark.parametrize("members,inflight,nframes,share",
                         [(2, 3, 7, (1, 1)), (3, 2, 5, (1, 1)), (3, 1, 3, (1, 1)), (1, 2, 3, (1, 1)),
                          (8, 3, 6, (1, 1)), (8, 1, 3, (1, 1)), (8, 3, 4, (7, 8)), (3, 2, 4, (1, 3)),
                          (4, 2, 3, (3, 1))])
def test_group_schedule_one_process(members, inflight, nframes, share):
    """A multi-device context (vr_create_mask) in ONE process: vr_frame_workers.h issues every
    frame on N members -- member 0 on the calling thread, the others on worker threads -- each
    member running the same FrameSchedule as vr_dist (vr_dist.cpp group_render).  Here the
    members' streams are host threads, the render is the CPU oracle on the member's 8-row blocks,
    the gather a host rendezvous standing in for ncclGather, the rows split by the row share
    (vr_set_row_share: w0 blocks for member 0 per w0 + (N - 1) w).  Every frame the caller consumes
    equals the oracle's single-device frame bit for bit, and each member's op log honours the
    schedule (slot reuse, gather order, assembly after the caller consumed the previous frame)."""
    import sys
    for sub in ("volumetric-renderer_amd", "oracle", "tools"):
        sys.path.insert(0, os.path.join(ROOT, sub))
    import vr_dist
    W, H, rb = 36, 41, 8
    rows = [vr_dist.shard_global_rows(H, rb, m, members, share) for m in range(members)]
    sr = len(rows[0])
    shards = [[np.zeros((sr, W, 4), np.float32) for _ in range(inflight)] for _ in range(members)]
    gbufs = [np.zeros((members, sr, W, 4), np.float32) for _ in range(inflight)]
    frame_buf = np.full((H, W, 4), np.nan, np.float32)
    consumed, errors = [], []
    logs = [[] for _ in range(members)]
    cond = threading.Condition()
    deposits = {}
    rng = np.random.default_rng(7)
    delays = rng.uniform(0.0, 0.01, size=(members, nframes, 4))

    def op_fn(_user, m, op, slot, frame):
        if op >= 4:  # OP_ABORT / OP_ISSUE hooks: nothing fails here
            return 0
        t0 = time.monotonic_ns()
        try:
            time.sleep(delays[m, frame, op])
            if op == 0:
                r = rows[m]
                img, _ = _scene(W, H, frame).render_rows(r[r >= 0], nthreads=1)
                sh = np.zeros((sr, W, 4), np.float32)
                sh[r >= 0] = img[r[r >= 0]]
                shards[m][slot][:] = sh
            elif op == 1:  # the collective: every member's shard to member 0
                with cond:
                    deposits[(frame, m)] = shards[m][slot].copy()
                    cond.notify_all()
                    if m == 0:
                        cond.wait_for(lambda: all((frame, k) in deposits for k in range(members)),
                                      timeout=60)
                        for k in range(members):
                            gbufs[slot][k] = deposits.pop((frame, k))
            elif op == 2:
                frame_buf[:] = vr_dist.assemble_numpy(gbufs[slot], H, rb, members, share)
            elif op == 3:
                consumed.append((frame, frame_buf.copy()))
        except Exception as e:  # reported by the test, never across the C boundary
            errors.append(repr(e))
            return -5
        logs[m].append((op, slot, frame, t0, time.monotonic_ns()))
        return 0

    cb = GCB(op_fn)
    lib = _glib()
    g = lib.vr_group_host_create(members, inflight, cb, None)
    assert g
    for _ in range(nframes):
        assert lib.vr_group_host_frame(g) == 0
    rc = lib.vr_group_host_synchronize(g)
    lib.vr_group_host_destroy(g)
    assert rc == 0 and not errors, (rc, errors)
    for m in range(members):
        _check_order(m, logs[m], inflight, nframes, consume=(m == 0))
    assert [f for f, _ in consumed] == list(range(nframes))
    for k, img in consumed:
        full, _ = _scene(W, H, k).render()
        assert np.array_equal(img, full), k


def test_group_schedule_reports_member_errors():
    """A member's failing op surfaces from synchronize (the worker's sticky error), and every
    member's streams still drain."""
    lib = _glib()

    def op_fn(_u, m, op, _slot, frame):
        return -5 if (m == 2 and op == 0 and frame == 1) else 0

    cb = GCB(op_fn)
    g = lib.vr_group_host_create(3, 2, cb, None)
    for _ in range(4):
        assert lib.vr_group_host_frame(g) == 0
    assert lib.vr_group_host_synchronize(g) == -5
    lib.vr_group_host_destroy(g)
    assert not lib.vr_group_host_create(0, 2, cb, None)


class _Rendezvous:
    """A collective with real matching, standing in for ncclGather: member m's gather of frame f
    returns only once every member posted frame f, or fails once the group is aborted (the
    stand-in for ncclCommAbort ending pending collectives)."""

    def __init__(self, members):
        self.members = members
        self.cond = threading.Condition()
        self.posted = {}
        self.aborted = False
        self.abort_calls = []

    def gather(self, m, frame):
        with self.cond:
            self.posted.setdefault(frame, set()).add(m)
            self.cond.notify_all()
            ok = self.cond.wait_for(
                lambda: self.aborted or len(self.posted[frame]) == self.members, timeout=60)
            assert ok, "collective hung (no abort)"
            return -5 if len(self.posted[frame]) < self.members else 0

    def abort(self, m):
        with self.cond:
            self.abort_calls.append(m)
            self.aborted = True
            self.cond.notify_all()


@pytest.mark.parametrize("members,fail_member,fail_frame", [(3, 2, 1), (8, 5, 2), (8, 0, 1)])
def test_group_member_issue_failure_aborts_collectives(members, fail_member, fail_frame):
    """a member whose issue fails never posts its gather, so its peers' gathers of
    that frame can never match and would block their streams forever.  The frame workers'
    settle() aborts every communicator (OP_ABORT, ncclCommAbort in vr_dist.cpp) before any
    stream is synchronised: synchronize returns the member's error in bounded time, and the
    context refuses further frames."""
    lib = _glib()
    rv = _Rendezvous(members)

    def op_fn(_u, m, op, _slot, frame):
        if op == 5:  # OP_ISSUE: the failing member's enqueue of frame fail_frame fails
            return -5 if (m == fail_member and frame == fail_frame) else 0
        if op == 4:
            rv.abort(m)
            return 0
        if op == 1:
            return rv.gather(m, frame)
        return 0

    cb = GCB(op_fn)
    g = lib.vr_group_host_create(members, 2, cb, None)
    t0 = time.monotonic()
    rcs = [lib.vr_group_host_frame(g) for _ in range(4)]
    rc = lib.vr_group_host_synchronize(g)
    assert time.monotonic() - t0 < 30
    assert rc == -5
    assert sorted(rv.abort_calls) == list(range(members))  # every communicator, once
    if fail_member == 0:  # member 0's issue fails on the caller's thread: reported at once
        assert rcs[fail_frame] == -5
    assert lib.vr_group_host_frame(g) != 0  # aborted: no further frames
    assert lib.vr_group_host_synchronize(g) == -5
    assert sorted(rv.abort_calls) == list(range(members))  # abort ran once only
    lib.vr_group_host_destroy(g)


@pytest.mark.parametrize("H,rb", [(53, 1), (1080, 8), (1080, 16), (7, 4), (4096, 8)])
@pytest.mark.parametrize("nranks", [1, 2, 3, 8])
@pytest.mark.parametrize("share", [(1, 1), (1, 2), (3, 4), (2, 1), (7, 8), (64, 1)])
def test_row_share_maps_every_row_once(H, rb, nranks, share):
    """The weighted block-cyclic split (vr_internal.h RowShare, restated in vr_dist.py): every
    frame row belongs to exactly one rank, shards are padded to the largest share, and the
    assembly inverts the shards; (1, 1) is the plain block-cyclic split of SURVEY.md 8e."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "volumetric-renderer_amd"))
    import vr_amd
    import vr_dist
    sr = vr_dist.shard_rows(H, rb, nranks, share)
    if share == (1, 1):
        assert sr == vr_amd.shard_rows(H, rb, nranks)
    rows = [vr_dist.shard_global_rows(H, rb, r, nranks, share) for r in range(nranks)]
    owned = np.concatenate([x[x >= 0] for x in rows])
    assert sorted(owned.tolist()) == list(range(H))
    assert max(int((x >= 0).sum()) for x in rows) <= sr
    g = np.stack(rows)
    assert np.array_equal(vr_dist.assemble_numpy(g, H, rb, nranks, share), np.arange(H))
