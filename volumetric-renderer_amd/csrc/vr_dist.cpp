// vr_dist.cpp — multi-GPU frames over RCCL (include/vr/vr_dist.h).
//
// Sort-first image tiling: each rank ray-marches its row blocks through the
// public vr.h entry points, one ncclGather per frame collects the shards on rank 0 over xGMI,
// and rank 0 de-interleaves them.  The whole frame is stream-ordered (vr_frame_schedule.h):
//
//   rank 0    slot stream k : [wait gathered_k] render shard_k ─► [rendered_k]
//             caller stream : wait rendered_k ─► ncclGather ─► assemble ─► [gathered_k]
//   rank r>0  slot stream k : render shard_k ─► wait gathered_(k-1) ─► ncclGather ─► [gathered_k]
//
// Frame i takes slot i mod F, so F frames are in flight and consecutive renders overlap on the
// device; the gathers run one at a time in frame order, which every rank issues identically.
//
// RCCL is resolved with dlopen at creation (the librccl.so.1 already loaded, e.g. PyTorch's,
// else the system one), so single-GPU users of the library never load it.
#include "vr/vr_dist.h"

#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include "vr_frame_schedule.h"
#include "vr_frame_workers.h"
#include "vr_group.h"

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

namespace {

thread_local std::string g_dist_err;

struct Rccl {
    bool ok = false;
    std::string err;
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_init_all)(ncclComm_t *, int, const int *) = nullptr;
    ncclResult_t (*gather)(const void *, void *, size_t, ncclDataType_t, int, ncclComm_t,
                           hipStream_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
};

template <typename F>
bool bind(void *h, const char *name, F &fn)
{
    fn = reinterpret_cast<F>(dlsym(h, name));
    return fn != nullptr;
}

Rccl load_rccl()
{
    Rccl r;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // already in the process
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
        const char *e = dlerror();
        r.err = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
        return r;
    }
    if (!bind(h, "ncclGetUniqueId", r.get_unique_id) ||
        !bind(h, "ncclCommInitRank", r.comm_init_rank) || !bind(h, "ncclGather", r.gather) ||
        !bind(h, "ncclCommInitAll", r.comm_init_all) ||
        !bind(h, "ncclCommDestroy", r.comm_destroy) ||
        !bind(h, "ncclCommAbort", r.comm_abort) ||
        !bind(h, "ncclGetErrorString", r.error_string)) {
        r.err = "librccl.so.1 lacks ncclGather/ncclCommInitRank/ncclCommInitAll/ncclCommAbort/...";
        return r;
    }
    r.ok = true;
    return r;
}

Rccl &rccl()
{
    static Rccl r = load_rccl();
    return r;
}

struct Buffers {
    void *shard = nullptr;  // shard_rows x W pixels (RGBA8, or RGBA32F in multi-device contexts)
    void *gbuf = nullptr;   // rank 0: nranks shards, rank-major
    hipEvent_t xev = nullptr;  // copy exchange: member > 0 shard ready / member 0 copies done
};

// The copy exchange of a multi-device context (vr_debug_create_members, VR_EXCHANGE_COPY):
// the frame's gather as device-to-device copies that member 0 enqueues on its communication
// stream, for members that RCCL cannot put in one communicator (the same device twice: the
// one-GPU rehearsal of the multi-device path) or when RCCL is absent.  Per frame f and slot k:
//   member m > 0 : [its comm stream, after rendered_k] record xev_k; publish sent[m] = f + 1;
//                  host-wait copied > f; its comm stream waits member 0's xev_k (the copy read
//                  its shard, so the slot may be reused after gathered_k)
//   member 0     : copy its own shard; for every m: host-wait sent[m] > f, wait m's xev_k,
//                  copy m's shard into gbuf_k + m * shard; record xev_k; publish copied = f + 1
// A stream only ever waits on an event recorded (and published) before: nothing on a device
// can wait for a record that never comes.  Slot events are re-recorded F frames later, only
// after every waiter has enqueued its wait (the host waits above order them).  A member that
// fails sets `aborted`, which ends every host wait with VR_EIO.
struct CopyExchange {
    std::mutex m;
    std::condition_variable cv;
    std::vector<uint64_t> sent;   // per member: frames whose shard-ready event is recorded
    uint64_t copied = 0;          // frames whose copies member 0 has enqueued
    bool aborted = false;
    std::vector<vr_dist *> peers;  // the members' pipelines (member order)

    void abort()
    {
        {
            std::lock_guard<std::mutex> g(m);
            aborted = true;
        }
        cv.notify_all();
    }
    // Waits until pred() holds (true) or the exchange is aborted (false).  No time limit: a
    // member held up in its enqueue (e.g. building a derived structure for a large volume) is
    // slow, not failed, and a failing member aborts the exchange, which wakes every waiter
    // (a 120 s limit used to fail a healthy context for good).
    template <class P>
    bool wait(P pred)
    {
        std::unique_lock<std::mutex> g(m);
        cv.wait(g, [&] { return aborted || pred(); });
        return !aborted;
    }
};

// Timing pairs (vr_dist_timing_enable): recorded per frame on the op's stream, read and freed
// by vr_dist_timing_read.
struct TimedOp {
    hipEvent_t t0 = nullptr, t1 = nullptr;
    bool closed = false;  // t1 recorded
};

// HIP + RCCL executor of vr::sched::FrameSchedule (members defined below vr_dist).
struct HipExec {
    using Stream = hipStream_t;
    using Event = hipEvent_t;
    vr_dist *d = nullptr;
    int record(Event e, Stream s);
    int wait(Stream s, Event e);
    int render(int slot, uint64_t frame, Stream s);
    int gather(int slot, uint64_t frame, Stream s);
    int assemble(int slot, uint64_t frame, void *frame_dev, Stream s);
};

}  // namespace

struct vr_dist {
    vr_ctx *ctx = nullptr;
    bool fences_registered = false;  // the slot streams' events are ctx's frame fences
    int device = 0;
    int nranks = 1, rank = 0;
    uint32_t row_block = 8, width = 0, height = 0, shard_rows = 0;
    ncclComm_t comm = nullptr;
    bool owns_comm = true;  // false: a multi-device context's communicator (vr_group.h)
    CopyExchange *xch = nullptr;  // not null: the copy exchange replaces ncclGather
    uint32_t share_w0 = 1, share_w = 1;  // the row share shard_rows was sized for
    int out_format = VR_OUT_RGBA8;
    uint32_t words_per_pixel = 1;  // 32-bit words a pixel of out_format takes (gather count)
    std::vector<Buffers> bufs;  // per slot
    vr::sched::FrameSchedule<HipExec> sched;
    const vr_camera *cam = nullptr;  // the frame being issued
    const vr_params *params = nullptr;
    bool timing = false;
    std::vector<TimedOp> t_render, t_gather, t_assemble;
    bool hprof = false;       // host profiling (vr_dist_host_profile_enable)
    vr_dist_host_profile hp{};
    std::string err;
};

namespace {

int dfail(vr_dist *d, int code, const std::string &msg)
{
    if (d)
        d->err = msg;
    else
        g_dist_err = msg;
    return code;
}

int hip_check(vr_dist *d, hipError_t e, const char *what)
{
    if (e == hipSuccess) return VR_OK;
    (void)hipGetLastError();  // reported here: not left for the next launch check to find
    return dfail(d, e == hipErrorOutOfMemory ? VR_ENOMEM : VR_EIO,
                 std::string(what) + ": " + hipGetErrorString(e));
}

int nccl_check(vr_dist *d, ncclResult_t r, const char *what)
{
    if (r == ncclSuccess) return VR_OK;
    return dfail(d, VR_EIO, std::string(what) + ": " + rccl().error_string(r));
}

#define DTRY(expr)                  \
    do {                            \
        int _rc = (expr);           \
        if (_rc != VR_OK) return _rc; \
    } while (0)

// With timing on, a pair of timing events brackets the op on its stream.  At most
// kMaxTimedFrames pairs per op are kept between reads: later frames go untimed (the count
// vr_dist_timing_read returns is the number actually timed), so timing left on without reads
// holds a bounded number of events.
constexpr size_t kMaxTimedFrames = 1u << 16;
// The op failed after timed_begin: drop its unfinished pair (a later read must not wait on an
// event that was never recorded).
void timed_abort(vr_dist *d, std::vector<TimedOp> &v)
{
    if (!d->timing || v.empty() || v.back().closed) return;
    hipEventDestroy(v.back().t0);
    hipEventDestroy(v.back().t1);
    v.pop_back();
}
int timed_begin(vr_dist *d, std::vector<TimedOp> &v, hipStream_t s)
{
    if (!d->timing || v.size() >= kMaxTimedFrames) return VR_OK;
    TimedOp t;
    // timing-only events: no system-scope cache writeback/invalidate when recorded
    DTRY(hip_check(d, hipEventCreateWithFlags(&t.t0, hipEventDisableSystemFence), "hipEventCreate"));
    if (hipEventCreateWithFlags(&t.t1, hipEventDisableSystemFence) != hipSuccess) {
        hipEventDestroy(t.t0);
        return dfail(d, VR_EIO, "hipEventCreate");
    }
    v.push_back(t);
    if (hipEventRecord(t.t0, s) != hipSuccess) {
        timed_abort(d, v);
        return dfail(d, VR_EIO, "hipEventRecord");
    }
    return VR_OK;
}
int timed_end(vr_dist *d, std::vector<TimedOp> &v, hipStream_t s)
{
    if (!d->timing || v.empty() || v.back().closed) return VR_OK;
    v.back().closed = true;
    if (hipEventRecord(v.back().t1, s) != hipSuccess) {
        timed_abort(d, v);
        return dfail(d, VR_EIO, "hipEventRecord");
    }
    return VR_OK;
}

// Host-time accumulator of one step of the frame path (only when d->hprof).
struct HostSpan {
    double *acc;
    std::chrono::steady_clock::time_point t0;
    explicit HostSpan(vr_dist *d, double vr_dist_host_profile::*field)
        : acc(d->hprof ? &(d->hp.*field) : nullptr)
    {
        if (acc) t0 = std::chrono::steady_clock::now();
    }
    ~HostSpan()
    {
        if (acc)
            *acc += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0)
                        .count();
    }
};

int HipExec::record(Event e, Stream s)
{
    HostSpan h(d, &vr_dist_host_profile::record_us);
    return hip_check(d, hipEventRecord(e, s), "hipEventRecord");
}
int HipExec::wait(Stream s, Event e)
{
    HostSpan h(d, &vr_dist_host_profile::wait_us);
    return hip_check(d, hipStreamWaitEvent(s, e, 0), "hipStreamWaitEvent");
}
int HipExec::render(int slot, uint64_t, Stream s)
{
    HostSpan h(d, &vr_dist_host_profile::render_us);
    vr_params q = *d->params;
    q.frames_in_flight = (int32_t)d->sched.slots.size();
    DTRY(timed_begin(d, d->t_render, s));
    if (vr_render_device(d->ctx, d->cam, &q, d->bufs[slot].shard, d->out_format, d->row_block,
                         (uint32_t)d->rank, (uint32_t)d->nranks, s) != VR_OK) {
        timed_abort(d, d->t_render);
        return dfail(d, VR_EIO, std::string("render: ") + vr_last_error(d->ctx));
    }
    return timed_end(d, d->t_render, s);
}
size_t shard_bytes(const vr_dist *d)
{
    return (size_t)d->shard_rows * d->width * 4 * d->words_per_pixel;
}

int copy_gather(vr_dist *d, int slot, uint64_t frame, hipStream_t s)
{
    CopyExchange &x = *d->xch;
    Buffers &b = d->bufs[slot];
    const size_t bytes = shard_bytes(d);
    if (d->rank != 0) {
        DTRY(hip_check(d, hipEventRecord(b.xev, s), "hipEventRecord(shard ready)"));
        {
            std::lock_guard<std::mutex> g(x.m);
            x.sent[d->rank] = frame + 1;
        }
        x.cv.notify_all();
        if (!x.wait([&] { return x.copied > frame; }))
            return dfail(d, VR_EIO, "copy exchange: member 0 did not copy frame " +
                                        std::to_string(frame) + " (aborted)");
        return hip_check(d, hipStreamWaitEvent(s, x.peers[0]->bufs[slot].xev, 0),
                         "hipStreamWaitEvent(copies done)");
    }
    char *dst = static_cast<char *>(b.gbuf);
    DTRY(hip_check(d, hipMemcpyAsync(dst, b.shard, bytes, hipMemcpyDeviceToDevice, s),
                   "hipMemcpyAsync(own shard)"));
    for (int m = 1; m < d->nranks; ++m) {
        if (!x.wait([&] { return x.sent[m] > frame; }))
            return dfail(d, VR_EIO, "copy exchange: member " + std::to_string(m) +
                                        " did not render frame " + std::to_string(frame) +
                                        " (aborted)");
        vr_dist *p = x.peers[m];
        DTRY(hip_check(d, hipStreamWaitEvent(s, p->bufs[slot].xev, 0),
                       "hipStreamWaitEvent(shard ready)"));
        const hipError_t e =
            p->device == d->device
                ? hipMemcpyAsync(dst + (size_t)m * bytes, p->bufs[slot].shard, bytes,
                                 hipMemcpyDeviceToDevice, s)
                : hipMemcpyPeerAsync(dst + (size_t)m * bytes, d->device, p->bufs[slot].shard,
                                     p->device, bytes, s);
        DTRY(hip_check(d, e, "copy exchange (shard copy)"));
    }
    DTRY(hip_check(d, hipEventRecord(b.xev, s), "hipEventRecord(copies done)"));
    {
        std::lock_guard<std::mutex> g(x.m);
        x.copied = frame + 1;
    }
    x.cv.notify_all();
    return VR_OK;
}

int HipExec::gather(int slot, uint64_t frame, Stream s)
{
    HostSpan h(d, &vr_dist_host_profile::gather_us);
    const Buffers &b = d->bufs[slot];
    DTRY(timed_begin(d, d->t_gather, s));
    if (d->xch) {
        const int rc = copy_gather(d, slot, frame, s);
        if (rc != VR_OK) {
            timed_abort(d, d->t_gather);
            return rc;
        }
        return timed_end(d, d->t_gather, s);
    }
    const int rc = nccl_check(d, rccl().gather(b.shard, d->rank == 0 ? b.gbuf : nullptr,
                                               (size_t)d->shard_rows * d->width * d->words_per_pixel,
                                               ncclUint32, 0,
                                               d->comm, s),
                              "ncclGather");
    if (rc != VR_OK) {
        timed_abort(d, d->t_gather);
        return rc;
    }
    return timed_end(d, d->t_gather, s);
}
int HipExec::assemble(int slot, uint64_t, void *frame_dev, Stream s)
{
    HostSpan h(d, &vr_dist_host_profile::assemble_us);
    DTRY(timed_begin(d, d->t_assemble, s));
    if (vr_assemble_rows(d->ctx, d->bufs[slot].gbuf, frame_dev, d->out_format, d->row_block,
                         (uint32_t)d->nranks, s) != VR_OK) {
        timed_abort(d, d->t_assemble);
        return dfail(d, VR_EIO, std::string("assemble: ") + vr_last_error(d->ctx));
    }
    return timed_end(d, d->t_assemble, s);
}

void free_timing(vr_dist *d)
{
    for (auto *v : {&d->t_render, &d->t_gather, &d->t_assemble}) {
        for (auto &t : *v) {
            hipEventDestroy(t.t0);
            hipEventDestroy(t.t1);
        }
        v->clear();
    }
}

// Summed span of each timed op since the last read (render, gather, assemble) and the frames
// timed; the record is cleared (on failure too).
int timing_read3(vr_dist *d, double ms[3], uint64_t *frames)
{
    DTRY(vr_dist_synchronize(d));
    int i = 0, rc = VR_OK;
    for (auto *v : {&d->t_render, &d->t_gather, &d->t_assemble}) {
        ms[i] = 0.0;
        for (auto &t : *v) {
            float x = 0.0f;
            if (rc == VR_OK)
                rc = hip_check(d, hipEventElapsedTime(&x, t.t0, t.t1), "hipEventElapsedTime");
            ms[i] += x;
        }
        ++i;
    }
    if (frames) *frames = d->t_render.size();
    free_timing(d);
    return rc;
}

void release(vr_dist *d)
{
    hipSetDevice(d->device);
    auto &S = d->sched;
    for (auto &s : S.slots)
        if (s.stream) hipStreamSynchronize(s.stream);
    // rank 0's gathers and assemblies ran on the callers' streams
    if (hipEvent_t e = S.last_gathered()) hipEventSynchronize(e);
    if (d->fences_registered)
        for (auto &s : S.slots) vr::unregister_stream_fence(d->ctx, s.stream);
    d->fences_registered = false;
    // the context's kernel-timing events on the slot streams, before the streams go
    vr::settle_timing(d->ctx);
    if (d->comm && d->owns_comm) rccl().comm_destroy(d->comm);
    free_timing(d);
    for (auto &b : d->bufs) {
        if (b.shard) hipFree(b.shard);
        if (b.gbuf) hipFree(b.gbuf);
        if (b.xev) hipEventDestroy(b.xev);
    }
    for (auto &s : S.slots) {
        for (hipEvent_t e : {s.rendered, s.gathered})
            if (e) hipEventDestroy(e);
        if (s.stream) hipStreamDestroy(s.stream);
    }
    S.slots.clear();
    d->bufs.clear();
}

// Join the communicator of `id` (vr_dist_create), adopt `comm` (multi-device contexts) or use
// the copy exchange (d->xch set), then allocate the slots.
int setup(vr_dist *d, const void *id, ncclComm_t comm, int frames)
{
    DTRY(hip_check(d, hipSetDevice(d->device), "hipSetDevice"));
    if (d->xch) {
        d->owns_comm = false;
    } else if (comm) {
        d->comm = comm;
        d->owns_comm = false;
    } else {
        ncclUniqueId uid;
        static_assert(sizeof(uid) == VR_DIST_ID_BYTES, "ncclUniqueId size");
        std::memcpy(&uid, id, sizeof(uid));
        DTRY(nccl_check(d, rccl().comm_init_rank(&d->comm, d->nranks, uid, d->rank),
                        "ncclCommInitRank"));
    }
    auto &S = d->sched;
    S.rank = d->rank;
    const size_t sbytes = shard_bytes(d);
    S.slots.resize(frames);
    d->bufs.resize(frames);
    for (int k = 0; k < frames; ++k) {
        auto &s = S.slots[k];
        auto &b = d->bufs[k];
        DTRY(hip_check(d, hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking),
                       "hipStreamCreate(slot)"));
        DTRY(hip_check(d, hipMalloc(&b.shard, sbytes), "hipMalloc(shard)"));
        if (d->rank == 0)
            DTRY(hip_check(d, hipMalloc(&b.gbuf, sbytes * d->nranks), "hipMalloc(gather)"));
        if (d->xch)
            DTRY(hip_check(d, hipEventCreateWithFlags(&b.xev, hipEventDisableTiming),
                           "hipEventCreate(exchange)"));
        for (hipEvent_t *e : {&s.rendered, &s.gathered})
            DTRY(hip_check(d, hipEventCreateWithFlags(e, hipEventDisableTiming), "hipEventCreate"));
    }
    // the event recorded on a slot stream after each of its renders (rank 0: rendered, after the
    // render; rank r > 0: gathered, after the render and the gather) is the context's frame
    // fence there: the context records none of its own (vr_group.h)
    for (auto &s : S.slots)
        DTRY(vr::register_stream_fence(d->ctx, s.stream, d->rank == 0 ? s.rendered : s.gathered));
    d->fences_registered = true;
    return VR_OK;
}

}  // namespace

extern "C" {

int vr_dist_unique_id(void *id_out)
{
    if (!id_out) return dfail(nullptr, VR_EINVAL, "id_out is NULL");
    if (!rccl().ok) return dfail(nullptr, VR_ENODEV, rccl().err);
    ncclUniqueId uid;
    int rc = nccl_check(nullptr, rccl().get_unique_id(&uid), "ncclGetUniqueId");
    if (rc) return rc;
    std::memcpy(id_out, &uid, sizeof(uid));
    return VR_OK;
}

}  // extern "C"

namespace {

vr_dist *dist_create(vr_ctx *ctx, const void *id, ncclComm_t comm, int nranks, int rank,
                     uint32_t row_block, int frames_in_flight, int out_format,
                     CopyExchange *xch = nullptr)
{
    if (nranks < 1 || rank < 0 || rank >= nranks || row_block == 0 || frames_in_flight < 1 ||
        frames_in_flight > 8) {
        dfail(nullptr, VR_EINVAL, "bad nranks/rank/row_block/frames_in_flight");
        return nullptr;
    }
    if (!xch && !rccl().ok) {
        dfail(nullptr, VR_ENODEV, rccl().err);
        return nullptr;
    }
    vr_dist *d = new (std::nothrow) vr_dist();
    if (!d) {
        dfail(nullptr, VR_ENOMEM, "out of host memory");
        return nullptr;
    }
    d->ctx = ctx;
    d->nranks = nranks;
    d->rank = rank;
    d->row_block = row_block;
    d->out_format = out_format;
    d->words_per_pixel = out_format == VR_OUT_RGBA32F ? 4 : 1;
    d->xch = xch;
    if (vr_get_device(ctx, &d->device) != VR_OK || vr_get_size(ctx, &d->width, &d->height) != VR_OK ||
        vr_get_row_share(ctx, &d->share_w0, &d->share_w) != VR_OK) {
        dfail(nullptr, VR_EINVAL, "bad ctx");
        delete d;
        return nullptr;
    }
    d->shard_rows = vr_shard_rows_ctx(ctx, d->height, row_block, (uint32_t)nranks);
    if (setup(d, id, comm, frames_in_flight) != VR_OK) {
        g_dist_err = d->err;
        release(d);
        delete d;
        return nullptr;
    }
    return d;
}

}  // namespace

extern "C" {

vr_dist *vr_dist_create(vr_ctx *ctx, const void *id, int nranks, int rank, uint32_t row_block,
                        int frames_in_flight)
{
    if (!ctx || !id) {
        dfail(nullptr, VR_EINVAL, "ctx or id is NULL");
        return nullptr;
    }
    if (vr::is_multi_device(ctx)) {
        dfail(nullptr, VR_EINVAL,
              "a multi-device context (vr_create_mask) distributes its own frames");
        return nullptr;
    }
    return dist_create(ctx, id, nullptr, nranks, rank, row_block, frames_in_flight, VR_OUT_RGBA8);
}

int vr_dist_render(vr_dist *d, const vr_camera *cam, const vr_params *p, void *frame_dev,
                   void *stream)
{
    if (!d) return dfail(nullptr, VR_EINVAL, "dist is NULL");
    HostSpan total(d, &vr_dist_host_profile::total_us);
    if (!cam || !p) return dfail(d, VR_EINVAL, "camera or params is NULL");
    if (d->rank == 0 && !frame_dev) return dfail(d, VR_EINVAL, "rank 0 needs frame_dev");
    uint32_t w = 0, h = 0, s0 = 1, s1 = 1;
    if (vr_get_size(d->ctx, &w, &h) != VR_OK || w != d->width || h != d->height)
        return dfail(d, VR_EINVAL, "the context was resized: create a new vr_dist");
    // the shard buffers, the gather count and the assembly stride were sized for the row share
    // in force at creation: a rank whose share grew would write past its shard
    if (vr_get_row_share(d->ctx, &s0, &s1) != VR_OK || s0 != d->share_w0 || s1 != d->share_w)
        return dfail(d, VR_EINVAL,
                     "the context's row share changed (vr_set_row_share): create a new vr_dist");
    DTRY(hip_check(d, hipSetDevice(d->device), "hipSetDevice"));
    d->cam = cam;
    d->params = p;
    HipExec x{d};
    const int rc = d->sched.issue(x, static_cast<hipStream_t>(stream), frame_dev);
    d->cam = nullptr;
    d->params = nullptr;
    if (d->hprof) ++d->hp.frames;
    return rc;
}

int vr_dist_host_profile_enable(vr_dist *d, int enable)
{
    if (!d) return dfail(nullptr, VR_EINVAL, "dist is NULL");
    d->hprof = enable != 0;
    return VR_OK;
}

int vr_dist_host_profile_read(vr_dist *d, vr_dist_host_profile *out)
{
    if (!d || !out) return dfail(d, VR_EINVAL, "NULL argument");
    *out = d->hp;
    d->hp = vr_dist_host_profile{};
    return VR_OK;
}

int vr_dist_synchronize(vr_dist *d)
{
    if (!d) return dfail(nullptr, VR_EINVAL, "dist is NULL");
    DTRY(hip_check(d, hipSetDevice(d->device), "hipSetDevice"));
    for (auto &s : d->sched.slots)
        DTRY(hip_check(d, hipStreamSynchronize(s.stream), "hipStreamSynchronize"));
    // rank 0's gathers and assemblies run on the callers' streams: the last one's event
    if (hipEvent_t e = d->sched.last_gathered()) {
        const hipError_t r = hipEventSynchronize(e);
        if (r != hipSuccess)
            return dfail(d, r == hipErrorOutOfMemory ? VR_ENOMEM : VR_EIO,
                         std::string("hipEventSynchronize (rank ") + std::to_string(d->rank) +
                             ", frame " + std::to_string(d->sched.frame) + " of " +
                             std::to_string(d->sched.slots.size()) + " slots): " +
                             hipGetErrorString(r));
    }
    return VR_OK;
}

int vr_dist_timing_enable(vr_dist *d, int enable)
{
    if (!d) return dfail(nullptr, VR_EINVAL, "dist is NULL");
    d->timing = enable != 0;
    return VR_OK;
}

int vr_dist_timing_read(vr_dist *d, double *render_ms, double *gather_ms, uint64_t *frames)
{
    if (!d) return dfail(nullptr, VR_EINVAL, "dist is NULL");
    double acc[3];
    const int rc = timing_read3(d, acc, frames);
    if (render_ms) *render_ms = acc[0];
    if (gather_ms) *gather_ms = acc[1];
    return rc;
}

const char *vr_dist_last_error(const vr_dist *d) { return d ? d->err.c_str() : g_dist_err.c_str(); }

void vr_dist_destroy(vr_dist *d)
{
    if (!d) return;
    release(d);
    delete d;
}

}  // extern "C"

// ---- multi-device contexts (vr_create_mask; vr_group.h) ---------------------------------------
// One process drives every device of the mask.  Member m renders its 8-row blocks of the frame
// with the slot pipeline above (rank m of N, communicator from ncclCommInitAll), member 0's
// pipeline gathers and assembles into the caller's frame.  The members' enqueues run on
// FrameWorkers threads (member 0 on the caller's), each issuing on its own communicator in
// frame order: NCCL's one-thread-per-device pattern, no ncclGroupStart needed.
namespace vr {

struct GroupJob {
    vr_camera cam;
    vr_params p;
    void *out = nullptr;            // member 0: the caller's frame
    hipStream_t stream = nullptr;   // member 0: the caller's stream
};

struct Group {
    std::vector<vr_ctx *> members;
    std::vector<int> devices;
    std::vector<ncclComm_t> comms;
    std::vector<vr_dist *> dists;      // per member; rebuilt when the frame shape changes
    std::vector<hipStream_t> own;      // members 1..: the stream standing in for the caller's
    uint32_t width = 0, height = 0;
    int frames = 0, out_format = -1;
    uint32_t share_w0 = 1, share_w = 1;  // the row share the pipelines were built for
    bool timing = false;                 // per-member render / gather / assembly spans
    bool hprof = false;                  // per-member host profile (vr_debug_host_profile_*)
    std::vector<vr_dist_host_profile> hp;  // per member: host sums of pipelines freed since
    // per member: spans read from the pipelines so far (render, gather, assemble ms; frames)
    struct Spans {
        double ms[3] = {0.0, 0.0, 0.0};
        uint64_t frames = 0;
    };
    std::vector<Spans> spans;
    std::unique_ptr<sched::FrameWorkers<GroupJob>> workers;
    // VR_EXCHANGE_COPY: the gather as device copies (one exchange per pipeline build, whose
    // frame counters start at 0 with the pipelines'); comms stay null
    int exchange = VR_EXCHANGE_RCCL;
    std::unique_ptr<CopyExchange> xch;
    // vr_debug_fail_member: member fail_member's issue of pipeline frame fail_frame fails.
    // Written by the API thread while the frame workers read them (member_issue): atomics, the
    // frame stored before the member (release) and read after it (acquire).
    std::atomic<int> fail_member{-1};
    std::atomic<uint64_t> fail_frame{0};
};

namespace {

int member_issue(Group *g, int m, const GroupJob &j, std::string *msg)
{
    vr_dist *d = g->dists[m];
    int rc;
    if (m == g->fail_member.load(std::memory_order_acquire) &&
        d->sched.frame == g->fail_frame.load(std::memory_order_relaxed))
        rc = dfail(d, VR_EIO, "injected failure (vr_debug_fail_member) of frame " +
                                  std::to_string(d->sched.frame));
    else
        rc = vr_dist_render(d, &j.cam, &j.p, m == 0 ? j.out : nullptr,
                            m == 0 ? j.stream : g->own[m]);
    if (rc) {
        if (msg) *msg = d->err;
        // the copy exchange's peers wait on this member's frames on their host threads
        if (g->xch) g->xch->abort();
    }
    return rc;
}

void fold_spans(Group *g)
{
    g->spans.resize(g->members.size());
    for (size_t m = 0; m < g->dists.size(); ++m) {
        double ms[3];
        uint64_t n = 0;
        if (g->dists[m] && timing_read3(g->dists[m], ms, &n) == VR_OK) {
            for (int i = 0; i < 3; ++i) g->spans[m].ms[i] += ms[i];
            g->spans[m].frames += n;
        }
    }
}

void fold_host_profile(Group *g)
{
    g->hp.resize(g->members.size());
    for (size_t m = 0; m < g->dists.size(); ++m) {
        vr_dist_host_profile &a = g->hp[m];
        const vr_dist_host_profile &b = g->dists[m]->hp;
        a.frames += b.frames;
        a.render_us += b.render_us;
        a.gather_us += b.gather_us;
        a.assemble_us += b.assemble_us;
        a.record_us += b.record_us;
        a.wait_us += b.wait_us;
        a.total_us += b.total_us;
        g->dists[m]->hp = vr_dist_host_profile{};
    }
}

void free_pipelines(Group *g)
{
    g->workers.reset();  // drains the queues and joins the threads
    fold_spans(g);
    fold_host_profile(g);
    for (vr_dist *d : g->dists) {
        if (!d) continue;
        release(d);
        delete d;
    }
    g->dists.clear();
    g->frames = 0;
    g->out_format = -1;
}

// The slot pipelines for this frame shape (size, frames in flight, pixel format).
int ensure_pipelines(Group *g, int frames, int out_format, std::string *err)
{
    uint32_t w = 0, h = 0, s0 = 1, s1 = 1;
    vr_get_size(g->members[0], &w, &h);
    vr_get_row_share(g->members[0], &s0, &s1);
    if (!g->dists.empty() && g->frames == frames && g->out_format == out_format && g->width == w &&
        g->height == h && g->share_w0 == s0 && g->share_w == s1)
        return VR_OK;
    std::string m;
    if (g->workers && g->workers->drain(&m) != VR_OK) {
        *err = m;
        return VR_EIO;
    }
    if (int rc = group_synchronize(g, err)) return rc;
    free_pipelines(g);
    const int n = (int)g->members.size();
    if (g->exchange == VR_EXCHANGE_COPY) {
        g->xch.reset(new CopyExchange());
        g->xch->sent.assign(n, 0);
    }
    for (int k = 0; k < n; ++k) {
        vr_dist *d = dist_create(g->members[k], nullptr, g->comms[k], n, k, kGroupRowBlock, frames,
                                 out_format, g->xch.get());
        if (!d) {
            *err = g_dist_err;
            free_pipelines(g);
            return VR_EIO;
        }
        d->timing = g->timing;
        d->hprof = g->hprof;
        g->dists.push_back(d);
    }
    if (g->xch) g->xch->peers = g->dists;
    g->width = w;
    g->height = h;
    g->share_w0 = s0;
    g->share_w = s1;
    g->frames = frames;
    g->out_format = out_format;
    g->workers.reset(new sched::FrameWorkers<GroupJob>(
        n, [g](int m, const GroupJob &j, std::string *msg) { return member_issue(g, m, j, msg); },
        [g](int m) { hipSetDevice(g->devices[m]); }));
    return VR_OK;
}

}  // namespace

Group *group_create(const std::vector<vr_ctx *> &members, int exchange, std::string *err)
{
    if (members.empty()) {
        *err = "no devices";
        return nullptr;
    }
    if (exchange != VR_EXCHANGE_RCCL && exchange != VR_EXCHANGE_COPY) {
        *err = "unknown exchange";
        return nullptr;
    }
    if (exchange == VR_EXCHANGE_RCCL && !rccl().ok) {
        *err = rccl().err;
        return nullptr;
    }
    std::unique_ptr<Group> g(new (std::nothrow) Group());
    if (!g) {
        *err = "out of host memory";
        return nullptr;
    }
    g->members = members;
    for (vr_ctx *c : members) {
        int dev = -1;
        vr_get_device(c, &dev);
        g->devices.push_back(dev);
    }
    g->comms.assign(members.size(), nullptr);
    g->exchange = exchange;
    if (exchange == VR_EXCHANGE_RCCL) {
        for (size_t a = 0; a < g->devices.size(); ++a)
            for (size_t b = a + 1; b < g->devices.size(); ++b)
                if (g->devices[a] == g->devices[b]) {
                    *err = "device " + std::to_string(g->devices[a]) +
                           " listed twice: RCCL holds one rank per device (use VR_EXCHANGE_COPY)";
                    return nullptr;
                }
        const ncclResult_t r =
            rccl().comm_init_all(g->comms.data(), (int)members.size(), g->devices.data());
        if (r != ncclSuccess) {
            *err = std::string("ncclCommInitAll: ") + rccl().error_string(r);
            return nullptr;
        }
    }
    g->own.assign(members.size(), nullptr);
    for (size_t m = 1; m < members.size(); ++m) {
        hipSetDevice(g->devices[m]);
        if (hipStreamCreateWithFlags(&g->own[m], hipStreamNonBlocking) != hipSuccess) {
            *err = "hipStreamCreate";
            Group *raw = g.release();
            group_destroy(raw);
            return nullptr;
        }
    }
    hipSetDevice(g->devices[0]);
    return g.release();
}

// A member failed: its peers' gathers of the failed frame (and of every later frame the workers
// had queued) can never be matched.  Abort every communicator so those collectives end instead
// of holding the streams forever (FrameWorkers::settle calls this once, after the enqueues
// drained, before any stream is synchronised).  The context is unusable afterwards.
void abort_comms(Group *g)
{
    if (g->xch) g->xch->abort();
    for (size_t m = 0; m < g->comms.size(); ++m)
        if (g->comms[m]) {
            hipSetDevice(g->devices[m]);
            rccl().comm_abort(g->comms[m]);
            g->comms[m] = nullptr;
        }
    if (!g->devices.empty()) hipSetDevice(g->devices[0]);
}

int group_drain(Group *g, std::string *err)
{
    if (!g->workers) return VR_OK;
    return g->workers->settle([g] { abort_comms(g); }, err) == 0 ? VR_OK : VR_EIO;
}

int group_synchronize(Group *g, std::string *err)
{
    // a member's failure aborts the communicators here, before the waits below
    const int failed = group_drain(g, err);
    std::string sync_err;
    for (vr_dist *d : g->dists)
        if (vr_dist_synchronize(d) != VR_OK && sync_err.empty()) sync_err = d->err;
    for (size_t m = 1; m < g->own.size(); ++m)
        if (g->own[m]) {
            hipSetDevice(g->devices[m]);
            if (hipStreamSynchronize(g->own[m]) != hipSuccess && sync_err.empty())
                sync_err = "hipStreamSynchronize";
        }
    hipSetDevice(g->devices[0]);
    if (failed) return failed;
    if (!sync_err.empty()) {
        *err = sync_err;
        return VR_EIO;
    }
    return VR_OK;
}

void group_destroy(Group *g)
{
    if (!g) return;
    std::string ignored;
    group_synchronize(g, &ignored);
    free_pipelines(g);
    for (size_t m = 0; m < g->comms.size(); ++m)
        if (g->comms[m]) {
            hipSetDevice(g->devices[m]);
            rccl().comm_destroy(g->comms[m]);
        }
    for (size_t m = 1; m < g->own.size(); ++m)
        if (g->own[m]) {
            hipSetDevice(g->devices[m]);
            hipStreamDestroy(g->own[m]);
        }
    if (!g->devices.empty()) hipSetDevice(g->devices[0]);
    delete g;
}

int group_exchange(const Group *g) { return g->exchange; }

int group_fail_member(Group *g, int member, uint64_t frame, std::string *err)
{
    if (member >= (int)g->members.size()) {
        *err = "no such member";
        return VR_EINVAL;
    }
    // frames count from the next pipeline build; the current pipelines' counter otherwise
    g->fail_frame.store(frame, std::memory_order_relaxed);
    g->fail_member.store(member, std::memory_order_release);
    return VR_OK;
}

void group_host_profile_enable(Group *g, bool on)
{
    std::string ignored;
    group_drain(g, &ignored);  // the workers write the sums while they enqueue
    g->hprof = on;
    for (vr_dist *d : g->dists) d->hprof = on;
}

int group_host_profile_member(Group *g, int m, vr_dist_host_profile *out, std::string *err)
{
    if (m < 0 || m >= (int)g->members.size()) {
        *err = "no such member";
        return VR_EINVAL;
    }
    if (int rc = group_drain(g, err)) return rc;
    fold_host_profile(g);
    *out = g->hp[(size_t)m];
    g->hp[(size_t)m] = vr_dist_host_profile{};
    return VR_OK;
}

void group_timing_enable(Group *g, bool on)
{
    g->timing = on;
    for (vr_dist *d : g->dists) d->timing = on;
}

int group_timing_member(Group *g, int m, double ms[3], uint64_t *frames, std::string *err)
{
    if (m < 0 || m >= (int)g->members.size()) {
        *err = "no such member";
        return VR_EINVAL;
    }
    if (int rc = group_synchronize(g, err)) return rc;
    fold_spans(g);
    for (int i = 0; i < 3; ++i) ms[i] = g->spans[m].ms[i];
    *frames = g->spans[m].frames;
    return VR_OK;
}

int group_timing_reset(Group *g, std::string *err)
{
    if (int rc = group_synchronize(g, err)) return rc;
    fold_spans(g);
    g->spans.assign(g->members.size(), Group::Spans());
    return VR_OK;
}

int group_render(Group *g, const vr_camera *cam, const vr_params *p, void *out_dev,
                 int out_format, hipStream_t stream, std::string *err)
{
    const int frames = p->frames_in_flight < 1 ? 1 : (p->frames_in_flight > 8 ? 8 : p->frames_in_flight);
    if (int rc = ensure_pipelines(g, frames, out_format, err)) return rc;
    GroupJob j;
    j.cam = *cam;
    j.p = *p;
    j.out = out_dev;
    j.stream = stream;
    int rc = g->workers->issue(j, err);
    if (rc != 0 && !g->workers->aborted()) {
        // member 0 or a worker failed: end the unmatched collectives now, so the
        // caller's stream and vr_destroy cannot wait on them forever
        std::string m;
        g->workers->settle([g] { abort_comms(g); }, &m);
    }
    return rc == 0 ? VR_OK : (rc < 0 ? rc : VR_EIO);
}

}  // namespace vr
