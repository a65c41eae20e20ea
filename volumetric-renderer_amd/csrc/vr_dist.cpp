// vr_dist.cpp — multi-GPU frames over RCCL (include/vr/vr_dist.h).
//
// Sort-first image tiling: each rank ray-marches its row blocks through the
// public vr.h entry points, one ncclGather per frame collects the shards on rank 0 over xGMI,
// and rank 0 de-interleaves them.  The whole frame is stream-ordered:
//
//   slot stream k : render shard_k ─► [rendered_k]                 ┌► assemble (rank 0) ─► [done_k]
//   comm stream   :        wait rendered_k ─► ncclGather ─► [gathered_k]
//   slot stream k :                                 wait gathered_k┘
//   caller stream : ... [called] ─────────────────────────────────────── wait done_k ...
//
// Frame i takes slot i mod F, so its render only queues behind frame i-F's assembly (which
// frees shard_k and gbuf_k) and F frames are in flight.  The gathers are serialised on one
// communication stream in frame order, which every rank issues identically.
//
// RCCL is resolved with dlopen at creation (the librccl.so.1 already loaded, e.g. PyTorch's,
// else the system one), so single-GPU users of the library never load it.
#include "vr/vr_dist.h"

#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <cstring>
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
    ncclResult_t (*gather)(const void *, void *, size_t, ncclDataType_t, int, ncclComm_t,
                           hipStream_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
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
        !bind(h, "ncclCommDestroy", r.comm_destroy) ||
        !bind(h, "ncclGetErrorString", r.error_string)) {
        r.err = "librccl.so.1 lacks ncclGather/ncclCommInitRank/...";
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

struct Slot {
    hipStream_t stream = nullptr;
    void *shard = nullptr;  // shard_rows x W RGBA8
    void *gbuf = nullptr;   // rank 0: nranks shards, rank-major
    hipEvent_t rendered = nullptr, gathered = nullptr, done = nullptr;
};

}  // namespace

struct vr_dist {
    vr_ctx *ctx = nullptr;
    int device = 0;
    int nranks = 1, rank = 0;
    uint32_t row_block = 8, width = 0, height = 0, shard_rows = 0;
    ncclComm_t comm = nullptr;
    hipStream_t comm_stream = nullptr;
    hipEvent_t called = nullptr;
    std::vector<Slot> slots;
    uint64_t frame = 0;
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

void release(vr_dist *d)
{
    hipSetDevice(d->device);
    for (auto &s : d->slots) {
        if (s.stream) hipStreamSynchronize(s.stream);
    }
    if (d->comm_stream) hipStreamSynchronize(d->comm_stream);
    if (d->comm) rccl().comm_destroy(d->comm);
    for (auto &s : d->slots) {
        if (s.shard) hipFree(s.shard);
        if (s.gbuf) hipFree(s.gbuf);
        if (s.rendered) hipEventDestroy(s.rendered);
        if (s.gathered) hipEventDestroy(s.gathered);
        if (s.done) hipEventDestroy(s.done);
        if (s.stream) hipStreamDestroy(s.stream);
    }
    if (d->called) hipEventDestroy(d->called);
    if (d->comm_stream) hipStreamDestroy(d->comm_stream);
    d->slots.clear();
}

int setup(vr_dist *d, const void *id, int frames)
{
    DTRY(hip_check(d, hipSetDevice(d->device), "hipSetDevice"));
    ncclUniqueId uid;
    static_assert(sizeof(uid) == VR_DIST_ID_BYTES, "ncclUniqueId size");
    std::memcpy(&uid, id, sizeof(uid));
    DTRY(nccl_check(d, rccl().comm_init_rank(&d->comm, d->nranks, uid, d->rank), "ncclCommInitRank"));
    DTRY(hip_check(d, hipStreamCreateWithFlags(&d->comm_stream, hipStreamNonBlocking),
                   "hipStreamCreate(comm)"));
    DTRY(hip_check(d, hipEventCreateWithFlags(&d->called, hipEventDisableTiming), "hipEventCreate"));
    const size_t shard_bytes = (size_t)d->shard_rows * d->width * 4;
    d->slots.resize(frames);
    for (auto &s : d->slots) {
        DTRY(hip_check(d, hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking),
                       "hipStreamCreate(slot)"));
        DTRY(hip_check(d, hipMalloc(&s.shard, shard_bytes), "hipMalloc(shard)"));
        if (d->rank == 0)
            DTRY(hip_check(d, hipMalloc(&s.gbuf, shard_bytes * d->nranks), "hipMalloc(gather)"));
        for (hipEvent_t *e : {&s.rendered, &s.gathered, &s.done})
            DTRY(hip_check(d, hipEventCreateWithFlags(e, hipEventDisableTiming), "hipEventCreate"));
    }
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

vr_dist *vr_dist_create(vr_ctx *ctx, const void *id, int nranks, int rank, uint32_t row_block,
                        int frames_in_flight)
{
    if (!ctx || !id) {
        dfail(nullptr, VR_EINVAL, "ctx or id is NULL");
        return nullptr;
    }
    if (nranks < 1 || rank < 0 || rank >= nranks || row_block == 0 || frames_in_flight < 1 ||
        frames_in_flight > 8) {
        dfail(nullptr, VR_EINVAL, "bad nranks/rank/row_block/frames_in_flight");
        return nullptr;
    }
    if (!rccl().ok) {
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
    if (vr_get_device(ctx, &d->device) != VR_OK || vr_get_size(ctx, &d->width, &d->height) != VR_OK) {
        dfail(nullptr, VR_EINVAL, "bad ctx");
        delete d;
        return nullptr;
    }
    d->shard_rows = vr_shard_rows(d->height, row_block, (uint32_t)nranks);
    if (setup(d, id, frames_in_flight) != VR_OK) {
        g_dist_err = d->err;
        release(d);
        delete d;
        return nullptr;
    }
    return d;
}

int vr_dist_render(vr_dist *d, const vr_camera *cam, const vr_params *p, void *frame_dev,
                   void *stream)
{
    if (!d) return dfail(nullptr, VR_EINVAL, "dist is NULL");
    if (!cam || !p) return dfail(d, VR_EINVAL, "camera or params is NULL");
    if (d->rank == 0 && !frame_dev) return dfail(d, VR_EINVAL, "rank 0 needs frame_dev");
    uint32_t w = 0, h = 0;
    if (vr_get_size(d->ctx, &w, &h) != VR_OK || w != d->width || h != d->height)
        return dfail(d, VR_EINVAL, "the context was resized: create a new vr_dist");
    DTRY(hip_check(d, hipSetDevice(d->device), "hipSetDevice"));
    hipStream_t caller = static_cast<hipStream_t>(stream);
    Slot &s = d->slots[d->frame % d->slots.size()];
    vr_params q = *p;
    q.frames_in_flight = (int32_t)d->slots.size();
    if (vr_render_device(d->ctx, cam, &q, s.shard, VR_OUT_RGBA8, d->row_block, (uint32_t)d->rank,
                         (uint32_t)d->nranks, s.stream) != VR_OK)
        return dfail(d, VR_EIO, std::string("render: ") + vr_last_error(d->ctx));
    DTRY(hip_check(d, hipEventRecord(s.rendered, s.stream), "hipEventRecord"));
    DTRY(hip_check(d, hipStreamWaitEvent(d->comm_stream, s.rendered, 0), "hipStreamWaitEvent"));
    DTRY(nccl_check(d, rccl().gather(s.shard, d->rank == 0 ? s.gbuf : nullptr,
                                     (size_t)d->shard_rows * d->width, ncclUint32, 0, d->comm,
                                     d->comm_stream),
                    "ncclGather"));
    DTRY(hip_check(d, hipEventRecord(s.gathered, d->comm_stream), "hipEventRecord"));
    DTRY(hip_check(d, hipStreamWaitEvent(s.stream, s.gathered, 0), "hipStreamWaitEvent"));
    if (d->rank == 0) {
        // the caller's earlier work on `stream` (e.g. reading frame_dev) precedes the write
        DTRY(hip_check(d, hipEventRecord(d->called, caller), "hipEventRecord"));
        DTRY(hip_check(d, hipStreamWaitEvent(s.stream, d->called, 0), "hipStreamWaitEvent"));
        if (vr_assemble_rows(d->ctx, s.gbuf, frame_dev, VR_OUT_RGBA8, d->row_block,
                             (uint32_t)d->nranks, s.stream) != VR_OK)
            return dfail(d, VR_EIO, std::string("assemble: ") + vr_last_error(d->ctx));
    }
    DTRY(hip_check(d, hipEventRecord(s.done, s.stream), "hipEventRecord"));
    DTRY(hip_check(d, hipStreamWaitEvent(caller, s.done, 0), "hipStreamWaitEvent"));
    d->frame++;
    return VR_OK;
}

int vr_dist_synchronize(vr_dist *d)
{
    if (!d) return dfail(nullptr, VR_EINVAL, "dist is NULL");
    DTRY(hip_check(d, hipSetDevice(d->device), "hipSetDevice"));
    for (auto &s : d->slots) DTRY(hip_check(d, hipStreamSynchronize(s.stream), "hipStreamSynchronize"));
    return hip_check(d, hipStreamSynchronize(d->comm_stream), "hipStreamSynchronize");
}

const char *vr_dist_last_error(const vr_dist *d) { return d ? d->err.c_str() : g_dist_err.c_str(); }

void vr_dist_destroy(vr_dist *d)
{
    if (!d) return;
    release(d);
    delete d;
}

}  // extern "C"
