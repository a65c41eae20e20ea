/*
 * vr_dist.h — multi-GPU frames over RCCL, one process (and one vr_ctx) per GPU.
 *
 * The reference renders on one device (OffscreenPass::record, offscreen_pass.cpp:163-230,
 * called once per frame by MainPass::render, main_pass.cpp:91).  This is the sort-first
 * form of that call for a node of GPUs: every rank ray-marches its row
 * blocks of the frame (vr_render_device with rank/nranks), ONE ncclGather per frame moves the
 * shards to rank 0 over xGMI, and rank 0 de-interleaves them into the caller's frame
 * (vr_assemble_rows).  The volume, TF and slicing are replicated: each rank's context gets
 * the same vr_set_* calls.
 *
 * Everything a frame does is stream-ordered on the device; the host never waits.  Frames
 * rotate over `frames_in_flight` internal slots, each with its own stream, shard and gather
 * buffer, so frame k+1 renders while frame k's gather is on the wire and consecutive frames
 * overlap on the device (the reference keeps MAX_FRAMES_IN_FLIGHT = 2,
 * vulkan_context.h:17).  The gathers run one at a time in frame order: on rank 0 on the
 * caller's stream, followed there by the assembly; on the other ranks on the slot streams,
 * each after the previous frame's (2 event records + 2 stream waits per frame on rank 0, 1 + 1
 * elsewhere; csrc/vr_frame_schedule.h).
 *
 * RCCL is loaded at vr_dist_create time (the librccl.so.1 already in the process, e.g.
 * PyTorch's, else the system one); single-GPU users of vr.h never load it.  Bootstrap: rank
 * 0 calls vr_dist_unique_id and sends the VR_DIST_ID_BYTES bytes to every rank by any
 * means (torch.distributed, MPI, a file); every rank then calls vr_dist_create together
 * (it blocks until all nranks have joined).
 *
 * Same conventions as vr.h: extern "C", 0 or a negative VR_E* code, messages via
 * vr_dist_last_error (or vr_last_error(NULL) when creation fails).  Not thread-safe.
 */
#ifndef VR_VR_DIST_H
#define VR_VR_DIST_H

#include "vr.h"

#ifdef __cplusplus
extern "C" {
#endif

#define VR_DIST_ID_BYTES 128 /* sizeof(ncclUniqueId) */

typedef struct vr_dist vr_dist;

/* Rank 0: a fresh communicator id (ncclGetUniqueId) into id_out[VR_DIST_ID_BYTES]. */
int vr_dist_unique_id(void *id_out);

/* Join the communicator (ncclCommInitRank on ctx's device) and allocate the slots:
 * frames_in_flight in [1, 8] (1 = serial frames), rows cut into blocks of row_block rows,
 * block b rendered by rank b % nranks.  The frame size is ctx's at creation; a later
 * vr_resize of ctx needs a new vr_dist.  Returns NULL on failure. */
vr_dist *vr_dist_create(vr_ctx *ctx, const void *id, int nranks, int rank, uint32_t row_block,
                        int frames_in_flight);

/* One frame: render this rank's rows, gather to rank 0, assemble there into frame_dev
 * (rank 0: W*H*4 bytes of device memory, RGBA8; ignored elsewhere).  Asynchronous: on rank 0
 * the frame is complete once `stream` (the caller's hipStream_t, NULL = default) passes the
 * point of this call, and work the caller enqueued on `stream` before the call (e.g. reading
 * frame_dev's previous contents) happens before frame_dev is written; rank 0's `stream` must
 * stay alive until the frame is complete (vr_dist_synchronize waits for it through an event
 * recorded there).  On the other ranks the call only enqueues: `stream` is not used, and
 * vr_dist_synchronize waits for the frames.  Every rank must call it for every frame, in the
 * same order, with the same camera and params. */
int vr_dist_render(vr_dist *d, const vr_camera *cam, const vr_params *p, void *frame_dev,
                   void *stream);

/* Wait for every frame issued so far (host wait on all slots and the gathers). */
int vr_dist_synchronize(vr_dist *d);

const char *vr_dist_last_error(const vr_dist *d);

/* Per-rank diagnostics (a straggler shows as a long render on its own rank and long gathers on
 * the others): with timing enabled, every later frame brackets its render and its ncclGather
 * with timing events on their streams.  vr_dist_timing_read waits for the outstanding frames,
 * returns the summed milliseconds and the number of frames timed, and clears the record. */
int vr_dist_timing_enable(vr_dist *d, int enable);
int vr_dist_timing_read(vr_dist *d, double *render_ms, double *gather_ms, uint64_t *frames);

/* Host cost of the frame path (diagnostics; tools/host_cost.cpp): with host profiling on,
 * vr_dist_render adds the host microseconds of each step it enqueues -- this rank's render
 * (vr_render_device), the gather (ncclGather or the copy exchange), the assembly, the event
 * records and the stream waits of the schedule -- and of the whole call.
 * vr_dist_host_profile_read returns the sums and the frames counted, and clears them. */
typedef struct vr_dist_host_profile {
    uint64_t frames;
    double render_us, gather_us, assemble_us, record_us, wait_us, total_us;
} vr_dist_host_profile;
int vr_dist_host_profile_enable(vr_dist *d, int enable);
int vr_dist_host_profile_read(vr_dist *d, vr_dist_host_profile *out);

/* Waits for outstanding frames, then frees the slots and the communicator. */
void vr_dist_destroy(vr_dist *d);

#ifdef __cplusplus
}
#endif

#endif /* VR_VR_DIST_H */
