/*
 * vr_debug.h — launch-policy overrides for tests and A/B experiments.
 *
 * Not part of the drop-in boundary (the reference has no equivalent): the library picks the
 * march kernel variant, the 8-bit brick layout and the tile order from the volume, the view
 * and vr_params alone (DESIGN.md §5 "Which kernel a launch runs").  Every variant renders the
 * same bytes, so these knobs change speed, never results -- except VR_KNOB_GRAD_FIELD when
 * vr_params.exact_gradient is 0 (the field then holds binary16 differences, the stencil exact
 * ones); the GPU tests use them to render each variant and compare.  The library never reads the process environment, except in
 * experiment builds (`make EXTRA=-DVR_EXPERIMENTS`), where vr_create() seeds the knobs from
 * VR_PIPELINE, VR_PAIR, VR_PAIR_LANES, VR_NO_GRAD_FIELD / VR_GRAD_FIELD_ALWAYS,
 * VR_U8_LAYOUT and VR_TILE_ORDER_DEFAULT (the names the round-1/2 A/B scripts under tools/
 * set).
 */
#ifndef VR_VR_DEBUG_H
#define VR_VR_DEBUG_H

#include "vr.h"
#include "vr_dist.h"

#ifdef __cplusplus
extern "C" {
#endif

enum vr_knob {
    VR_KNOB_PIPELINE = 1,   /* -1 auto, 0 one sample in flight per ray, 1 pipelined (two)   */
    VR_KNOB_PAIR = 2,       /* -1 auto, 0 never, 1 lane groups (march_pair_kernel) if legal */
    VR_KNOB_PAIR_LANES = 3, /* 0 auto, 2 or 4 lanes per ray                                 */
    VR_KNOB_GRAD_FIELD = 4, /* -1 auto (dense-row views), 0 stencil gradient, 1 the f32
                               difference field on every view                               */
    /* 5: retired (the LDS-staged march, measured 1.6-2.7x slower: tools/experiments/r04_pruned/) */
    VR_KNOB_U8_LAYOUT = 6,  /* -1 auto, 0 plain 7x8x8 bricks, 1 yz-quads (next upload)      */
    VR_KNOB_TILE_ORDER = 7, /* tile order used when vr_params.tile_order == 0: 0 auto (4),
                               1..4 as vr_params.tile_order                                */
    VR_KNOB_NARROW = 8,     /* 1 (default): 32/64-bit uploads whose voxels are all integers
                               that fit 8/16 bits are stored in that type (same frames); 0:
                               keep f32 storage (next upload)                              */
    VR_KNOB_ALT_GEOMETRY = 9 /* f32 volumes: -1 auto (oblique views and rays along x read a
                               7x15x8-cell-brick copy; sparse views along the bricks' rows the
                               stencil copy when shaded, a plain one-voxel-per-element 15^3
                               one when not), 0 never, 1 the
                               oblique copy, 3 the plain copy, 4 the stencil copy (29^3-cell
                               plain bricks with a 1-below / 2-above apron), whenever the
                               launch allows it (2, the retired z-pair sparse copy: EINVAL) */
};

/* Per-device timing of a context (ABI 7), so that a multi-GPU frame that runs slow names its
 * straggler.  With vr_timing_enable on, summed since vr_timing_reset, for member m of a
 * vr_create_mask context (member 0 = the lowest device, which also assembles; a one-device
 * context has member 0 only, kernel time alone):
 *   kernel_ms    its ray-march kernels (HIP events around each launch)
 *   render_ms    its render step on its slot streams (the march plus the tile-order kernel)
 *   gather_ms    its ncclGather (member 0: on the caller's stream, receiving every shard)
 *   assemble_ms  member 0: the de-interleave of the gathered shards into the frame
 *   frames       frames timed on that member
 * (vr_timing_read on a multi-device context sums kernel_ms over the devices.) */
typedef struct vr_member_timing {
    int32_t device;
    uint64_t frames;
    double kernel_ms, render_ms, gather_ms, assemble_ms;
} vr_member_timing;
int vr_debug_timing_member(vr_ctx *ctx, int member, vr_member_timing *out);

/* One-GPU rehearsal of the multi-device path (round 5).  A multi-device context over an explicit
 * member list: devices[m] is member m's device (member 0 assembles the frame), and a device may
 * be listed more than once -- two members on device 0 exercise on one GPU what vr_create_mask
 * runs on several: the frame workers, the volume replication, the per-member slot pipelines,
 * the row shares and the assembly.  `exchange` is how the shards reach member 0:
 *   VR_EXCHANGE_RCCL  ncclGather over ncclCommInitAll communicators (vr_create_mask's; the
 *                     devices must be distinct -- RCCL holds one rank per device)
 *   VR_EXCHANGE_COPY  stream-ordered device-to-device copies of every member's shard into
 *                     member 0's gather buffer, enqueued by member 0 (peer copies across
 *                     devices), with host-side frame handshakes between the member threads
 * Frames are byte-identical to a one-device context's in both.  NULL on failure
 * (vr_last_error(NULL)). */
enum vr_exchange { VR_EXCHANGE_RCCL = 0, VR_EXCHANGE_COPY = 1 };
vr_ctx *vr_debug_create_members(const int *devices, int n, uint32_t width, uint32_t height,
                                int exchange);
/* Failure injection on a multi-device context: member `member`'s enqueue of its pipelines'
 * frame number `frame` (counted from 0 since the pipelines were built for the current frame
 * shape; the first frame after creation is 0) fails with VR_EIO, as a device error would.  The
 * context then aborts the frame exchange and every later frame fails; vr_destroy still returns
 * (no stream waits forever).  member < 0 clears it.  VR_EINVAL on a one-device context. */
int vr_debug_fail_member(vr_ctx *ctx, int member, uint64_t frame);

/* Host cost of a multi-device context's frames (round 6; tools/host_cost.cpp): with host
 * profiling on, every member's frame enqueue -- member 0 on the caller's thread, the others on
 * their frame-worker threads -- adds the host microseconds of its steps as vr_dist_render does
 * (vr_dist_host_profile, vr_dist.h).  vr_debug_host_profile_member waits until every member has
 * enqueued the frames issued so far (not for the device), returns member `member`'s sums and
 * clears them.  VR_EINVAL on a one-device context. */
int vr_debug_host_profile_enable(vr_ctx *ctx, int enable);
int vr_debug_host_profile_member(vr_ctx *ctx, int member, vr_dist_host_profile *out);

/* Set / read one knob of `ctx` (a multi-device context sets it on every device).
 * VR_EINVAL for an unknown knob or an out-of-range value. */
int vr_debug_set_knob(vr_ctx *ctx, int knob, int value);
int vr_debug_get_knob(const vr_ctx *ctx, int knob, int *value);

#ifdef __cplusplus
}
#endif

#endif /* VR_VR_DEBUG_H */
