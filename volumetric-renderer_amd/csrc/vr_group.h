// vr_group.h — internal: the frame path of a multi-device context (vr_create_mask, vr.h).
//
// vr_api.hip owns the member contexts (one vr_ctx per device, the volume/TF/slicing replicated
// on each); this part (vr_dist.cpp) owns what a frame needs across them: one RCCL communicator
// per member from ncclCommInitAll, the per-member slot pipelines of vr_dist (render this
// member's 8-row blocks -> ncclGather to member 0 -> assemble there, stream-ordered), and the
// frame workers (vr_frame_workers.h) that enqueue every member's part in parallel.
#pragma once

#include <hip/hip_runtime_api.h>

#include <string>
#include <vector>

#include "../../include/vr/vr.h"
#include "../../include/vr/vr_debug.h"
#include "../../include/vr/vr_dist.h"

namespace vr {

struct Group;

// Rows per block of the block-cyclic split (block b -> member b mod N), as SURVEY.md §8e.
constexpr uint32_t kGroupRowBlock = 8;

// True for a vr_create_mask context (vr_api.hip).
bool is_multi_device(const vr_ctx *c);

// Frame fences of a context (vr_api.hip): every render on a stream is followed by a record of the
// stream's fence event, which evictions of derived structures wait on.  A caller that itself
// records `ev` on `stream` after every render it issues there before its next render call (a
// vr_dist slot stream) registers it, and the context records nothing of its own on that stream;
// unregister after the stream's work is complete, before the event or the stream is destroyed.
int register_stream_fence(vr_ctx *c, hipStream_t stream, hipEvent_t ev);
void unregister_stream_fence(vr_ctx *c, hipStream_t stream);
// Fold the context's pending kernel-timing events into its totals; call after draining, before
// destroying, the streams they were recorded on (vr_dist slot streams).
void settle_timing(vr_ctx *c);

// The frame exchange over the members' devices (member 0 = the frame's device):
// VR_EXCHANGE_RCCL, one communicator per member from ncclCommInitAll (distinct devices), or
// VR_EXCHANGE_COPY, device copies onto member 0 (any devices, the same one repeated included).
// nullptr on failure (*err says why).
Group *group_create(const std::vector<vr_ctx *> &members, int exchange, std::string *err);
int group_exchange(const Group *g);
// vr_debug_fail_member: member's issue of pipeline frame `frame` fails (member < 0: never).
int group_fail_member(Group *g, int member, uint64_t frame, std::string *err);
// Waits for every frame issued so far (enqueue and device work), then frees the pipelines and
// communicators; the member contexts stay.
void group_destroy(Group *g);
// Waits until every member has enqueued every frame issued so far (not for the device).
int group_drain(Group *g, std::string *err);
// Waits for every frame issued so far on the devices as well.
int group_synchronize(Group *g, std::string *err);
// One frame across the members into out_dev (member 0's device, W*H pixels of out_format),
// complete once `stream` passes this point (the vr_dist_render contract).
int group_render(Group *g, const vr_camera *cam, const vr_params *p, void *out_dev,
                 int out_format, hipStream_t stream, std::string *err);
// Per-member spans (HIP events on the member's own streams; vr_debug_timing_member): render of
// its row blocks, its ncclGather, and (member 0) the assembly, summed since the last reset.
void group_timing_enable(Group *g, bool on);
// Per-member host profile (vr_dist_host_profile of each member's pipeline, summed across
// pipeline rebuilds): read waits until every member has enqueued the frames issued so far, then
// returns member m's sums and clears them.
void group_host_profile_enable(Group *g, bool on);
int group_host_profile_member(Group *g, int m, vr_dist_host_profile *out, std::string *err);
int group_timing_member(Group *g, int member, double ms[3], uint64_t *frames, std::string *err);
int group_timing_reset(Group *g, std::string *err);

}  // namespace vr
