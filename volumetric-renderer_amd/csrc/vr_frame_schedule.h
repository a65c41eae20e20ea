// vr_frame_schedule.h — the per-frame schedule of a multi-GPU frame (include/vr/vr_dist.h),
// written once against an executor so that the same code drives HIP streams/events with
// ncclGather (vr_dist.cpp) and host threads with a stand-in collective (vr_sched_host.cpp,
// exercised by the world-size-2 gloo test tests/test_sched_host.py on CPU).
//
//   slot stream k : render shard_k ─► [rendered_k]                 ┌► assemble (rank 0) ─► [done_k]
//   comm stream   :        wait rendered_k ─► gather ─► [gathered_k]
//   slot stream k :                                 wait gathered_k┘
//   caller stream : ... [called] ─────────────────────────────────────── wait done_k ...
//
// Frame i takes slot i mod F, so its render only queues behind frame i-F's assembly (which
// frees shard_k and gbuf_k) and F frames are in flight.  The gathers run on one
// communication stream in frame order, which every rank issues identically.
//
// Executor X provides the types Stream and Event and, each returning 0 or a negative VR_E*
// code (all asynchronous: they enqueue on the stream given):
//   record(Event, Stream)             event completes when the stream reaches this point
//   wait(Stream, Event)               the stream waits for the event's latest record
//   render(int slot, uint64_t frame, Stream)
//   gather(int slot, uint64_t frame, Stream)          the collective to rank 0
//   assemble(int slot, uint64_t frame, void *frame_dev, Stream)   rank 0 only
#pragma once

#include <stdint.h>

#include <vector>

namespace vr {
namespace sched {

template <class X>
struct FrameSchedule {
    using Stream = typename X::Stream;
    using Event = typename X::Event;
    struct Slot {
        Stream stream{};
        Event rendered{}, gathered{}, done{};
    };
    int rank = 0;
    Stream comm{};
    Event called{};
    std::vector<Slot> slots;
    uint64_t frame = 0;

    // Enqueue one frame; rank 0's frame_dev is complete once `caller` passes this point.
    int issue(X &x, Stream caller, void *frame_dev)
    {
        const int k = (int)(frame % slots.size());
        Slot &s = slots[k];
        int rc;
#define VR_SCHED_TRY(e)              \
    do {                             \
        if ((rc = (e)) != 0) return rc; \
    } while (0)
        VR_SCHED_TRY(x.render(k, frame, s.stream));
        VR_SCHED_TRY(x.record(s.rendered, s.stream));
        VR_SCHED_TRY(x.wait(comm, s.rendered));
        VR_SCHED_TRY(x.gather(k, frame, comm));
        VR_SCHED_TRY(x.record(s.gathered, comm));
        VR_SCHED_TRY(x.wait(s.stream, s.gathered));
        if (rank == 0) {
            // the caller's earlier work on its stream (e.g. reading frame_dev) precedes the write
            VR_SCHED_TRY(x.record(called, caller));
            VR_SCHED_TRY(x.wait(s.stream, called));
            VR_SCHED_TRY(x.assemble(k, frame, frame_dev, s.stream));
        }
        VR_SCHED_TRY(x.record(s.done, s.stream));
        VR_SCHED_TRY(x.wait(caller, s.done));
#undef VR_SCHED_TRY
        ++frame;
        return 0;
    }
};

}  // namespace sched
}  // namespace vr
