// vr_frame_schedule.h — the per-frame schedule of a multi-GPU frame (include/vr/vr_dist.h),
// written once against an executor so that the same code drives HIP streams/events with
// ncclGather (vr_dist.cpp) and host threads with a stand-in collective (vr_sched_host.cpp,
// exercised by the world-size-2 gloo test tests/test_sched_host.py on CPU).
//
// Frame i takes slot i mod F (F = frames in flight); each slot has its own stream, so the
// renders of consecutive frames overlap on the device.  The gathers run one at a time, in frame
// order, which every rank issues identically.  Every cross-stream edge costs a record and a
// wait on the host (about 2.4 + 3.7 us on MI355X against a pending event, tools/host_cost.cpp),
// so each rank's schedule keeps the fewest edges its work needs (round 6):
//
//   rank 0 (gathers and assembles on the caller's stream, which orders them and makes the
//           caller's earlier reads of frame_dev precede the write, with no extra event):
//     slot stream k : [wait gathered_k: frame i-F freed the slot] render ─► [rendered_k]
//     caller stream : wait rendered_k ─► gather ─► assemble into frame_dev ─► [gathered_k]
//   rank r > 0 (nothing to assemble; the previous frame's gather on its own slot stream):
//     slot stream k : render ─► wait gathered_(k-1) ─► gather ─► [gathered_k]
//
// Rank 0: 2 records + 2 waits per frame (a caller stream other than the previous frame's also
// waits for that frame's gather); rank r > 0: 1 + 1.  (Rounds 1-5 used a separate
// communication stream and 4 + 4.)  On rank r > 0 the call only enqueues: its caller's stream
// is not ordered after the frame (vr_dist_synchronize waits for it).
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
        Event rendered{}, gathered{};
    };
    int rank = 0;
    std::vector<Slot> slots;
    uint64_t frame = 0;
    Stream last_caller{};  // rank 0: the stream the previous frame's gather ran on

    // The event recorded after the latest frame's gather (and assembly): every frame issued so
    // far is complete once it is.  Null before the first frame.
    Event last_gathered() const
    {
        return frame ? slots[(frame - 1) % slots.size()].gathered : Event{};
    }

    // Enqueue one frame; rank 0's frame_dev is complete once `caller` passes this point.
    int issue(X &x, Stream caller, void *frame_dev)
    {
        const uint64_t F = slots.size();
        const int k = (int)(frame % F);
        Slot &s = slots[k];
        const Slot &prev = slots[(frame + F - 1) % F];
        int rc;
#define VR_SCHED_TRY(e)              \
    do {                             \
        if ((rc = (e)) != 0) return rc; \
    } while (0)
        if (rank == 0) {
            // frame i - F's gather and assembly (caller stream) read this slot's buffers
            if (frame >= F) VR_SCHED_TRY(x.wait(s.stream, s.gathered));
            VR_SCHED_TRY(x.render(k, frame, s.stream));
            VR_SCHED_TRY(x.record(s.rendered, s.stream));
            // gathers in frame order: a caller stream other than the last one follows its gather
            if (frame > 0 && caller != last_caller) VR_SCHED_TRY(x.wait(caller, prev.gathered));
            VR_SCHED_TRY(x.wait(caller, s.rendered));
            VR_SCHED_TRY(x.gather(k, frame, caller));
            VR_SCHED_TRY(x.assemble(k, frame, frame_dev, caller));
            VR_SCHED_TRY(x.record(s.gathered, caller));
            last_caller = caller;
        } else {
            // the slot stream's own order: frame i - F's gather preceded this render
            VR_SCHED_TRY(x.render(k, frame, s.stream));
            if (frame > 0 && F > 1) VR_SCHED_TRY(x.wait(s.stream, prev.gathered));
            VR_SCHED_TRY(x.gather(k, frame, s.stream));
            VR_SCHED_TRY(x.record(s.gathered, s.stream));
        }
#undef VR_SCHED_TRY
        ++frame;
        return 0;
    }
};

}  // namespace sched
}  // namespace vr
