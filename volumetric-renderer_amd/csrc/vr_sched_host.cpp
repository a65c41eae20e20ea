// vr_sched_host.cpp — host executor of the multi-GPU frame schedule (vr_frame_schedule.h).
//
// vr_dist.cpp runs vr::sched::FrameSchedule on HIP streams and events with ncclGather as the
// collective.  This file runs the SAME schedule code on host threads: a stream is a worker
// thread draining an in-order queue, an event completes when its stream reaches the record
// (a wait targets the latest record at enqueue time, as hipStreamWaitEvent does), and render,
// gather, assemble and the caller's per-frame consume are callbacks (in the tests: numpy
// shards, torch.distributed.gather over gloo, numpy assembly, a frame check).  It lets the
// world-size-2 CPU test (tests/test_sched_host.py) drive the exact slot/stream/event order a
// multi-GPU frame uses, without a GPU.  Built by g++ into lib/libvr_sched_host.so.
//
// vr_group_host_* does the same for a multi-device context (vr_create_mask): N members in one
// process, each with its own FrameSchedule, issued by the same vr::sched::FrameWorkers
// (vr_frame_workers.h: member 0 on the calling thread, the others on worker threads) that
// vr_dist.cpp's group_render uses.
#include <stdint.h>

#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "vr_frame_schedule.h"
#include "vr_frame_workers.h"

namespace {

struct HostEvent {
    std::mutex m;
    std::condition_variable cv;
    uint64_t recorded = 0;   // records enqueued
    uint64_t completed = 0;  // records reached by their stream
};

struct HostStream {
    struct Op {
        std::function<int()> f;
        bool callback;  // skipped after an error (records and waits always run: no deadlock)
    };
    std::mutex m;
    std::condition_variable cv;
    std::deque<Op> q;
    bool stop = false, busy = false;
    int error = 0;  // first failing callback's code
    std::thread th;

    HostStream() { th = std::thread([this] { run(); }); }
    ~HostStream()
    {
        {
            std::lock_guard<std::mutex> g(m);
            stop = true;
        }
        cv.notify_all();
        th.join();
    }
    void push(std::function<int()> f, bool callback = false)
    {
        {
            std::lock_guard<std::mutex> g(m);
            q.push_back(Op{std::move(f), callback});
        }
        cv.notify_all();
    }
    // waits until every op enqueued so far has run
    int drain()
    {
        std::unique_lock<std::mutex> g(m);
        cv.wait(g, [this] { return q.empty() && !busy; });
        return error;
    }

  private:
    void run()
    {
        std::unique_lock<std::mutex> g(m);
        for (;;) {
            cv.wait(g, [this] { return stop || !q.empty(); });
            if (q.empty()) return;  // stop requested and drained
            Op op = std::move(q.front());
            q.pop_front();
            busy = true;
            const bool skip = op.callback && error != 0;
            g.unlock();
            const int rc = skip ? 0 : op.f();
            g.lock();
            if (rc && !error) error = rc;
            busy = false;
            cv.notify_all();
        }
    }
};

typedef int (*vr_sched_op_fn)(void *user, int op, int slot, uint64_t frame);
enum { OP_RENDER = 0, OP_GATHER = 1, OP_ASSEMBLE = 2, OP_CONSUME = 3, OP_ABORT = 4, OP_ISSUE = 5 };

struct HostExec {
    using Stream = HostStream *;
    using Event = HostEvent *;
    vr_sched_op_fn fn = nullptr;
    void *user = nullptr;
    uint64_t n_records = 0, n_waits = 0;  // cross-stream edges issued (vr_sched_host_edges)

    int record(Event e, Stream s)
    {
        ++n_records;
        uint64_t target;
        {
            std::lock_guard<std::mutex> g(e->m);
            target = ++e->recorded;
        }
        s->push([e, target] {
            {
                std::lock_guard<std::mutex> g(e->m);
                if (target > e->completed) e->completed = target;
            }
            e->cv.notify_all();
            return 0;
        });
        return 0;
    }
    int wait(Stream s, Event e)
    {
        ++n_waits;
        uint64_t target;
        {
            std::lock_guard<std::mutex> g(e->m);
            target = e->recorded;
        }
        s->push([e, target] {
            std::unique_lock<std::mutex> g(e->m);
            e->cv.wait(g, [e, target] { return e->completed >= target; });
            return 0;
        });
        return 0;
    }
    int call(Stream s, int op, int slot, uint64_t frame)
    {
        vr_sched_op_fn f = fn;
        void *u = user;
        s->push([f, u, op, slot, frame] { return f(u, op, slot, frame); }, true);
        return 0;
    }
    int render(int slot, uint64_t frame, Stream s) { return call(s, OP_RENDER, slot, frame); }
    int gather(int slot, uint64_t frame, Stream s) { return call(s, OP_GATHER, slot, frame); }
    int assemble(int slot, uint64_t frame, void *, Stream s)
    {
        return call(s, OP_ASSEMBLE, slot, frame);
    }
};

}  // namespace

struct vr_sched_host {
    HostExec x;
    vr::sched::FrameSchedule<HostExec> sched;
    std::vector<std::unique_ptr<HostStream>> streams;
    std::vector<std::unique_ptr<HostEvent>> events;
    HostStream *caller = nullptr;

    HostStream *new_stream()
    {
        streams.emplace_back(new HostStream());
        return streams.back().get();
    }
    HostEvent *new_event()
    {
        events.emplace_back(new HostEvent());
        return events.back().get();
    }
    int sync()
    {
        int rc = 0;
        for (auto &s : streams) {
            const int r = s->drain();
            if (r && !rc) rc = r;
        }
        return rc;
    }
    ~vr_sched_host()
    {
        sync();
        streams.clear();  // joins the workers before the events go
    }
};

extern "C" {

// rank/frames_in_flight as vr_dist_create; fn(user, op, slot, frame) runs render (0) on slot
// streams, gather (1) on rank 0's caller stream or rank r > 0's slot streams, assemble (2) and
// consume (3) -- the application's use of rank 0's finished frame -- on the caller stream, as
// vr_frame_schedule.h places them.  NULL on bad args.
vr_sched_host *vr_sched_host_create(int rank, int frames_in_flight, vr_sched_op_fn fn, void *user)
{
    if (rank < 0 || frames_in_flight < 1 || frames_in_flight > 8 || !fn) return nullptr;
    vr_sched_host *h = new (std::nothrow) vr_sched_host();
    if (!h) return nullptr;
    h->x.fn = fn;
    h->x.user = user;
    auto &S = h->sched;
    S.rank = rank;
    S.slots.resize(frames_in_flight);
    for (auto &s : S.slots) {
        s.stream = h->new_stream();
        s.rendered = h->new_event();
        s.gathered = h->new_event();
    }
    h->caller = h->new_stream();
    return h;
}

// One frame as vr_dist_render (the same FrameSchedule::issue), then the caller's consume of
// it enqueued on the caller stream behind the frame's done event.
int vr_sched_host_frame(vr_sched_host *h)
{
    if (!h) return -22;
    const uint64_t frame = h->sched.frame;
    int rc = h->sched.issue(h->x, h->caller, nullptr);
    if (rc) return rc;
    return h->x.call(h->caller, OP_CONSUME, (int)(frame % h->sched.slots.size()), frame);
}

// Waits for every op enqueued so far; the first failing callback's code, else 0.
int vr_sched_host_synchronize(vr_sched_host *h) { return h ? h->sync() : -22; }

// Event records and stream waits the schedule has issued so far (each costs host time on HIP).
int vr_sched_host_edges(const vr_sched_host *h, uint64_t *records, uint64_t *waits)
{
    if (!h) return -22;
    if (records) *records = h->x.n_records;
    if (waits) *waits = h->x.n_waits;
    return 0;
}

void vr_sched_host_destroy(vr_sched_host *h) { delete h; }

// ---- multi-device context on host threads ----
typedef int (*vr_group_op_fn)(void *user, int member, int op, int slot, uint64_t frame);

struct vr_group_host;
struct GroupMember {
    vr_group_host *g = nullptr;
    int member = 0;
};

struct vr_group_host {
    vr_group_op_fn fn = nullptr;
    void *user = nullptr;
    std::vector<std::unique_ptr<GroupMember>> tags;
    std::vector<vr_sched_host *> members;
    std::unique_ptr<vr::sched::FrameWorkers<uint64_t>> workers;
    ~vr_group_host()
    {
        workers.reset();
        for (auto *m : members) delete m;
    }
};

static int group_member_op(void *user, int op, int slot, uint64_t frame)
{
    GroupMember *t = static_cast<GroupMember *>(user);
    return t->g->fn(t->g->user, t->member, op, slot, frame);
}

// Stand-in for ncclCommAbort on every member's communicator.
static void group_abort(vr_group_host *g)
{
    for (int m = 0; m < (int)g->members.size(); ++m) g->fn(g->user, m, OP_ABORT, -1, 0);
}

// One frame on member m (rank m of the members): the schedule, plus (member 0) the caller's
// consume of the assembled frame.  fn(OP_ISSUE) first, synchronously on the issuing thread:
// non-zero fails this member's issue (as a vr_dist_render enqueue error would).
static int group_member_frame(vr_group_host *g, int m)
{
    vr_sched_host *h = g->members[m];
    const uint64_t frame = h->sched.frame;
    if (int rc = g->fn(g->user, m, OP_ISSUE, -1, frame)) return rc;
    int rc = h->sched.issue(h->x, h->caller, nullptr);
    if (rc || m != 0) return rc;
    return h->x.call(h->caller, OP_CONSUME, (int)(frame % h->sched.slots.size()), frame);
}

// fn(user, member, op, slot, frame) as vr_sched_host's, with the member index (= its rank).
vr_group_host *vr_group_host_create(int members, int frames_in_flight, vr_group_op_fn fn, void *user)
{
    if (members < 1 || members > 32 || frames_in_flight < 1 || frames_in_flight > 8 || !fn)
        return nullptr;
    vr_group_host *g = new (std::nothrow) vr_group_host();
    if (!g) return nullptr;
    g->fn = fn;
    g->user = user;
    for (int m = 0; m < members; ++m) {
        g->tags.emplace_back(new GroupMember{g, m});
        vr_sched_host *h = vr_sched_host_create(m, frames_in_flight, group_member_op, g->tags.back().get());
        if (!h) {
            delete g;
            return nullptr;
        }
        g->members.push_back(h);
    }
    g->workers.reset(new vr::sched::FrameWorkers<uint64_t>(
        members, [g](int m, const uint64_t &, std::string *) { return group_member_frame(g, m); },
        nullptr));
    return g;
}

int vr_group_host_frame(vr_group_host *g)
{
    if (!g) return -22;
    std::string msg;
    const int rc = g->workers->issue(0, &msg);
    if (rc && !g->workers->aborted()) {  // as vr_dist.cpp group_render: end the collectives now
        std::string m;
        g->workers->settle([g] { group_abort(g); }, &m);
    }
    return rc;
}

// Waits until every member has issued and run every op so far; the first failure, else 0.
// A member whose issue failed aborts the group first (FrameWorkers::settle, as vr_dist.cpp's
// group_synchronize): fn(user, m, OP_ABORT, -1, 0) for every member -- ncclCommAbort on each
// communicator there -- so peers blocked in that frame's collective return instead of hanging.
int vr_group_host_synchronize(vr_group_host *g)
{
    if (!g) return -22;
    std::string msg;
    int rc = g->workers->settle([g] { group_abort(g); }, &msg);
    for (auto *m : g->members) {
        const int r = m->sync();
        if (r && !rc) rc = r;
    }
    return rc;
}

void vr_group_host_destroy(vr_group_host *g) { delete g; }

}  // extern "C"
