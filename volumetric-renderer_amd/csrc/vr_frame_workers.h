// vr_frame_workers.h — the host side of a multi-device context (vr_create_mask, vr.h): one
// frame is issued on every device of the context, member 0 on the calling thread and each
// other member on its own worker thread, so the per-device enqueue work (render launch,
// events, ncclGather, about 25-35 us per member) runs in parallel instead of adding up.
//
// Written once against a per-member issue function, so the same code drives the HIP members
// (vr_dist.cpp: vr::sched::FrameSchedule on HIP streams + RCCL) and the host-thread members of
// the CPU test (vr_sched_host.cpp, tests/test_sched_host.py).
//
// Ordering: every member receives the frames in the order issue() is called (one FIFO queue
// per worker), which is what the collective needs: each member's ncclGather calls are issued
// in frame order on its communicator.  issue() returns once member 0's frame is enqueued;
// the other members' enqueues may still be running.  drain() waits for them (callers drain
// before changing what the members render from: volume, TF, slicing, size).
//
// Errors are sticky per worker: the first failing issue is reported by the next issue() or
// drain(), with its message, and the worker skips its later jobs (the frame stream on that
// member is broken; the context must be destroyed).
//
// A failed member breaks the collective: its peers have already issued (or will issue) their
// gathers of that frame, which can never be matched, so their streams would wait forever.
// settle(abort) is the one place that resolves this for both executors: it drains the
// enqueues, and if any member (member 0 included) failed it calls abort() once -- the HIP
// executor aborts every communicator (ncclCommAbort), which ends the pending collectives --
// before the caller synchronises any stream.  After that every issue() fails.
#pragma once

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace vr {
namespace sched {

template <class Job>
class FrameWorkers {
  public:
    // issue(member, job): enqueue one frame on that member, 0 or a negative code (message via
    // *msg).  init(member) runs once on the member's thread before its first job (e.g. binds
    // the thread to the member's device).
    using IssueFn = std::function<int(int member, const Job &job, std::string *msg)>;
    using InitFn = std::function<void(int member)>;

    FrameWorkers(int members, IssueFn issue, InitFn init) : issue_(std::move(issue))
    {
        for (int m = 1; m < members; ++m) {
            workers_.emplace_back(new Worker());
            Worker *w = workers_.back().get();
            w->th = std::thread([this, w, m, init] {
                if (init) init(m);
                run(w, m);
            });
        }
    }
    ~FrameWorkers()
    {
        for (auto &w : workers_) {
            {
                std::lock_guard<std::mutex> g(w->m);
                w->stop = true;
            }
            w->cv.notify_all();
        }
        for (auto &w : workers_) w->th.join();
    }
    FrameWorkers(const FrameWorkers &) = delete;
    FrameWorkers &operator=(const FrameWorkers &) = delete;

    int members() const { return (int)workers_.size() + 1; }

    // One frame on every member: members 1.. get the job on their threads, member 0 runs it
    // here.  A failure already recorded on a worker is returned first.
    int issue(const Job &job, std::string *msg)
    {
        if (aborted_) {
            if (msg) *msg = "a device member failed and the frame collectives were aborted: "
                            "destroy the context (" + first_msg_ + ")";
            return first_rc_ ? first_rc_ : -5;
        }
        if (int rc = sticky(msg)) return rc;
        for (auto &w : workers_) {
            {
                std::lock_guard<std::mutex> g(w->m);
                w->q.push_back(job);
            }
            w->cv.notify_one();
        }
        const int rc = issue_(0, job, msg);
        if (rc && !failed0_) {
            failed0_ = rc;
            failed0_msg_ = "device member 0: " + (msg ? *msg : std::string());
        }
        return rc;
    }

    // Drains the enqueues; if any member failed (now or before), calls abort() once and
    // returns that member's error (message in *msg), else 0.  Call before synchronising the
    // members' streams.
    int settle(const std::function<void()> &abort, std::string *msg)
    {
        std::string m;
        int rc = drain(&m);
        if (!rc && failed0_) {
            rc = failed0_;
            m = failed0_msg_;
        }
        if (!rc && aborted_) {
            rc = first_rc_;
            m = first_msg_;
        }
        if (rc && !aborted_) {
            aborted_ = true;
            first_rc_ = rc;
            first_msg_ = m;
            if (abort) abort();
        }
        if (rc && msg) *msg = m;
        return rc;
    }

    bool aborted() const { return aborted_; }

    // Waits until every member has issued every frame posted so far; the first worker error.
    int drain(std::string *msg)
    {
        for (auto &w : workers_) {
            std::unique_lock<std::mutex> g(w->m);
            w->cv.wait(g, [&] { return w->q.empty() && !w->busy; });
        }
        return sticky(msg);
    }

  private:
    struct Worker {
        std::thread th;
        std::mutex m;
        std::condition_variable cv;
        std::deque<Job> q;
        bool stop = false, busy = false;
        int err = 0;
        std::string msg;
    };

    int sticky(std::string *msg)
    {
        for (auto &w : workers_) {
            std::lock_guard<std::mutex> g(w->m);
            if (w->err) {
                if (msg) *msg = w->msg;
                return w->err;
            }
        }
        return 0;
    }

    void run(Worker *w, int member)
    {
        std::unique_lock<std::mutex> g(w->m);
        for (;;) {
            w->cv.wait(g, [w] { return w->stop || !w->q.empty(); });
            if (w->q.empty()) return;  // stop requested, queue drained
            Job job = std::move(w->q.front());
            w->q.pop_front();
            w->busy = true;
            const bool skip = w->err != 0;
            g.unlock();
            std::string m;
            const int rc = skip ? 0 : issue_(member, job, &m);
            g.lock();
            if (rc && !w->err) {
                w->err = rc;
                w->msg = "device member " + std::to_string(member) + ": " + m;
            }
            w->busy = false;
            w->cv.notify_all();
        }
    }

    IssueFn issue_;
    std::vector<std::unique_ptr<Worker>> workers_;
    // member 0's failure (it runs on the caller's thread) and the abort state; touched only
    // by the caller's thread (issue / settle)
    int failed0_ = 0, first_rc_ = 0;
    bool aborted_ = false;
    std::string failed0_msg_, first_msg_;
};

}  // namespace sched
}  // namespace vr
