// group_commit.hpp -- group commit of concurrent single-item requests, with no thread of its own
// (rsmi_coalesce.cpp; plain C++, so tests/cpp runs it under ThreadSanitizer without a device).
//
// DagNode.Put hands the engine one block per call (node.go:358-408) from many goroutines at
// once.  A caller whose request is still queued and that finds a free lane becomes that lane's
// executor: it takes every request queued so far (optionally waiting up to wait_us for the queue
// to reach cap), runs them as one batch through exec(batch, lane) with the lock released, marks
// them done and wakes their callers.  Up to `lanes` batches execute at once, each on its own lane
// (0 .. lanes-1, distinct among the batches executing), so one batch can be launched while the
// one before it is still coded; requests that arrive while every lane is busy form the next
// batch.  A lone caller never waits: its batch is itself.  An executor may go on to up to `carry`
// further batches queued by the time its own completes (its caller returns that much later, and
// no thread is woken per batch).  Req needs a `bool done` member, false on submission, and an
// `int rc`.  If exec throws (std::bad_alloc from its own vectors), every request of the batch
// completes with rc = the fail code given at construction and the lane is released, so no
// current or later caller waits forever; the exception does not cross the C-ABI.
//
// Wake-ups are targeted: every waiting caller sleeps on its own condition variable, a finished
// batch wakes exactly its own callers, and a released lane wakes the first queued caller to
// execute the next batch.  (One shared condition variable woke every waiting caller at each
// batch's end, and the woken callers then took the queue's lock one after another before the
// next executor could: with 16 callers that convoy cost more than a small batch's launch.)
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <vector>

namespace rsmi {

template <class Req>
class GroupCommit {
public:
    static constexpr int kMaxLanes = 32;
    explicit GroupCommit(int fail_rc) : fail_rc_(fail_rc) {}
    // carry: batches a lane runs after its own before it hands over (0: hand over at once)
    template <class Exec>
    void submit(Req& req, size_t cap, long wait_us, int lanes, Exec&& exec, int carry = 0) {
        calls_++;
        lanes = std::min(std::max(lanes, 1), kMaxLanes);
        cap = std::max<size_t>(cap, 1);
        Waiter me;
        me.req = &req;
        std::unique_lock<std::mutex> lk(mu_);
        pending_.push_back(&me);
        me.queued = true;
        fill_cv_.notify_one();  // an executor waiting out wait_us may now have enough
        while (!req.done) {
            // only a caller whose own request is still queued executes: it is then certain to
            // find work, and a caller whose request is already in a batch just waits for it
            if (!me.queued || executing_ >= lanes) {
                sleep(me, lk);
                continue;
            }
            int lane = 0;
            while (busy_ & (uint64_t(1) << lane)) lane++;
            busy_ |= uint64_t(1) << lane;
            executing_++;
            if (wait_us > 0 && pending_.size() < cap)
                fill_cv_.wait_for(lk, std::chrono::microseconds(wait_us), [&] { return pending_.size() >= cap; });
            // the batch that holds this caller's request, then up to `carry` more on the same lane
            // when requests are queued by then
            for (int round = 0; round <= carry && !pending_.empty(); round++) {
                const size_t take = std::min(cap, pending_.size());
                std::vector<Waiter*> batch;
                std::vector<Req*> reqs;
                try {
                    batch.assign(pending_.begin(), pending_.begin() + take);
                    reqs.reserve(take);
                    for (Waiter* w : batch) reqs.push_back(w->req);
                } catch (...) {  // no memory for the batch list: fail these requests in place
                    for (size_t i = 0; i < take; i++) {
                        pending_[i]->queued = false;
                        pending_[i]->req->rc = fail_rc_;
                        pending_[i]->req->done = true;
                        wake(*pending_[i]);
                    }
                    pending_.erase(pending_.begin(), pending_.begin() + take);
                    break;
                }
                for (Waiter* w : batch) w->queued = false;
                pending_.erase(pending_.begin(), pending_.begin() + take);
                lk.unlock();
                try {
                    exec(reqs, lane);
                } catch (...) {
                    for (Req* r : reqs) r->rc = fail_rc_;
                }
                batches_++;
                lk.lock();
                for (Waiter* w : batch) {  // this batch's callers return now, whatever the lane does next
                    w->req->done = true;
                    if (w != &me) wake(*w);
                }
            }
            busy_ &= ~(uint64_t(1) << lane);
            executing_--;
            if (!pending_.empty()) wake(*pending_.front());  // the next batch's executor
        }
    }
    uint64_t calls() const { return calls_.load(); }
    uint64_t batches() const { return batches_.load(); }

private:
    struct Waiter {
        Req* req = nullptr;
        bool queued = false;  // in pending_ (under mu_)
        std::mutex m;
        std::condition_variable cv;
        bool woken = false;  // under m
    };
    // wake a waiting caller (caller holds mu_: lock order mu_, then the waiter's m)
    static void wake(Waiter& w) {
        {
            std::lock_guard<std::mutex> g(w.m);
            w.woken = true;
        }
        w.cv.notify_one();
    }
    // sleep until woken; mu_ is released meanwhile and held again on return
    static void sleep(Waiter& w, std::unique_lock<std::mutex>& lk) {
        std::unique_lock<std::mutex> g(w.m);
        w.woken = false;  // under mu_ and m: no wake-up can fall between the caller's check and here
        lk.unlock();
        w.cv.wait(g, [&] { return w.woken; });
        g.unlock();
        lk.lock();
    }
    std::mutex mu_;
    std::condition_variable fill_cv_;  // an executor waiting out wait_us for the queue to fill
    std::vector<Waiter*> pending_;
    int executing_ = 0;
    uint64_t busy_ = 0;  // lanes with a batch executing
    const int fail_rc_;
    std::atomic<uint64_t> calls_{0}, batches_{0};
};

}  // namespace rsmi
