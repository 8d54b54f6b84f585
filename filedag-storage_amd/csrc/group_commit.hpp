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
// next executor could: with 16 callers that convoy cost more than a small batch's launch.)  An
// executor that leaves callers queued while a lane is free (a batch capped at `cap`) wakes the
// first of them too, so two lanes released together cannot leave a free lane idle.
//
// Idle work (rsmi_set_wait_hook): a caller may hand submit a host task of its own to run while
// its request is coded.  A caller that waits for another thread's batch runs it before it first
// sleeps (it then checks the queue again, so a lane freed meanwhile is not lost: a released lane
// wakes the first queued caller that is not inside its task).  An executor whose batch is its own
// request alone runs it once the batch is launched, before the batch's wait; an executor coding
// other callers' requests runs it after they are completed, so none of them waits for it.  Either
// way it runs exactly once, before submit returns.
//
// Pipelined batches: exec may return a finisher (a callable; empty or exec returning void: the
// batch ran to completion) instead of waiting for its own work.  The executor then launches the
// next queued batch (within `carry`) behind it before it calls the finisher, so the device is
// handed the next batch while the host waits for the current one; a batch's callers return once
// its finisher has run, and finishers run in launch order.
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <mutex>
#include <type_traits>
#include <vector>

#ifndef RSMI_GC_SPIN_US
#define RSMI_GC_SPIN_US 0
#endif
// 1: a caller with an idle task runs it before it would execute a batch as well, so the callers
// queued meanwhile join that batch (A/B builds; 0, the default: only while waiting, see above)
#ifndef RSMI_GC_IDLE_FIRST
#define RSMI_GC_IDLE_FIRST 0
#endif

namespace rsmi {

template <class Req>
class GroupCommit {
public:
    static constexpr int kMaxLanes = 32;
    explicit GroupCommit(int fail_rc) : fail_rc_(fail_rc) {}
    // carry: batches a lane runs after its own before it hands over (0: hand over at once)
    // idle (may be null): the caller's own host task, run once on this thread (see above)
    template <class Exec>
    void submit(Req& req, size_t cap, long wait_us, int lanes, Exec&& exec, int carry = 0,
                void (*idle)(void*) = nullptr, void* idle_arg = nullptr) {
        calls_++;
        lanes = std::min(std::max(lanes, 1), kMaxLanes);
        cap = std::max<size_t>(cap, 1);
        Waiter me;
        me.req = &req;
        std::unique_lock<std::mutex> lk(mu_);
        pending_.push_back(&me);
        me.queued = true;
        fill_cv_.notify_one();  // an executor waiting out wait_us may now have enough
        // the idle task, unlocked; returns with lk held
        auto run_idle = [&]() {
            void (*fn)(void*) = idle;
            idle = nullptr;
            me.in_idle = true;
            lk.unlock();
            try {
                fn(idle_arg);
            } catch (...) {  // the caller's task: its failure is its own, the batch goes on
            }
            lk.lock();
            me.in_idle = false;
        };
        while (!req.done) {
            // only a caller whose own request is still queued executes: it is then certain to
            // find work, and a caller whose request is already in a batch just waits for it
            if (!me.queued || executing_ >= lanes || (RSMI_GC_IDLE_FIRST && idle)) {
                if (idle) {
                    run_idle();  // then look again: a lane may have been freed meanwhile
                    continue;
                }
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
            // when requests are queued by then; a batch whose exec left work in flight (a
            // finisher) has the next one launched behind it before it is finished
            std::deque<Flight> flights;
            int started = 0;
            auto start = [&]() {  // under lk; launches unlocked and returns with lk held
                if (pending_.empty() || started > carry) return;
                started++;
                const size_t take = std::min(cap, pending_.size());
                Flight f;
                try {
                    f.batch.assign(pending_.begin(), pending_.begin() + take);
                    f.reqs.reserve(take);
                    for (Waiter* w : f.batch) f.reqs.push_back(w->req);
                } catch (...) {  // no memory for the batch list: fail these requests in place
                    for (size_t i = 0; i < take; i++) {
                        pending_[i]->queued = false;
                        pending_[i]->req->rc = fail_rc_;
                        pending_[i]->req->done = true;
                        if (pending_[i] != &me) wake(*pending_[i]);
                    }
                    pending_.erase(pending_.begin(), pending_.begin() + take);
                    return;
                }
                for (Waiter* w : f.batch) w->queued = false;
                pending_.erase(pending_.begin(), pending_.begin() + take);
                // a batch capped at `cap` leaves callers queued: with a lane free, the first of
                // them executes the next batch now instead of waiting for this lane
                if (!pending_.empty() && executing_ < lanes) wake_next();
                lk.unlock();
                try {
                    if constexpr (std::is_void_v<std::invoke_result_t<Exec&, std::vector<Req*>&, int>>)
                        exec(f.reqs, lane);
                    else
                        f.fin = exec(f.reqs, lane);
                } catch (...) {
                    for (Req* r : f.reqs) r->rc = fail_rc_;
                    f.fin = nullptr;
                }
                batches_++;
                lk.lock();
                try {
                    flights.push_back(std::move(f));
                } catch (...) {  // cannot track it: finish it here
                    lk.unlock();
                    if (f.fin) finish(f);
                    lk.lock();
                    complete(f, me);
                }
            };
            start();
            while (!flights.empty()) {
                if (flights.size() == 1 && flights.front().fin) start();  // the next, behind it
                Flight f = std::move(flights.front());
                flights.pop_front();
                // a batch of this caller's request alone: its idle task overlaps the batch's work
                if (idle && f.fin && f.batch.size() == 1 && f.batch[0] == &me) run_idle();
                if (f.fin) {
                    lk.unlock();
                    finish(f);
                    lk.lock();
                }
                complete(f, me);  // this batch's callers return now, whatever the lane does next
                if (flights.empty()) start();
            }
            busy_ &= ~(uint64_t(1) << lane);
            executing_--;
            if (!pending_.empty()) wake_next();  // the next batch's executor
        }
        if (idle) run_idle();  // an executor of other callers' requests too: after they returned
    }
    uint64_t calls() const { return calls_.load(); }
    uint64_t batches() const { return batches_.load(); }
    // wake-ups of sleeping callers and the time from each wake() to the caller running again
    // (diagnostic: the scheduler's wake-up latency under the group commit)
    uint64_t wakes() const { return wakes_.load(); }
    uint64_t wake_ns() const { return wake_ns_.load(); }

private:
    struct Waiter;
    struct Flight {
        std::vector<Waiter*> batch;
        std::vector<Req*> reqs;
        std::function<void()> fin;  // the batch's wait, when exec left it in flight
    };
    void finish(Flight& f) {
        try {
            f.fin();
        } catch (...) {
            for (Req* r : f.reqs) r->rc = fail_rc_;
        }
    }
    // caller holds mu_
    static void complete(Flight& f, Waiter& me) {
        for (Waiter* w : f.batch) {
            w->req->done = true;
            if (w != &me) wake(*w);
        }
    }
    struct Waiter {
        Req* req = nullptr;
        bool queued = false;   // in pending_ (under mu_)
        bool in_idle = false;  // running its idle task, not asleep (under mu_)
        std::mutex m;
        std::condition_variable cv;
        bool woken = false;            // under m
        std::atomic<bool> ready{false};  // woken, readable without m (the spin before the sleep)
        std::chrono::steady_clock::time_point woke_at;  // under m: when wake() ran
    };
    // wake a waiting caller (caller holds mu_: lock order mu_, then the waiter's m)
    static void wake(Waiter& w) {
        {
            std::lock_guard<std::mutex> g(w.m);
            w.woken = true;
            w.woke_at = std::chrono::steady_clock::now();
            w.ready.store(true, std::memory_order_release);
        }
        w.cv.notify_one();
    }
    // wake the first queued caller that is not inside its idle task (it would take the free lane
    // only once the task ends), else the first (caller holds mu_, pending_ not empty)
    void wake_next() {
        for (Waiter* w : pending_)
            if (!w->in_idle) {
                wake(*w);
                return;
            }
        wake(*pending_.front());
    }
    // sleep until woken; mu_ is released meanwhile and held again on return.  With
    // RSMI_GC_SPIN_US > 0 the caller first spins that long on the waiter's flag, so a batch that
    // completes within it costs no futex wake-up (A/B builds; default 0: sleep at once)
    void sleep(Waiter& w, std::unique_lock<std::mutex>& lk) {
        std::unique_lock<std::mutex> g(w.m);
        w.woken = false;  // under mu_ and m: no wake-up can fall between the caller's check and here
        w.ready.store(false, std::memory_order_relaxed);
        lk.unlock();
        if (RSMI_GC_SPIN_US > 0) {
            g.unlock();
            const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(RSMI_GC_SPIN_US);
            for (uint32_t i = 0; !w.ready.load(std::memory_order_acquire); i++) {
                if ((i & 63u) == 63u && std::chrono::steady_clock::now() > until) break;
#if defined(__x86_64__)
                __builtin_ia32_pause();
#endif
            }
            g.lock();
        }
        w.cv.wait(g, [&] { return w.woken; });
        wakes_++;
        wake_ns_ += uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() -
                                                                                  w.woke_at).count());
        g.unlock();
        lk.lock();
    }
    std::mutex mu_;
    std::condition_variable fill_cv_;  // an executor waiting out wait_us for the queue to fill
    std::vector<Waiter*> pending_;
    int executing_ = 0;
    uint64_t busy_ = 0;  // lanes with a batch executing
    const int fail_rc_;
    std::atomic<uint64_t> calls_{0}, batches_{0}, wakes_{0}, wake_ns_{0};
};

}  // namespace rsmi
