// fanout.hpp -- the datanode fan-out of the Dag Node mirror.
//
// node.go runs one goroutine per datanode for Put (:376-399), Get (:234-270), readAllMeta
// (:450-489) and DeleteBlock (:191-208), so the k+m datanode calls of one block proceed at
// once.  FanOut gives the C++ mirror the same concurrency: a small persistent pool shared by
// every caller thread.  A caller queues its n calls, runs queued calls itself while it waits
// (so concurrent callers never deadlock on a busy pool), and returns when its own n are done.
// Callers replay the results in node order, so the quorum outcome is the sequential one.
#pragma once
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace rsmi {
namespace host {

class FanOut {
public:
    explicit FanOut(int workers);
    ~FanOut();
    FanOut(const FanOut&) = delete;
    FanOut& operator=(const FanOut&) = delete;
    // f(i) for every i in [0, n); returns once all n have run
    void run(int n, const std::function<void(int)>& f);

private:
    struct Job {
        const std::function<void(int)>* f;
        int remaining;
    };
    struct Task {
        Job* job;
        int i;
    };
    void execute(const Task& t);
    std::mutex mu_;
    std::condition_variable work_cv_, done_cv_;
    std::deque<Task> q_;
    std::vector<std::thread> threads_;
    bool stop_ = false;
};

}  // namespace host
}  // namespace rsmi
