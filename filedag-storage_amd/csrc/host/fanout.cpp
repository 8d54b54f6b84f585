// fanout.cpp -- see fanout.hpp.
#include "fanout.hpp"

namespace rsmi {
namespace host {

FanOut::FanOut(int workers) {
    for (int w = 0; w < workers; w++)
        threads_.emplace_back([this] {
            std::unique_lock<std::mutex> lk(mu_);
            for (;;) {
                work_cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
                if (stop_ && q_.empty()) return;
                const Task t = q_.front();
                q_.pop_front();
                lk.unlock();
                execute(t);
                lk.lock();
            }
        });
}

FanOut::~FanOut() {
    {
        std::lock_guard<std::mutex> g(mu_);
        stop_ = true;
    }
    work_cv_.notify_all();
    for (auto& t : threads_) t.join();
}

void FanOut::execute(const Task& t) {
    (*t.job->f)(t.i);
    std::lock_guard<std::mutex> g(mu_);
    if (--t.job->remaining == 0) done_cv_.notify_all();
}

void FanOut::run(int n, const std::function<void(int)>& f) {
    if (n <= 0) return;
    if (n == 1 || threads_.empty()) {
        for (int i = 0; i < n; i++) f(i);
        return;
    }
    Job job{&f, n};
    std::unique_lock<std::mutex> lk(mu_);
    for (int i = 1; i < n; i++) q_.push_back(Task{&job, i});
    work_cv_.notify_all();
    lk.unlock();
    f(0);  // the caller's own share
    lk.lock();
    --job.remaining;
    while (job.remaining > 0) {
        if (!q_.empty()) {  // help: run whatever is queued (ours or another caller's)
            const Task t = q_.front();
            q_.pop_front();
            lk.unlock();
            execute(t);
            lk.lock();
            continue;
        }
        done_cv_.wait(lk);
    }
}

}  // namespace host
}  // namespace rsmi
