// wait_hook.hpp -- the calling thread's one-shot wait hook (rsmi_set_wait_hook, include/rsmi.h):
// a host task that the next codec call runs between launching its device work and waiting for
// it.  Storage and the C entry points are in rsmi_common.cpp (plain C++, shared with the host
// mirror's sanitizer builds).
#pragma once

namespace rsmi {

struct WaitHook {
    void (*fn)(void*) = nullptr;
    void* arg = nullptr;
    explicit operator bool() const { return fn != nullptr; }
    void operator()() const { fn(arg); }
};

// the calling thread's pending hook, cleared (empty when none is set)
WaitHook take_wait_hook();

// run the calling thread's pending hook, if any (a codec call's wait point); the hook is a C
// function, so nothing should escape it, and nothing may escape here with a kernel in flight
inline void run_pending_wait_hook() {
    if (const WaitHook h = take_wait_hook()) {
        try {
            h();
        } catch (...) {
        }
    }
}

}  // namespace rsmi
