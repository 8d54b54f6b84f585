// rsmi_coalesce.cpp -- group commit of concurrent single-block calls (group_commit.hpp has the
// queue).  DagNode.Put hands the engine one block per call (node.go:358-408), from many
// goroutines at once; each executing batch runs its requests grouped by key (kind, shard size
// and, for reconstruct, the erasure pattern) through the host batch paths.

#include "rsmi_impl.hpp"

#include <thread>

#include <cassert>

using namespace rsmi;
using namespace rsmi::impl;

namespace rsmi {
namespace impl {

// page-locked staging of the executing batch (only the executor touches it)
uint8_t* coal_stage(rsmi_ctx* c, size_t need) {
    if (c->h_coal_cap >= need) return c->h_coal;
    if (c->h_coal) (void)hipHostFree(c->h_coal);
    c->h_coal = nullptr;
    c->h_coal_cap = 0;
    if (pinned_alloc(reinterpret_cast<void**>(&c->h_coal), need) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    c->h_coal_cap = need;
    return c->h_coal;
}

// Landing area `slot` of the pipelined table launches' R(shard) (caller holds ctx->mu; the slot's
// previous batch has been finished: a lane has at most two batches in flight, alternating slots)
static uint8_t* pipe_area(rsmi_ctx* c, int slot, size_t bytes) {
    if (c->h_pipe_cap[slot] < bytes) {
        if (c->h_pipe[slot]) (void)hipHostFree(c->h_pipe[slot]);
        c->h_pipe[slot] = nullptr;
        c->h_pipe_cap[slot] = 0;
        const size_t cap = std::max<size_t>(bytes, 64 << 10);
        if (pinned_alloc(reinterpret_cast<void**>(&c->h_pipe[slot]), cap) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        c->h_pipe_cap[slot] = cap;
    }
    return c->h_pipe[slot];
}

// The context's two completion flags (caller holds ctx->mu): page-locked, 64 bytes apart, with
// device counters zeroed on `st` before first use.  The flag page is fine-grained
// (hipHostMallocCoherent, whatever HIP_HOST_COHERENT says): the host spins on it while the kernel
// runs, so the kernel's system-scope release store must reach host memory then, not at the end of
// the kernel.  The R(shard) areas and shard buffers the flag guards may be
// coarse-grained: the launch_done release (every wave: buffer_wbl2 sc0 sc1 + vmcnt(0), then the
// counting atomic at system scope) writes their lines back to host memory before the flag moves.
int done_area(rsmi_ctx* c, hipStream_t st) {
    if (c->h_done) return RSMI_OK;
    void* h = nullptr;
    HIP_TRY(hipHostMalloc(&h, 128, hipHostMallocPortable | hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(h, 0, 128);
    uint8_t* hd = host_alias(h, 128);
    void* d = nullptr;
    hipError_t e = hd ? hipMalloc(&d, 128) : hipErrorInvalidValue;
    if (e == hipSuccess) e = hipMemsetAsync(d, 0, 128, st);  // stream-ordered before the kernels
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        if (d) (void)hipFree(d);
        (void)hipHostFree(h);
        return hip_status(e);
    }
    c->h_done = static_cast<uint32_t*>(h);
    c->h_done_dev = reinterpret_cast<uint32_t*>(hd);
    c->d_done_ctr = static_cast<uint32_t*>(d);
    return RSMI_OK;
}

// Arm a table launch's completion flag (caller holds ctx->mu): the next sequence number, its
// slot's counter and flag in tb; the host view of the flag is done_flag(c, seq)
int arm_flag(rsmi_ctx* c, hipStream_t st, BlockBases& tb, uint32_t& seq) {
    // the flags' slots and counters are ordered by staging[0]'s stream (two launches in flight at
    // most, alternating slots); a flagged launch on another stream would break that order
    assert(st == c->staging[0].stream && "completion flag armed on a stream other than staging[0]");
    int rc = done_area(c, st);
    if (rc) return rc;
    if (++c->done_seq == 0) ++c->done_seq;  // 0 is the flags' first value
    seq = c->done_seq;
    tb.done_ctr = c->d_done_ctr + (seq & 1u) * 16u;
    tb.done_flag = c->h_done_dev + (seq & 1u) * 16u;
    tb.done_seq = seq;
    return RSMI_OK;
}
const uint32_t* done_flag(const rsmi_ctx* c, uint32_t seq) { return c->h_done + (seq & 1u) * 16u; }

// Poll a table launch's completion flag until it holds seq or a later sequence number: a slot's
// flag is released by launches on the context's one stream in sequence order, so a later number
// (a synchronous group of the next batch, queued behind this one) means this launch is done too.
// The poll touches nothing but the flag (a stream or event query every 20 us measured +2 us on a
// 256 KiB call and slowed concurrent lanes' launches); after 200 us the wait blocks in the event
// or stream synchronisation instead, which also reports a failed launch, and a launch that
// finished without its flag is an error.
bool flag_reached(const uint32_t* flag, uint32_t seq) {
    return int32_t(__atomic_load_n(flag, __ATOMIC_ACQUIRE) - seq) >= 0;
}
#ifndef RSMI_FLAG_SPIN_US  // pure spinning for this long, then polls that yield the core (A/B builds)
#define RSMI_FLAG_SPIN_US 200
#endif
int wait_flag(const uint32_t* flag, uint32_t seq, hipStream_t st, hipEvent_t ev) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    const auto until = t0 + std::chrono::microseconds(200), spin = t0 + std::chrono::microseconds(RSMI_FLAG_SPIN_US);
    bool yielding = false;
    for (uint32_t i = 0;; i++) {
        if (flag_reached(flag, seq)) return RSMI_OK;
        if ((i & 63u) == 63u || yielding) {
            const auto now = clk::now();
            if (now > until) break;
            yielding = now > spin;
        }
        if (yielding) std::this_thread::yield();
        else __builtin_ia32_pause();
    }
    const hipError_t e = ev ? hipEventSynchronize(ev) : hipStreamSynchronize(st);
    if (e != hipSuccess) return hip_status(e);
    return flag_reached(flag, seq) ? RSMI_OK : RSMI_ERR_DEVICE;
}

// A group whose requests' shard buffers are page-locked, coded where they lie (see
// run_coalesced_group): one launch over a table of the blocks' bases for up to kTableBlocks
// requests (BlockBases, the table kernels of the BASELINE shapes), else one launch per request,
// and one wait: the completion flag of a one-launch fused encode + CRC-16, else a stream
// synchronisation.  Encode: each block is Split into its own buffer first (the caller's
// block is pageable), outside the context lock -- unless the caller Split it there itself
// (block == out), as the host mirror does, so the copies run on the callers' threads in
// parallel instead of one after another on the executor's.
// fin (option coalesce_pipeline): a group coded by table launches is left in flight behind an
// event, and *fin set to its wait (the R(shard) copies and any error land in the requests then),
// so the executor can launch the next batch first (group_commit.hpp); other groups wait here and
// leave *fin empty.
int run_coalesced_in_place(rsmi_ctx* c, rsmi_ctx::CoalReq* const* rq, size_t nb, size_t S,
                           std::function<void()>* fin) {
    const size_t k = size_t(c->k), n = size_t(c->n);
    const std::string& key = rq[0]->key;
    const bool enc = key[0] == 'E';
    bool want16 = false, want32 = false;
    if (enc)
        for (size_t j = 0; j < nb; j++) {
            if (rq[j]->block != rq[j]->out) std::memcpy(rq[j]->out, rq[j]->block, rq[j]->B);
            std::memset(rq[j]->out + rq[j]->B, 0, k * S - rq[j]->B);  // Split zero-padding
            want16 |= rq[j]->raw != nullptr;
            want32 |= rq[j]->raw32 != nullptr;
        }
    std::vector<uint8_t> present(n), want(n);
    if (!enc) {
        const char* f = key.c_str() + key.find(':') + 1;
        for (size_t i = 0; i < n; i++) {
            present[i] = uint8_t(f[i] == '1');
            want[i] = uint8_t(f[n + i] == '1');
        }
    }
    std::vector<uint32_t> r16(want16 ? nb * n : 0), r32(want32 ? nb * n : 0);
    std::vector<uint8_t*> dev(nb);
    {
        std::lock_guard<std::mutex> g(c->mu);
        HIP_TRY(hipSetDevice(c->device));
        std::shared_ptr<Plan> plan;
        int rc = enc ? encode_plan(c, plan) : reconstruct_plan(c, present.data(), want.data(), plan);
        if (rc) return rc;
        if (want16 && (rc = reserve(c->d_crc, c->crc_cap, nb * n * 4))) return rc;
        if (want32 && (rc = reserve(c->d_crc32, c->crc32_cap, nb * n * 4))) return rc;
        for (size_t j = 0; j < nb; j++)
            if (!(dev[j] = host_alias(rq[j]->out, n * S))) return RSMI_ERR_DEVICE;
        hipStream_t st = c->staging[0].stream;
        // after the first launch an error must not return before the stream is idle: the queued
        // kernels still read and write the callers' buffers, which the callers reuse once told
        // 
        bool launched = false;
        auto fail = [&](int e) {
            if (launched) (void)hipStreamSynchronize(st);
            return e;
        };
        uint32_t* d16 = want16 ? reinterpret_cast<uint32_t*>(c->d_crc) : nullptr;
        uint32_t* d32 = want32 ? reinterpret_cast<uint32_t*>(c->d_crc32) : nullptr;
        // the table form: in / out are offsets from each block's base ([k data | m parity] at
        // pitch S for encode, n rows in place for reconstruct); the CRC-32 keeps a launch per block.
        // The fused kernel's combine writes each R(shard) once, so the table launches store them
        // straight into the page-locked read-back area (no read-back kernel after them)
        bool table = nb >= size_t(RSMI_TABLE_MIN_BLOCKS) && !want32;
        const bool pipe = fin && table && c->opt_coalesce_pipeline;
        const int slot = c->pipe_slot;
        if (pipe && !c->pipe_ev[slot]) HIP_TRY(hipEventCreateWithFlags(&c->pipe_ev[slot], hipEventDisableTiming));
        uint32_t* h16 = nullptr;  // the table launches' R(shard): host view, and its device alias
        uint32_t* h16_dev = nullptr;
        if (table && want16) {
            uint8_t* h = pipe ? pipe_area(c, slot, nb * n * 4) : raw_area(c, nb * n * 4);
            if (!h) return RSMI_ERR_DEVICE;
            h16 = reinterpret_cast<uint32_t*>(h);
            h16_dev = reinterpret_cast<uint32_t*>(host_alias(h, nb * n * 4));
            if (!h16_dev) return RSMI_ERR_DEVICE;
        }
        // a group of one table launch of the fused encode + CRC-16 signals its end through a
        // completion flag (BlockBases::done_flag), polled instead of synchronising the stream
        const uint32_t* flag = nullptr;
        uint32_t seq = 0;
        for (size_t j0 = 0; j0 < nb && table; j0 += size_t(kTableBlocks)) {
            const size_t cnt = std::min(size_t(kTableBlocks), nb - j0);
            BlockBases tb;
            for (size_t i = 0; i < cnt; i++) tb.b[i] = uint64_t(reinterpret_cast<uintptr_t>(dev[j0 + i]));
            uint8_t* const par = reinterpret_cast<uint8_t*>(uintptr_t(k * S));  // offset of the parity rows
            const bool arm = enc && want16 && c->opt_coalesce_flag && nb <= size_t(kTableBlocks);
            if (arm && (rc = arm_flag(c, st, tb, seq))) return fail(rc);
            bool armed = false;
            if (enc && want16)
                rc = launch_plan_crc(c, *plan, nullptr, S, 0, par, S, 0, S, cnt, h16_dev + j0 * n, st, &tb, &armed);
            else if (enc)
                rc = launch_plan(c, *plan, nullptr, S, 0, par, S, 0, S, cnt, st, nullptr, &tb);
            else
                rc = launch_plan(c, *plan, nullptr, S, 0, nullptr, S, 0, S, cnt, st, nullptr, &tb);
            if (rc == RSMI_ERR_INVALID_ARG && j0 == 0) {
                table = false;  // no table kernel for this shape: a launch per request
                break;
            }
            if (rc) return fail(rc);
            launched = true;
            if (armed) flag = done_flag(c, seq);
        }
        if (!table) h16 = nullptr;  // a launch per request: its R(shard) come back by read-back
        if (pipe && table) {
            hipError_t e = hipEventRecord(c->pipe_ev[slot], st);
            if (e != hipSuccess) return fail(hip_status(e));
            c->pipe_slot ^= 1;
            std::vector<rsmi_ctx::CoalReq*> reqs(rq, rq + nb);
            hipEvent_t ev = c->pipe_ev[slot];
            *fin = [reqs = std::move(reqs), ev, h16, n, flag, seq, st]() {
                const int w = flag ? wait_flag(flag, seq, st, ev) : hip_status(hipEventSynchronize(ev));
                for (size_t j = 0; j < reqs.size(); j++) {
                    if (w != RSMI_OK) reqs[j]->rc = w;
                    else if (reqs[j]->raw && h16) std::memcpy(reqs[j]->raw, h16 + j * n, n * 4);
                }
            };
            return RSMI_OK;
        }
        for (size_t j = 0; j < nb && !table; j++) {
            if (enc)
                rc = launch_encode_rows(c, *plan, dev[j], n * S, dev[j] + k * S, n * S, S, 1, d16 ? d16 + j * n : nullptr,
                                        d32 ? d32 + j * n : nullptr, st);
            else
                rc = launch_plan(c, *plan, dev[j], S, n * S, dev[j], S, n * S, S, 1, st);
            if (rc) return fail(rc);
            launched = true;
        }
        const uint32_t *g16 = h16, *g32 = nullptr;
        if (!h16 && (rc = readback(c, d16, d32, nb * n * 4, st, g16, g32))) return fail(rc);
        if (flag) {
            if ((rc = wait_flag(flag, seq, st, nullptr))) return fail(rc);
        } else {
            HIP_TRY(hipStreamSynchronize(st));
        }
        if (want16) std::memcpy(r16.data(), g16, nb * n * 4);
        if (want32) std::memcpy(r32.data(), g32, nb * n * 4);
    }
    for (size_t j = 0; j < nb; j++) {
        if (rq[j]->raw) std::memcpy(rq[j]->raw, r16.data() + j * n, n * 4);
        if (rq[j]->raw32) std::memcpy(rq[j]->raw32, r32.data() + j * n, n * 4);
    }
    return RSMI_OK;
}

// One group of a coalesced batch: same request key, i.e. same kind and shard size (and,
// for reconstruct, the same survivor pattern and requested rows).
void run_coalesced_group(rsmi_ctx* c, rsmi_ctx::CoalReq* const* rq, size_t nb, std::function<void()>* fin) {
    const size_t k = size_t(c->k), m = size_t(c->m), n = k + m;
    const std::string& key = rq[0]->key;
    const size_t S = std::stoull(key.substr(1, key.find(':') - 1));
    // Requests whose shard buffers are all page-locked (the host mirror's block scratch) are coded
    // in place: one zero-copy launch per request on the context's stream and one synchronisation
    // for the group, so neither the staging copy in nor the n*S copy back out happens (per-block
    // DagNode.Put and degraded Gets from many threads)
    bool pinned = true;
    for (size_t j = 0; j < nb && pinned; j++) pinned = host_alias(rq[j]->out, n * S) != nullptr;
    if (pinned) {
        const int rc = run_coalesced_in_place(c, rq, nb, S, fin);
        for (size_t j = 0; j < nb; j++) rq[j]->rc = rc;
        return;
    }
    uint8_t* h = coal_stage(c, nb * n * S);
    if (!h) {
        for (size_t j = 0; j < nb; j++) rq[j]->rc = RSMI_ERR_DEVICE;
        return;
    }
    if (key[0] == 'E') {
        bool want_raw = false, want32 = false;
        for (size_t j = 0; j < nb; j++) {
            uint8_t* dst = h + j * n * S;
            std::memcpy(dst, rq[j]->block, rq[j]->B);
            std::memset(dst + rq[j]->B, 0, k * S - rq[j]->B);  // Split zero-padding
            want_raw |= rq[j]->raw != nullptr;
            want32 |= rq[j]->raw32 != nullptr;
        }
        std::vector<uint32_t> raw(want_raw ? nb * n : 0), raw32(want32 ? nb * n : 0);
        const int rc = encode_host_impl(c, h, n * S, h + k * S, n * S, S, nb, want_raw ? raw.data() : nullptr,
                                        want32 ? raw32.data() : nullptr);
        for (size_t j = 0; j < nb; j++) {
            rq[j]->rc = rc;
            if (rc) continue;
            std::memcpy(rq[j]->out, h + j * n * S, n * S);
            if (rq[j]->raw) std::memcpy(rq[j]->raw, raw.data() + j * n, n * 4);
            if (rq[j]->raw32) std::memcpy(rq[j]->raw32, raw32.data() + j * n, n * 4);
        }
        return;
    }
    // 'R': key = "R<S>:<n flags present><n flags want>"
    const char* f = key.c_str() + key.find(':') + 1;
    std::vector<uint8_t> present(n), want(n);
    for (size_t i = 0; i < n; i++) {
        present[i] = uint8_t(f[i] == '1');
        want[i] = uint8_t(f[n + i] == '1');
    }
    for (size_t j = 0; j < nb; j++) std::memcpy(h + j * n * S, rq[j]->out, n * S);
    const int rc = reconstruct_host_impl(c, h, n * S, S, nb, present.data(), want.data());
    for (size_t j = 0; j < nb; j++) {
        rq[j]->rc = rc;
        if (rc) continue;
        for (size_t i = 0; i < n; i++)
            if (!present[i] && want[i]) std::memcpy(rq[j]->out + i * S, h + (j * n + i) * S, S);
    }
}

// The context that codes lane `lane`'s batches: the context itself for lane 0, else its child
// lane context, opened with the same k, m, device and options on first use.  nullptr with *rc
// set when it cannot be opened.
rsmi_ctx* lane_context(rsmi_ctx* c, int lane, int* rc) {
    *rc = RSMI_OK;
    if (lane == 0) return c;
    std::lock_guard<std::mutex> g(c->lanes_mu);
    if (c->lanes.size() < size_t(lane)) c->lanes.resize(size_t(lane), nullptr);
    rsmi_ctx*& l = c->lanes[size_t(lane - 1)];
    if (l) return l;
    // test hook (option "inject_lane_fault"): this lane's open fails as a device error would,
    // leaving its slot null
    for (int v = c->opt_inject_lane_fault.load(); v > 0;)
        if (c->opt_inject_lane_fault.compare_exchange_weak(v, v - 1)) {
            *rc = RSMI_ERR_DEVICE;
            return nullptr;
        }
    rsmi_ctx* x = nullptr;
    if ((*rc = rsmi_open(c->k, c->m, c->device, &x))) return nullptr;
    {
        // the parent's coding options, read under its lock (rsmi_set_option writes them there;
        // lock order c->lanes_mu, then c->mu, then x->mu, as in rsmi_set_option's lane loop)
        std::lock_guard<std::mutex> gc(c->mu);
        std::lock_guard<std::mutex> gx(x->mu);
        x->opt_crc16_fold = c->opt_crc16_fold;
        x->opt_crc32_fold = c->opt_crc32_fold;
        x->opt_fused_fold = c->opt_fused_fold;
        x->opt_waves_per_cu = c->opt_waves_per_cu;
        x->opt_zero_copy = c->opt_zero_copy;
        x->opt_small_bytes = c->opt_small_bytes;
        x->opt_coalesce_pipeline = c->opt_coalesce_pipeline;
        x->opt_coalesce_flag = c->opt_coalesce_flag;
    }
    {
        std::lock_guard<std::mutex> gx(x->mu);
        *rc = ensure_device(x);
    }
    if (*rc) {
        rsmi_close(x);
        return nullptr;
    }
    l = x;
    return l;
}

std::function<void()> run_coalesced(rsmi_ctx* c, int lane, std::vector<rsmi_ctx::CoalReq*>& batch) {
    const size_t n = size_t(c->n);
    // test hook (option "inject_host_fault"): this batch fails as a host allocation would
    for (int v = c->opt_inject_host_fault.load(); v > 0;)
        if (c->opt_inject_host_fault.compare_exchange_weak(v, v - 1)) throw std::bad_alloc();
    int rc;
    rsmi_ctx* x = lane_context(c, lane, &rc);
    if (!x) {
        for (auto* r : batch) r->rc = rc;
        return nullptr;
    }
    std::map<std::string, std::vector<rsmi_ctx::CoalReq*>> groups;
    for (auto* r : batch) groups[r->key].push_back(r);
    // a batch of one group that one launch sequence codes may be left in flight (pipelined)
    std::function<void()> fin;
    for (auto& g : groups) {
        const std::string& key = g.first;
        const size_t S = std::stoull(key.substr(1, key.find(':') - 1));
        const size_t chunk = std::max<size_t>(1, (size_t(64) << 20) / (n * S));
        const bool one = groups.size() == 1 && g.second.size() <= chunk;
        for (size_t j0 = 0; j0 < g.second.size(); j0 += chunk)
            run_coalesced_group(x, g.second.data() + j0, std::min(chunk, g.second.size() - j0), one ? &fin : nullptr);
    }
    if (x != c) set_last_kernel(c, rsmi_last_kernel(x));
    return fin;
}

// Queue a request and either wait for an executor or become one (group_commit.hpp).  The device
// check takes no lock once the context is bound, so callers queue while a batch is being coded
// (under the lock) instead of waiting behind it.
// The calling thread's wait hook (rsmi_set_wait_hook) goes in as the caller's idle task: run
// while another thread's batch codes its request, or once its own lone batch is launched.
int coalesce(rsmi_ctx* c, rsmi_ctx::CoalReq& req) {
    int rc = ensure_device_fast(c);
    if (rc) return rc;
    const WaitHook h = take_wait_hook();
    c->coal.submit(req, size_t(c->opt_coalesce_max), c->opt_coalesce_us, int(c->opt_coalesce_lanes),
                   [c](std::vector<rsmi_ctx::CoalReq*>& batch, int lane) { return run_coalesced(c, lane, batch); },
                   int(c->opt_coalesce_carry), h.fn, h.arg);
    return req.rc;
}

}  // namespace impl
}  // namespace rsmi

extern "C" {

int rsmi_encode_block_coalesced_crcs(rsmi_ctx* c, const uint8_t* block, size_t B, uint8_t* shards_out,
                                     uint32_t* raw16_out, uint32_t* raw32_out) try {
    if (!c) return RSMI_ERR_INVALID_ARG;
    if (B == 0) return RSMI_ERR_SHORT_DATA;
    if (!block || !shards_out) return RSMI_ERR_INVALID_ARG;
    rsmi_ctx::CoalReq req{block, B, shards_out, raw16_out, raw32_out, "E" + std::to_string(rsmi_shard_size(B, c->k)) + ":",
                          RSMI_OK, false};
    return coalesce(c, req);
} catch (...) {
    return rsmi::impl::exception_status();
}

int rsmi_encode_block_coalesced(rsmi_ctx* c, const uint8_t* block, size_t B, uint8_t* shards_out,
                                uint32_t* raw_out) try {
    return rsmi_encode_block_coalesced_crcs(c, block, B, shards_out, raw_out, nullptr);
} catch (...) {
    return rsmi::impl::exception_status();
}

int rsmi_reconstruct_coalesced(rsmi_ctx* c, uint8_t* shards, size_t S, const uint8_t* present, int data_only) try {
    if (!c || !shards || !present) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    const std::vector<uint8_t> want = want_mask(c, present, data_only);
    int pre = reconstruct_precheck(c, present, want.data());
    if (pre < 0) return -pre;
    if (pre == 1) return RSMI_OK;
    std::string key = "R" + std::to_string(S) + ":";
    for (int i = 0; i < c->n; i++) key.push_back(present[i] ? '1' : '0');
    for (int i = 0; i < c->n; i++) key.push_back(want[i] ? '1' : '0');
    rsmi_ctx::CoalReq req{nullptr, 0, shards, nullptr, nullptr, std::move(key), RSMI_OK, false};
    return coalesce(c, req);
} catch (...) {
    return rsmi::impl::exception_status();
}

int rsmi_warm(rsmi_ctx* c) try {
    if (!c) return RSMI_ERR_INVALID_ARG;
    int rc = ensure_device_fast(c);
    if (rc) return rc;
    // one tiny in-place encode + CRC-16 per lane (S = 64: the fused kernel), as a lone request of
    // that lane, so each lane's context binds its streams, plan, tables and read-back area now
    const size_t n = size_t(c->n), S = 64, B = size_t(c->k) * S;
    uint8_t* buf = nullptr;
    if (pinned_alloc(reinterpret_cast<void**>(&buf), n * S) != hipSuccess) {
        (void)hipGetLastError();
        return RSMI_ERR_DEVICE;
    }
    std::memset(buf, 1, B);
    std::vector<uint32_t> raw(n);
    for (int lane = 0; lane < int(c->opt_coalesce_lanes) && rc == RSMI_OK; lane++) {
        rsmi_ctx* x = lane_context(c, lane, &rc);
        if (!x) break;
        rsmi_ctx::CoalReq req{buf, B, buf, raw.data(), nullptr, "E" + std::to_string(S) + ":", RSMI_OK, false};
        rsmi_ctx::CoalReq* r = &req;
        run_coalesced_group(x, &r, 1, nullptr);
        rc = req.rc;
    }
    (void)hipHostFree(buf);
    return rc;
} catch (...) {
    return rsmi::impl::exception_status();
}

long rsmi_get_stat(const rsmi_ctx* c, const char* key) {
    if (!c || !key) return -1;
    if (!std::strcmp(key, "coalesced_calls")) return long(c->coal.calls());
    if (!std::strcmp(key, "coalesced_batches")) return long(c->coal.batches());
    if (!std::strcmp(key, "coalesced_wakes")) return long(c->coal.wakes());
    if (!std::strcmp(key, "coalesced_wake_ns")) return long(c->coal.wake_ns());
    return -1;
}

}  // extern "C"
