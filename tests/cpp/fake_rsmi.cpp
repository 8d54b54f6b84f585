// fake_rsmi.cpp -- TEST INFRASTRUCTURE, never linked into the product.
//
// A stand-in for the device entry points of include/rsmi.h that the C++ host mirror calls
// (csrc/host/*), coding with the CPU oracle (oracle/rs_oracle.c) and the host CRC halves, so
// the mirror's concurrency -- datanode fan-out, quorum replay, the read-repair queue and
// worker, GetMany / PutMany key concurrency, and the group-commit queue itself (the product's
// csrc/group_commit.hpp, used here unchanged) -- runs under ThreadSanitizer and
// AddressSanitizer on a host without a GPU (tests/cpp/Makefile sanitizer targets).  The
// device-free entry points (status strings, shard checks, checksum host halves) are the
// product's own csrc/rsmi_common.cpp.  Outputs are checked against the oracle by the tests as
// usual; what the sanitizers check is the host code around the calls.
//
// FAKE_RSMI_FAST (tools/Makefile bench_dagnode_cpu): the same layer with the multi-threaded SIMD
// twin of the oracle (oracle/rs_cpu_fast.c, AVX-512 GFNI) and carry-less CRC folding, so the Dag
// Node mirror runs end to end on a CPU codec -- the reference's own shape (klauspost encode on
// host cores, erasure.go:37) -- and tools/bench_dagnode can time it beside the GPU build.
// Batches split their blocks over FAKE_RSMI_THREADS (default OMP_NUM_THREADS, else every core)
// threads; a single block codes on the calling thread.
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>
#ifdef FAKE_RSMI_FAST
#include "../../filedag-storage_amd/csrc/host/crc_clmul.hpp"
#endif

#include "../../filedag-storage_amd/csrc/crc16.hpp"
#include "../../filedag-storage_amd/csrc/crc32.hpp"
#include "../../filedag-storage_amd/csrc/group_commit.hpp"
#include "../../filedag-storage_amd/csrc/wait_hook.hpp"
#include "../../include/rsmi.h"
#include "../../oracle/rs_oracle.h"

namespace {

struct Req {
    bool encode;
    const uint8_t* block;
    size_t B;
    uint8_t* out;  // encode: (k+m)*S shards; reconstruct: n*S shards in place
    size_t S;
    const uint8_t* present;
    int data_only;
    uint32_t* raw16;
    uint32_t* raw32;
    int rc;
    bool done;
};

#ifdef FAKE_RSMI_FAST
uint32_t r16(const uint8_t* p, size_t n) {
    bool done = false;
    const uint32_t s = rsmi::host::clmul_crc16(0, p, n, &done);
    return done ? s : rsmi::crc16_tables().fold(0, p, n);
}
uint32_t r32(const uint8_t* p, size_t n) {
    bool done = false;
    const uint32_t s = rsmi::host::clmul_crc32(0, p, n, &done);
    return done ? s : rsmi::crc32_tables().fold(0, p, n);
}
int cpu_threads() {
    for (const char* v : {"FAKE_RSMI_THREADS", "OMP_NUM_THREADS"}) {
        const char* e = std::getenv(v);
        if (e && std::atoi(e) > 0) return std::atoi(e);
    }
    return int(std::max(1u, std::thread::hardware_concurrency()));
}
// f(b0, b1) over [0, nblocks) split into contiguous ranges on up to cpu_threads() threads; the
// first nonzero status
template <class F>
int par_blocks(size_t nblocks, F f) {
    const size_t T = std::min<size_t>(size_t(cpu_threads()), nblocks);
    if (T <= 1) return f(size_t(0), nblocks);
    std::vector<int> rc(T, 0);
    std::vector<std::thread> th;
    for (size_t t = 1; t < T; t++) th.emplace_back([&, t] { rc[t] = f(nblocks * t / T, nblocks * (t + 1) / T); });
    rc[0] = f(0, nblocks / T);
    for (auto& x : th) x.join();
    for (int r : rc)
        if (r) return r;
    return 0;
}
#else
uint32_t r16(const uint8_t* p, size_t n) { return rsmi::crc16_tables().fold(0, p, n); }
uint32_t r32(const uint8_t* p, size_t n) { return rsmi::crc32_tables().fold(0, p, n); }
template <class F>
int par_blocks(size_t nblocks, F f) {
    return f(size_t(0), nblocks);
}
#endif

}  // namespace

struct rsmi_ctx {
    int k = 0, m = 0, n = 0;
    rsmi::GroupCommit<Req> coal{RSMI_ERR_HOST};
    std::atomic<int> inject_host_fault{0};  // option "inject_host_fault", as the product's
};

namespace {
// batches coded at once: the CPU codec runs concurrent callers side by side on every core (the
// fair comparison for tools/bench_dagnode_cpu); the sanitizer builds use 4 lanes
int coal_lanes() {
#ifdef FAKE_RSMI_FAST
    return std::min(cpu_threads(), rsmi::GroupCommit<Req>::kMaxLanes);
#else
    return 4;
#endif
}
}  // namespace

namespace {

int encode_one(rsmi_ctx* c, const uint8_t* data, uint8_t* parity, size_t S) {
#ifdef FAKE_RSMI_FAST
    return rs_cpu_encode_batch(c->k, c->m, data, size_t(c->k) * S, parity, size_t(c->m) * S, S, 1, 1) ? RSMI_ERR_INVALID_ARG
                                                                                                      : RSMI_OK;
#endif
    std::vector<uint8_t> sh(size_t(c->n) * S);
    std::memcpy(sh.data(), data, size_t(c->k) * S);
    if (rs_oracle_encode(c->k, c->m, sh.data(), S)) return RSMI_ERR_INVALID_ARG;
    std::memcpy(parity, sh.data() + size_t(c->k) * S, size_t(c->m) * S);
    return RSMI_OK;
}

// rebuild the rows flagged in want (and missing) of one block of n rows at p
int reconstruct_one(rsmi_ctx* c, uint8_t* p, size_t S, const uint8_t* present, const uint8_t* want) {
#ifdef FAKE_RSMI_FAST
    // in place when the wanted rows are what ReconstructData / Reconstruct rebuild
    bool all = true, data = true;
    for (int i = 0; i < c->n; i++) {
        all &= bool(want[i]) == !present[i];
        data &= bool(want[i]) == (!present[i] && i < c->k);
    }
    if (all || data)
        return rs_cpu_reconstruct_batch(c->k, c->m, p, size_t(c->n) * S, S, 1, present, data ? 1 : 0, 1)
                   ? RSMI_ERR_TOO_FEW_SHARDS
                   : RSMI_OK;
#endif
    std::vector<uint8_t> sh(p, p + size_t(c->n) * S);
    if (rs_oracle_reconstruct(c->k, c->m, sh.data(), S, present, 0)) return RSMI_ERR_TOO_FEW_SHARDS;
    for (int i = 0; i < c->n; i++)
        if (!present[i] && want[i]) std::memcpy(p + size_t(i) * S, sh.data() + size_t(i) * S, S);
    return RSMI_OK;
}

void run_batch(rsmi_ctx* c, std::vector<Req*>& batch) {
    // test hook (option "inject_host_fault"): this batch fails as a host allocation would
    for (int v = c->inject_host_fault.load(); v > 0;)
        if (c->inject_host_fault.compare_exchange_weak(v, v - 1)) throw std::bad_alloc();
    for (Req* r : batch) {
        if (r->encode) {
            const size_t S = r->S, k = size_t(c->k), n = size_t(c->n);
            if (r->block != r->out) std::memcpy(r->out, r->block, r->B);  // block == out: Split by the caller
            std::memset(r->out + r->B, 0, n * S - r->B);
            r->rc = encode_one(c, r->out, r->out + k * S, S);
            for (size_t i = 0; i < n && r->rc == RSMI_OK; i++) {
                if (r->raw16) r->raw16[i] = r16(r->out + i * S, S);
                if (r->raw32) r->raw32[i] = r32(r->out + i * S, S);
            }
        } else {
            std::vector<uint8_t> want(size_t(c->n));
            for (int i = 0; i < c->n; i++) want[size_t(i)] = !r->present[i] && (i < c->k || !r->data_only);
            r->rc = reconstruct_one(c, r->out, r->S, r->present, want.data());
        }
    }
}

}  // namespace

extern "C" {

int rsmi_open(int k, int m, int device, rsmi_ctx** out) {
    (void)device;
    if (!out) return RSMI_ERR_INVALID_ARG;
    *out = nullptr;
    if (k <= 0 || m <= 0) return RSMI_ERR_INV_SHARD_NUM;
    if (k + m > 256) return RSMI_ERR_MAX_SHARD_NUM;
    auto* c = new rsmi_ctx();
    c->k = k;
    c->m = m;
    c->n = k + m;
    *out = c;
    return RSMI_OK;
}

void rsmi_close(rsmi_ctx* c) { delete c; }
int rsmi_warm(rsmi_ctx* c) { return c ? RSMI_OK : RSMI_ERR_INVALID_ARG; }

void* rsmi_host_alloc(size_t bytes) { return std::malloc(bytes ? bytes : 1); }
void rsmi_host_free(void* p) { std::free(p); }

int rsmi_encode_batch_host_crcs(rsmi_ctx* c, const uint8_t* data, size_t dbs, uint8_t* parity, size_t pbs, size_t S,
                                size_t nblocks, uint32_t* raw16, uint32_t* raw32) {
    if (!c || !data || !parity) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    for (int v = c->inject_host_fault.load(); v > 0;)  // as the product's direct host encodes
        if (c->inject_host_fault.compare_exchange_weak(v, v - 1)) return RSMI_ERR_HOST;
    const size_t k = size_t(c->k), m = size_t(c->m), n = k + m;
    (void)m;
    if (nblocks == 1) rsmi::run_pending_wait_hook();  // as the product's one-block call, before the coding
    return par_blocks(nblocks, [&](size_t b0, size_t b1) {
        for (size_t b = b0; b < b1; b++) {
            const int rc = encode_one(c, data + b * dbs, parity + b * pbs, S);
            if (rc) return rc;
            for (size_t i = 0; i < n; i++) {
                const uint8_t* row = i < k ? data + b * dbs + i * S : parity + b * pbs + (i - k) * S;
                if (raw16) raw16[b * n + i] = r16(row, S);
                if (raw32) raw32[b * n + i] = r32(row, S);
            }
        }
        return int(RSMI_OK);
    });
}

int rsmi_encode_batch_host(rsmi_ctx* c, const uint8_t* data, size_t dbs, uint8_t* parity, size_t pbs, size_t S,
                           size_t nblocks) {
    return rsmi_encode_batch_host_crcs(c, data, dbs, parity, pbs, S, nblocks, nullptr, nullptr);
}

int rsmi_reconstruct_rows_batch_host_crcs(rsmi_ctx* c, uint8_t* shards, size_t bs, size_t S, size_t nblocks,
                                          const uint8_t* present, const uint8_t* required, uint32_t* raw16,
                                          uint32_t* raw32) {
    if (!c || !shards || !present || !required) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    const size_t n = size_t(c->n);
    if (nblocks == 1) rsmi::run_pending_wait_hook();  // as the product's one-block call, before the coding
    return par_blocks(nblocks, [&](size_t b0, size_t b1) {
        for (size_t b = b0; b < b1; b++) {
            const int rc = reconstruct_one(c, shards + b * bs, S, present, required);
            if (rc) return rc;
            for (size_t i = 0; i < n; i++) {
                const bool rebuilt = !present[i] && required[i];
                if (raw16) raw16[b * n + i] = rebuilt ? r16(shards + b * bs + i * S, S) : 0;
                if (raw32) raw32[b * n + i] = rebuilt ? r32(shards + b * bs + i * S, S) : 0;
            }
        }
        return int(RSMI_OK);
    });
}

int rsmi_reconstruct_rows_batch_host(rsmi_ctx* c, uint8_t* shards, size_t bs, size_t S, size_t nblocks,
                                     const uint8_t* present, const uint8_t* required) {
    return rsmi_reconstruct_rows_batch_host_crcs(c, shards, bs, S, nblocks, present, required, nullptr, nullptr);
}

int rsmi_reconstruct_batch_host(rsmi_ctx* c, uint8_t* shards, size_t bs, size_t S, size_t nblocks,
                                const uint8_t* present, int data_only) {
    if (!c || !present) return RSMI_ERR_INVALID_ARG;
    std::vector<uint8_t> want(size_t(c->n));
    for (int i = 0; i < c->n; i++) want[size_t(i)] = !present[i] && (i < c->k || !data_only);
    return rsmi_reconstruct_rows_batch_host(c, shards, bs, S, nblocks, present, want.data());
}

int rsmi_reconstruct_batch_host_verify(rsmi_ctx* c, uint8_t* shards, size_t bs, size_t S, size_t nblocks,
                                       const uint8_t* present, int data_only, uint32_t* raw16_in) {
    if (!c || !shards || !present || !raw16_in) return RSMI_ERR_INVALID_ARG;
    std::vector<int> used;
    for (int i = 0; i < c->n && int(used.size()) < c->k; i++)
        if (present[i]) used.push_back(i);
    if (int(used.size()) < c->k) return RSMI_ERR_TOO_FEW_SHARDS;
    for (size_t b = 0; b < nblocks; b++)
        for (size_t j = 0; j < used.size(); j++)
            raw16_in[b * used.size() + j] = r16(shards + b * bs + size_t(used[j]) * S, S);
    return rsmi_reconstruct_batch_host(c, shards, bs, S, nblocks, present, data_only);
}

int rsmi_crc_rows_host(rsmi_ctx* c, const uint8_t* rows, size_t row_stride, size_t nrows, size_t S,
                       uint32_t* raw16, uint32_t* raw32) {
    if (!c || !rows || (!raw16 && !raw32)) return RSMI_ERR_INVALID_ARG;
    for (size_t r = 0; r < nrows; r++) {
        if (raw16) raw16[r] = r16(rows + r * row_stride, S);
        if (raw32) raw32[r] = r32(rows + r * row_stride, S);
    }
    return RSMI_OK;
}

int rsmi_encode_block_coalesced_crcs(rsmi_ctx* c, const uint8_t* block, size_t B, uint8_t* shards_out,
                                     uint32_t* raw16, uint32_t* raw32) {
    if (!c) return RSMI_ERR_INVALID_ARG;
    if (B == 0) return RSMI_ERR_SHORT_DATA;
    if (!block || !shards_out) return RSMI_ERR_INVALID_ARG;
    Req req{true, block, B, shards_out, rsmi_shard_size(B, c->k), nullptr, 0, raw16, raw32, RSMI_OK, false};
    const rsmi::WaitHook h = rsmi::take_wait_hook();  // the caller's idle task, as the product's
    c->coal.submit(req, 256, 0, coal_lanes(), [c](std::vector<Req*>& batch, int) { run_batch(c, batch); }, 0, h.fn,
                   h.arg);
    return req.rc;
}

int rsmi_encode_block_coalesced(rsmi_ctx* c, const uint8_t* block, size_t B, uint8_t* shards_out, uint32_t* raw) {
    return rsmi_encode_block_coalesced_crcs(c, block, B, shards_out, raw, nullptr);
}

int rsmi_reconstruct_coalesced(rsmi_ctx* c, uint8_t* shards, size_t S, const uint8_t* present, int data_only) {
    if (!c || !shards || !present) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    int np = 0;
    bool any = false;
    for (int i = 0; i < c->n; i++) {
        np += present[i] ? 1 : 0;
        any |= !present[i] && (i < c->k || !data_only);
    }
    if (!any) return RSMI_OK;
    if (np < c->k) return RSMI_ERR_TOO_FEW_SHARDS;
    Req req{false, nullptr, 0, shards, S, present, data_only, nullptr, nullptr, RSMI_OK, false};
    const rsmi::WaitHook h = rsmi::take_wait_hook();
    c->coal.submit(req, 256, 0, coal_lanes(), [c](std::vector<Req*>& batch, int) { run_batch(c, batch); }, 0, h.fn,
                   h.arg);
    return req.rc;
}

int rsmi_set_option(rsmi_ctx* c, const char* key, long value) {
    if (!c || !key) return RSMI_ERR_INVALID_ARG;
    if (!std::strcmp(key, "inject_host_fault")) c->inject_host_fault.store(int(value));
    return RSMI_OK;  // the coding options have no meaning on the CPU codec
}

long rsmi_get_stat(const rsmi_ctx* c, const char* key) {
    if (!c || !key) return -1;
    if (!std::strcmp(key, "coalesced_calls")) return long(c->coal.calls());
    if (!std::strcmp(key, "coalesced_batches")) return long(c->coal.batches());
    return -1;
}

}  // extern "C"
