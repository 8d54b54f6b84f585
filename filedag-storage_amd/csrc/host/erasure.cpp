// erasure.cpp -- see erasure.hpp.
#include "erasure.hpp"

#include <emmintrin.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <memory>

#include <atomic>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <tuple>
#include <vector>

namespace rsmi {
namespace host {

void copy_streaming(uint8_t* dst, const uint8_t* src, size_t n) {
    size_t i = 0;
    while (i < n && (reinterpret_cast<uintptr_t>(dst + i) & 15)) {
        dst[i] = src[i];
        i++;
    }
    for (; i + 64 <= n; i += 64) {
        const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
        const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 16));
        const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 32));
        const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 48));
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), a);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 32), c);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 48), d);
    }
    for (; i < n; i++) dst[i] = src[i];
    _mm_sfence();  // the streaming stores are visible before the codec call reads them
}

void copy_to_staging(uint8_t* dst, const uint8_t* src, size_t n) {
    if (n >= (size_t(1) << 20)) copy_streaming(dst, src, n);
    else std::memcpy(dst, src, n);
}

Status rsmi_status(int rc) {
    switch (rc) {
        case RSMI_OK: return Status::Ok();
        case RSMI_ERR_SHORT_DATA: return Status::Error("not enough data to fill the number of requested shards");
        case RSMI_ERR_TOO_FEW_SHARDS: return Status::Error("too few shards given");
        case RSMI_ERR_SHARD_NO_DATA: return Status::Error("no shard data");
        case RSMI_ERR_SHARD_SIZE: return Status::Error("shard sizes do not match");
        case RSMI_ERR_INV_SHARD_NUM:
            return Status::Error("cannot create Encoder with less than one data shard or less than zero parity shards");
        case RSMI_ERR_MAX_SHARD_NUM: return Status::Error("cannot create Encoder with more than 256 data+parity shards");
        default: return Status::Error(std::string("rsmi: ") + rsmi_status_string(rc));
    }
}

int64_t ceil_frac(int64_t numerator, int64_t denominator) {
    if (denominator == 0) return 0;
    if (denominator < 0) {
        numerator = -numerator;
        denominator = -denominator;
    }
    int64_t c = numerator / denominator;
    if (numerator > 0 && numerator % denominator != 0) c++;
    return c;
}

uint8_t* PinnedBuf::reserve(size_t bytes) {
    if (bytes <= cap_ && p_) return p_;
    release();
    const size_t want = bytes ? bytes : 1;
    p_ = static_cast<uint8_t*>(rsmi_host_alloc(want));
    pinned_ = p_ != nullptr;
    if (!p_) p_ = new (std::nothrow) uint8_t[want];
    cap_ = p_ ? want : 0;
    return p_;
}

void PinnedBuf::release() {
    if (p_) {
        if (pinned_) rsmi_host_free(p_);
        else delete[] p_;
    }
    p_ = nullptr;
    cap_ = 0;
    pinned_ = false;
}

PinnedBuf& thread_staging() {
    static thread_local PinnedBuf buf;
    return buf;
}

// per-thread scratch for one block's (k+m)*S rows around a single-block encode or
// reconstruct: neither zero-filled (the call writes every byte it returns) nor allocated per
// call (a 364 KB vector per Put or Get was a fresh value-initialised allocation each time), and
// page-locked, so a lone coalesced call codes it in place on the GPU (rsmi_coalesce.cpp) instead
// of through the engine's staging and a copy back
namespace {
// scratch of ended threads, by the NUMA node it was placed on (the allocating thread's), freed
// at exit; a new thread takes one placed on its own node
std::mutex g_scratch_mu;
std::map<int, std::vector<std::unique_ptr<PinnedBuf>>> g_scratch_pool;
int current_node() {
    unsigned cpu = 0, node = 0;
    return syscall(SYS_getcpu, &cpu, &node, nullptr) == 0 ? int(node) : 0;
}
struct ScratchHolder {
    std::unique_ptr<PinnedBuf> buf;
    int node = 0;
    ~ScratchHolder() {
        if (!buf) return;
        std::lock_guard<std::mutex> g(g_scratch_mu);
        try {
            g_scratch_pool[node].push_back(std::move(buf));
        } catch (...) {  // no room in the pool: the buffer is simply freed
        }
    }
};
}  // namespace

uint8_t* block_scratch(size_t bytes) {
    static thread_local ScratchHolder h;
    if (!h.buf) {
        h.node = current_node();
        std::lock_guard<std::mutex> g(g_scratch_mu);
        auto& free = g_scratch_pool[h.node];
        // the largest free one: it most likely already fits
        auto best = free.end();
        for (auto it = free.begin(); it != free.end(); ++it)
            if (best == free.end() || (*it)->capacity() > (*best)->capacity()) best = it;
        if (best != free.end()) {
            h.buf = std::move(*best);
            free.erase(best);
        }
    }
    if (!h.buf) h.buf.reset(new (std::nothrow) PinnedBuf());
    return h.buf ? h.buf->reserve(bytes) : nullptr;
}

namespace {
std::mutex g_ctx_mu;
// (k, m, device, replica, lane); lives for the process
std::map<std::tuple<int, int, int, int, int>, rsmi_ctx*> g_ctx_cache;

rsmi_ctx* lane_context(int k, int m, int device, int replica, int lane, int* rc) {
    std::lock_guard<std::mutex> g(g_ctx_mu);
    auto key = std::make_tuple(k, m, device, replica, lane);
    auto it = g_ctx_cache.find(key);
    if (it != g_ctx_cache.end()) {
        *rc = RSMI_OK;
        return it->second;
    }
    rsmi_ctx* c = nullptr;
    *rc = rsmi_open(k, m, device, &c);
    if (*rc == RSMI_OK) g_ctx_cache[key] = c;
    return c;
}
}  // namespace

void release_shared_contexts() {
    std::lock_guard<std::mutex> g(g_ctx_mu);
    for (auto& e : g_ctx_cache) rsmi_close(e.second);
    g_ctx_cache.clear();
}

rsmi_ctx* shared_context(int k, int m, int device, int* rc, int replica) {
    return lane_context(k, m, device, replica, 0, rc);
}

rsmi_ctx* call_context(int k, int m, int device, int* rc, int replica) {
    static std::atomic<unsigned> next{0};
    thread_local const int lane = int(next.fetch_add(1) % unsigned(kCallLanes));
    return lane_context(k, m, device, replica, lane, rc);
}

void warm_contexts(int k, int m, int device, int replica) {
    for (int lane = 0; lane < kCallLanes; lane++) {
        int rc;
        rsmi_ctx* c = lane_context(k, m, device, replica, lane, &rc);
        if (c) (void)rsmi_warm(c);  // the context and each of its coalescing lanes
    }
}

long lane_stat(int k, int m, int device, const char* key, int replica) {
    long v = 0;
    for (int lane = 0; lane < kCallLanes; lane++) {
        int rc;
        rsmi_ctx* c = lane_context(k, m, device, replica, lane, &rc);
        if (c) v += rsmi_get_stat(c, key);
    }
    return v;
}

Status Erasure::New(int data_blocks, int parity_blocks, int64_t block_size, Erasure* out, int device, int replica) {
    if (data_blocks <= 0 || parity_blocks <= 0) return rsmi_status(RSMI_ERR_INV_SHARD_NUM);
    if (data_blocks + parity_blocks > 256) return rsmi_status(RSMI_ERR_MAX_SHARD_NUM);
    out->data_blocks_ = data_blocks;
    out->parity_blocks_ = parity_blocks;
    out->block_size_ = block_size;
    out->device_ = device;
    out->replica_ = replica;
    return Status::Ok();
}

Status Erasure::EncodeData(const Bytes& data, std::vector<Bytes>* shards) const {
    const int n = data_blocks_ + parity_blocks_;
    shards->assign(size_t(n), Bytes());
    if (data.empty()) return Status::Ok();  // erasure.go:52-54
    int rc;
    rsmi_ctx* c = call_context(data_blocks_, parity_blocks_, device_, &rc, replica_);
    if (!c) return rsmi_status(rc);
    const size_t S = rsmi_shard_size(data.size(), data_blocks_);
    uint8_t* flat = block_scratch(size_t(n) * S);
    if (!flat) return Status::Error("out of host memory");
    copy_to_staging(flat, data.data(), data.size());  // Split's copy, on this thread
    rc = rsmi_encode_block_coalesced(c, flat, data.size(), flat, nullptr);
    if (rc) return rsmi_status(rc);
    for (int i = 0; i < n; i++) (*shards)[i].assign(flat + i * S, flat + (i + 1) * S);
    return Status::Ok();
}

Status Erasure::EncodeDataWithCrc(const Bytes& data, std::vector<Bytes>* shards, std::vector<uint32_t>* raw) const {
    return EncodeDataWithCrcs(data, shards, raw, nullptr);
}

Status Erasure::EncodeDataFlat(const Bytes& data, uint8_t* flat, uint32_t* raw, uint32_t* raw32) const {
    if (data.empty()) return Status::Ok();  // erasure.go:52-54
    int rc;
    rsmi_ctx* c = call_context(data_blocks_, parity_blocks_, device_, &rc, replica_);
    if (!c) return rsmi_status(rc);
    // Split's copy on this thread (concurrent callers copy in parallel), then coded in place
    copy_to_staging(flat, data.data(), data.size());
    rc = raw ? rsmi_encode_block_coalesced_crcs(c, flat, data.size(), flat, raw, raw32)
             : rsmi_encode_block_coalesced(c, flat, data.size(), flat, nullptr);
    return rsmi_status(rc);
}

Status Erasure::EncodeSplitFlat(size_t B, uint8_t* flat, uint32_t* raw, uint32_t* raw32) const {
    if (B == 0) return Status::Ok();  // erasure.go:52-54
    int rc;
    rsmi_ctx* c = call_context(data_blocks_, parity_blocks_, device_, &rc, replica_);
    if (!c) return rsmi_status(rc);
    rc = raw ? rsmi_encode_block_coalesced_crcs(c, flat, B, flat, raw, raw32)
             : rsmi_encode_block_coalesced(c, flat, B, flat, nullptr);
    return rsmi_status(rc);
}

Status Erasure::EncodeDataWithCrcs(const Bytes& data, std::vector<Bytes>* shards, std::vector<uint32_t>* raw,
                                   std::vector<uint32_t>* raw32) const {
    const int n = data_blocks_ + parity_blocks_;
    shards->assign(size_t(n), Bytes());
    raw->clear();
    if (raw32) raw32->clear();
    if (data.empty()) return Status::Ok();  // erasure.go:52-54
    int rc;
    rsmi_ctx* c = call_context(data_blocks_, parity_blocks_, device_, &rc, replica_);
    if (!c) return rsmi_status(rc);
    const size_t S = rsmi_shard_size(data.size(), data_blocks_);
    uint8_t* flat = block_scratch(size_t(n) * S);
    if (!flat) return Status::Error("out of host memory");
    raw->assign(size_t(n), 0);
    if (raw32) raw32->assign(size_t(n), 0);
    copy_to_staging(flat, data.data(), data.size());  // Split's copy, on this thread
    rc = rsmi_encode_block_coalesced_crcs(c, flat, data.size(), flat, raw->data(),
                                          raw32 ? raw32->data() : nullptr);
    if (rc) return rsmi_status(rc);
    for (int i = 0; i < n; i++) (*shards)[i].assign(flat + i * S, flat + (i + 1) * S);
    return Status::Ok();
}

Status Erasure::reconstruct(std::vector<Bytes>& shards, bool data_only) const {
    const int n = data_blocks_ + parity_blocks_;
    if (int(shards.size()) != n) return rsmi_status(RSMI_ERR_TOO_FEW_SHARDS);
    std::vector<size_t> lens(static_cast<size_t>(n));
    std::vector<uint8_t> present(static_cast<size_t>(n));
    for (int i = 0; i < n; i++) {
        lens[i] = shards[i].size();
        present[i] = shards[i].empty() ? 0 : 1;
    }
    size_t S = 0;
    int rc = rsmi_check_shards(n, lens.data(), 1, &S);
    if (rc) return rsmi_status(rc);
    int np = 0, dp = 0;
    for (int i = 0; i < n; i++)
        if (present[i]) {
            np++;
            if (i < data_blocks_) dp++;
        }
    if (np == n || (data_only && dp == data_blocks_)) return Status::Ok();
    rsmi_ctx* c = call_context(data_blocks_, parity_blocks_, device_, &rc, replica_);
    if (!c) return rsmi_status(rc);
    // [][]byte -> one contiguous buffer for the C-ABI: the first k present rows, the only ones the
    // decode reads (upstream reconstruct(); missing and later rows: don't-care bytes)
    uint8_t* flat = block_scratch(size_t(n) * S);
    if (!flat) return Status::Error("out of host memory");
    // streaming stores once the k rows reach 1 MiB together (copy_to_staging's threshold is for
    // the bytes the GPU then reads, not for one row)
    const bool stream = size_t(data_blocks_) * S >= (size_t(1) << 20);
    for (int i = 0, used = 0; i < n && used < data_blocks_; i++)
        if (present[i]) {
            if (stream) copy_streaming(flat + size_t(i) * S, shards[i].data(), S);
            else std::memcpy(flat + size_t(i) * S, shards[i].data(), S);
            used++;
        }
    // coalesced: concurrent degraded Gets usually miss the same node's shard, so they batch
    rc = rsmi_reconstruct_coalesced(c, flat, S, present.data(), data_only ? 1 : 0);
    if (rc) return rsmi_status(rc);
    for (int i = 0; i < n; i++)
        if (!present[i] && (i < data_blocks_ || !data_only)) shards[i].assign(flat + size_t(i) * S, flat + size_t(i + 1) * S);
    return Status::Ok();
}

Status Erasure::DecodeDataBlocks(std::vector<Bytes>& shards) const {
    size_t is_zero = 0;
    for (auto& b : shards)
        if (b.empty()) {
            is_zero++;
            break;  // erasure.go:72-77: counts at most one
        }
    if (is_zero == 0 || is_zero == shards.size()) return Status::Ok();
    return reconstruct(shards, true);
}

Status Erasure::DecodeDataAndParityBlocks(std::vector<Bytes>& shards) const { return reconstruct(shards, false); }

}  // namespace host
}  // namespace rsmi
