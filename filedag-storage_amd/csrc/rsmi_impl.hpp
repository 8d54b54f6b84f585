// rsmi_impl.hpp -- internals shared by the C-ABI implementation files (include/rsmi.h):
//   rsmi_core.cpp      contexts, coding plans, kernel dispatch, options, device-resident calls
//   rsmi_host.cpp      host-memory calls: zero-copy single kernel, copy-engine pipeline
//   rsmi_crc.cpp       datanode CRC-16 on the GPU (separate pass and fused into the encode)
//   rsmi_coalesce.cpp  group commit of concurrent single-block calls
// No CPU compute path anywhere: every byte of parity, reconstructed data or CRC comes out of
// the HIP kernels in rs_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rsmi.h"
#include "crc16.hpp"
#include "crc32.hpp"
#include "gf256.hpp"
#include "wait_hook.hpp"
#include "group_commit.hpp"
#include "rs_plan.hpp"

namespace rsmi {
namespace impl {

inline size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// The status of the exception being handled at the C-ABI boundary (the entry points' function
// try blocks): a C++ exception must not unwind into C or cgo callers.
int exception_status() noexcept;


struct DevTile {
    RsPlanDev* dev = nullptr;
    int K = 0, MT = 0;
};

struct Plan {
    std::vector<DevTile> tiles;
    int device = -1;
    ~Plan() {
        if (device >= 0) {
            (void)hipSetDevice(device);
            for (auto& t : tiles)
                if (t.dev) (void)hipFree(t.dev);
        }
    }
};

struct Staging {
    hipStream_t stream = nullptr;
    uint8_t* d_in = nullptr;
    uint8_t* d_out = nullptr;
    uint8_t* d_lin = nullptr;  // linear (pitch S) landing buffer for odd S
    size_t in_cap = 0, out_cap = 0, lin_cap = 0;
};

// Launch every tile of a plan over nblocks blocks.
// Fused CRC-16 output of an encode launch (rs_fast_kernel CRC variants): per-tile quad records
// of every shard and, for unaligned-window layouts, the rows' last chunks (rs_kernels.hip).
struct CrcFuse {
    const uint32_t* tbl = nullptr;
    uint32_t* rec = nullptr;
    uint32_t* tail = nullptr;
};

}  // namespace impl
}  // namespace rsmi

// Device scratch of the fused encode + CRC-16 (records of the tiles or units, and the inline
// combine's per-block unit counters), one per stream its launches go to, so concurrent calls on
// different streams never share records or counters.  Every caller stream of the
// device-resident calls gets its own.  The context's own streams share one, and only staging[0]
// ever launches a fused (or flagged) kernel (asserted in crc_scratch and arm_flag): host calls
// hold the context lock through their synchronisation, and a pipelined coalesced batch that is
// still in flight after the lock is released (rsmi_coalesce.cpp) is ordered before the next
// launch by staging[0]'s stream order.  The same holds for the page-locked R(shard)
// areas (raw_area, pipe_area): written by staging[0]'s kernels only.
struct CrcScratch {
    uint8_t* d_chunks = nullptr;  // tile records and tails (CrcFuse) or unit records
    size_t chunks_cap = 0;
    uint32_t* d_fctr = nullptr;  // per-block unit counters of the inline combine
    size_t fctr_cap = 0;
};

// defaults of options "coalesce_lanes" / "coalesce_carry" (build macros for A/B library variants)
#ifndef RSMI_COALESCE_LANES
#define RSMI_COALESCE_LANES 2
#endif
#ifndef RSMI_COALESCE_CARRY
#define RSMI_COALESCE_CARRY 1
#endif
// default of option "coalesce_flag" (rsmi_coalesce.cpp)
#ifndef RSMI_COALESCE_FLAG
#define RSMI_COALESCE_FLAG 1
#endif
// default of option "coalesce_pipeline" (rsmi_coalesce.cpp)
#ifndef RSMI_COALESCE_PIPELINE
#define RSMI_COALESCE_PIPELINE 1
#endif
// the fewest blocks a coalesced group codes through the table kernels (R(shard) straight into
// page-locked memory, no read-back dispatch): 1, a lone caller too (build macro for A/B variants;
// 2 before profiles/r05/r/)
#ifndef RSMI_TABLE_MIN_BLOCKS
#define RSMI_TABLE_MIN_BLOCKS 1
#endif

struct rsmi_ctx {
    int k = 0, m = 0, n = 0, device = 0;
    rsmi::Matrix M;  // n x k
    std::mutex mu;
    std::atomic<bool> dev_ready_flag{false};  // dev_ready, readable without mu (coalesce)
    bool dev_ready = false;
    int dev_status = RSMI_OK;
    int num_cu = 256;
    std::map<std::string, std::shared_ptr<rsmi::impl::Plan>> plans;
    std::vector<rsmi::impl::Staging> staging;  // [0] single-block calls, [0..2] batch pipeline
    uint8_t* h_stage = nullptr;    // pinned landing area for rebuilt rows (odd S)
    size_t h_stage_cap = 0;
    uint32_t* d_crc_tbl = nullptr;  // CRC-16 device tables (crc16.hpp), uploaded on first use
    uint8_t* d_crc = nullptr;       // raw row CRCs (u32) of host batch calls
    size_t crc_cap = 0;
    uint32_t* d_crc32_tbl = nullptr;  // CRC-32 device tables (crc32.hpp), uploaded on first use
    uint8_t* d_crc32 = nullptr;       // raw row CRC-32s of host batch calls
    size_t crc32_cap = 0;
    rsmi::Crc32Shift crc32_shift{};  // launch_crc32's per-S shift matrix, for crc32_shift_S
    uint64_t crc32_shift_S = ~uint64_t(0);
    CrcScratch own_scratch;  // the fused encode + CRC-16's scratch on the context's own streams
    std::map<hipStream_t, CrcScratch> stream_scratch;  // ... and on each caller stream (device-resident calls)
    // options
    int opt_crc16_fold = 1;     // aligned CRC-16 rows pass: 0 = nibble tables, 1 = matrix cores (fp4)
    int opt_crc32_fold = RSMI_CRC32_FOLD_DEFAULT;  // CRC-32 rows pass: 0 = nibble tables, 1 = matrix cores
    int opt_fused_fold = 1;     // aligned fused encode + CRC-16: 0 = nibble tables, 1 = matrix cores (fp4)
    long opt_waves_per_cu = 0;  // grid cap (0 = one tile per wave / the CRC passes' defaults)
    int opt_zero_copy = 1;  // results into page-locked host buffers by kernel stores
    long opt_small_bytes = 2L << 20;  // host calls up to this many shard bytes run zero-copy
    uint8_t* h_small = nullptr;       // page-locked staging of small calls (pageable callers)
    size_t h_small_cap = 0;
    uint8_t* h_raw = nullptr;  // page-locked landing area of row CRCs read back by kernel (readback)
    size_t h_raw_cap = 0;
    // pipelined coalesced batches (rsmi_coalesce.cpp): two page-locked landing areas of the table
    // launches' R(shard) and an event per area, so a lane's next batch launches while this one is
    // still coded
    uint8_t* h_pipe[2] = {nullptr, nullptr};
    size_t h_pipe_cap[2] = {0, 0};
    hipEvent_t pipe_ev[2] = {nullptr, nullptr};
    int pipe_slot = 0;
    int opt_coalesce_pipeline = RSMI_COALESCE_PIPELINE;
    // completion flags of table launches (BlockBases::done_flag): two page-locked flags (64 bytes
    // apart; slot = sequence number & 1, at most two launches of a context in flight) and their
    // device counters
    uint32_t* h_done = nullptr;
    uint32_t* h_done_dev = nullptr;
    uint32_t* d_done_ctr = nullptr;
    uint32_t done_seq = 0;
    int opt_coalesce_flag = RSMI_COALESCE_FLAG;
    // the coalescer's options are read by callers without ctx->mu (coalesce), so they are atomic
    std::atomic<long> opt_coalesce_us{0};     // extra wait for more callers before a coalesced batch runs
    std::atomic<long> opt_coalesce_max{256};  // blocks per coalesced batch
    std::string last_kernel;  // diagnostics (rsmi_last_kernel), under lk_mu
    mutable std::mutex lk_mu;
    // group commit for rsmi_encode_block_coalesced (see there)
    struct CoalReq {
        // encode: block/B in, out = (k+m)*S shards, raw optional; reconstruct: out = n*S
        // shards in place, present / want flags (group key covers S, pattern, want)
        const uint8_t* block;
        size_t B;
        uint8_t* out;
        uint32_t* raw;
        uint32_t* raw32;  // encode: optional CRC-32 R32(shard) per shard
        std::string key;
        int rc;
        bool done;
    };
    // a batch that throws (std::bad_alloc from the executor's host containers) fails its
    // requests as the boundary reports host-resource exceptions (include/rsmi.h ABI v3)
    rsmi::GroupCommit<CoalReq> coal{RSMI_ERR_HOST};
    std::atomic<int> opt_inject_host_fault{0};  // test hook: the next coalesced batches or direct host encodes throw std::bad_alloc
    std::atomic<int> opt_inject_lane_fault{0};  // test hook: the next lane contexts fail to open (RSMI_ERR_DEVICE)
    uint8_t* h_coal = nullptr;  // page-locked staging of the executing batch
    size_t h_coal_cap = 0;
    // Coalesced batches run on up to opt_coalesce_lanes lanes at once: lane 0 is this context, lane
    // i > 0 the child context lanes[i - 1] (same k, m, device and options; opened on first use), so
    // one batch can be coded while the next is launched and the callers' queue stays one queue
    std::atomic<long> opt_coalesce_lanes{RSMI_COALESCE_LANES};
    std::atomic<long> opt_coalesce_carry{RSMI_COALESCE_CARRY};  // batches a lane runs after its own before handing over (group_commit.hpp)
    std::vector<rsmi_ctx*> lanes;
    std::mutex lanes_mu;
};

namespace rsmi {
namespace impl {

#define HIP_TRY(expr)                                   \
    do {                                                \
        hipError_t _e = (expr);                         \
        if (_e != hipSuccess) return hip_status(_e);    \
    } while (0)

int hip_status(hipError_t e);
hipError_t pinned_alloc(void** p, size_t bytes);
int ensure_device(rsmi_ctx* c);
int make_plan(rsmi_ctx* c, const Matrix& coef, const std::vector<int>& in_rows, const std::vector<int>& out_rows,
              std::shared_ptr<Plan>& out);
int encode_plan(rsmi_ctx* c, std::shared_ptr<Plan>& out);
int decode_rows(const rsmi_ctx* c, const uint8_t* present, Matrix& dec, std::vector<int>& used);
int reconstruct_plan(rsmi_ctx* c, const uint8_t* present, const uint8_t* want, std::shared_ptr<Plan>& out);
std::vector<uint8_t> want_mask(const rsmi_ctx* c, const uint8_t* present, int data_only);
const char* kernel_label(int K, int MT, int NT, bool fast);
int auto_cache_policy(int K, int MT);
// tb: a table of block bases, in / out then being offsets from each (at most kTableBlocks blocks,
// the table kernels only: RSMI_ERR_INVALID_ARG when the shape has none, callers then launch per block)
int launch_plan(rsmi_ctx* c, const Plan& plan, const uint8_t* in, uint64_t in_rs, uint64_t in_bs, uint8_t* out,
                uint64_t out_rs, uint64_t out_bs, uint64_t S, uint64_t nblocks, hipStream_t stream,
                const CrcFuse* fuse = nullptr, const BlockBases* tb = nullptr, bool* armed = nullptr);
uintptr_t table_alignment(const BlockBases* tb, uint64_t nblocks);  // OR of the table's first nblocks bases
void set_last_kernel(rsmi_ctx* c, const std::string& label);
CrcScratch& crc_scratch(rsmi_ctx* c, hipStream_t st);  // caller holds ctx->mu
// reserve() for device scratch a stream's kernels may still be reading: that stream is
// synchronised before the old buffer is freed
int reserve_on(uint8_t*& p, size_t& cap, size_t need, hipStream_t st);
int reserve(uint8_t*& p, size_t& cap, size_t need);
int count_present(const rsmi_ctx* c, const uint8_t* present, int& np, int& dp);
int reconstruct_precheck(const rsmi_ctx* c, const uint8_t* present, const uint8_t* want);
int reconstruct_dev_impl(rsmi_ctx* c, uint8_t* d_shards, size_t shard_stride, size_t block_stride, size_t S,
                                size_t nblocks, const uint8_t* present, const uint8_t* want, void* stream);
bool dma_2d_ok(size_t S);
int repitch(uint8_t* dst, size_t dpitch, const uint8_t* src, size_t spitch, size_t width, size_t rows,
            hipStream_t stream);
uint8_t* host_alias(void* p, size_t len);
uint8_t* small_stage(rsmi_ctx* c, size_t need);
uint8_t* raw_area(rsmi_ctx* c, size_t bytes);
int readback(rsmi_ctx* c, const uint32_t* d16, const uint32_t* d32, size_t sz, hipStream_t st, const uint32_t*& h16,
             const uint32_t*& h32);
int encode_small(rsmi_ctx* c, const Plan& plan, const uint8_t* data, size_t dbs, uint8_t* parity, size_t pbs,
                        size_t S, size_t nblocks, uint32_t* raw_out, uint32_t* raw32_out = nullptr);
int encode_host_impl(rsmi_ctx* c, const uint8_t* data, size_t data_block_stride, uint8_t* parity,
                            size_t parity_block_stride, size_t S, size_t nblocks, uint32_t* raw_out, uint32_t* raw32_out = nullptr);
int reconstruct_small(rsmi_ctx* c, const Plan& plan, uint8_t* shards, size_t bs, size_t S, size_t nblocks,
                             const uint8_t* present, const uint8_t* want, uint32_t* raw16 = nullptr,
                      uint32_t* raw32 = nullptr);
int reconstruct_host_impl(rsmi_ctx* c, uint8_t* shards, size_t block_stride, size_t S, size_t nblocks,
                                 const uint8_t* present, const uint8_t* want, uint32_t* raw16 = nullptr,
                          uint32_t* raw32 = nullptr);
int ensure_crc_tables(rsmi_ctx* c);
int ensure_crc32_tables(rsmi_ctx* c);
// R(row) / R32(row) of the rows the plan rebuilt (want && !present), one row per block at
// base + b*bstride + r*rpitch, into the device buffers d16 / d32 at [b*n + r] (either may be
// null; zeroed here), stream-ordered
int launch_rebuilt_crcs(rsmi_ctx* c, const uint8_t* base, uint64_t rpitch, uint64_t bstride, uint64_t S,
                        uint64_t nblocks, const uint8_t* present, const uint8_t* want, uint32_t* d16, uint32_t* d32,
                        hipStream_t stream);
int launch_crc32(rsmi_ctx* c, const uint8_t* base, uint64_t rpitch, uint64_t bstride, uint32_t nrows, uint64_t S,
                 uint64_t nblocks, uint32_t* out, uint64_t out_bs, hipStream_t stream);
int launch_crc(rsmi_ctx* c, const uint8_t* base, uint64_t rpitch, uint64_t bstride, uint32_t nrows, uint64_t S,
               uint64_t nblocks, uint32_t* out, uint64_t out_bs, hipStream_t stream, bool zero = true);
int launch_encode_crc(rsmi_ctx* c, const Plan& plan, const uint8_t* in, size_t in_rs, size_t in_bs, uint8_t* out,
                             size_t out_rs, size_t out_bs, size_t S, size_t nblocks, uint32_t* raw, hipStream_t st);
int launch_plan_crc(rsmi_ctx* c, const Plan& plan, const uint8_t* in, size_t in_rs, size_t in_bs, uint8_t* out,
                    size_t out_rs, size_t out_bs, size_t S, size_t nblocks, uint32_t* raw, hipStream_t st,
                    const BlockBases* tb = nullptr, bool* armed = nullptr);
int launch_encode_rows(rsmi_ctx* c, const Plan& plan, const uint8_t* in, size_t in_bs, uint8_t* out, size_t out_bs,
                       size_t S, size_t nblocks, uint32_t* d16, uint32_t* d32, hipStream_t st);
uint8_t* coal_stage(rsmi_ctx* c, size_t need);
// completion flags of table launches (rsmi_coalesce.cpp): arm one in tb (caller holds ctx->mu),
// its host view, and the poll that replaces the stream (or event) synchronisation
int arm_flag(rsmi_ctx* c, hipStream_t st, BlockBases& tb, uint32_t& seq);
const uint32_t* done_flag(const rsmi_ctx* c, uint32_t seq);
int wait_flag(const uint32_t* flag, uint32_t seq, hipStream_t st, hipEvent_t ev);
int run_coalesced_in_place(rsmi_ctx* c, rsmi_ctx::CoalReq* const* rq, size_t nb, size_t S, std::function<void()>* fin);
void run_coalesced_group(rsmi_ctx* c, rsmi_ctx::CoalReq* const* rq, size_t nb, std::function<void()>* fin);
std::function<void()> run_coalesced(rsmi_ctx* c, int lane, std::vector<rsmi_ctx::CoalReq*>& batch);
int coalesce(rsmi_ctx* c, rsmi_ctx::CoalReq& req);
int ensure_device_fast(rsmi_ctx* c);
rsmi_ctx* lane_context(rsmi_ctx* c, int lane, int* rc);  // coalescing lane `lane`'s context (0: c)  // ensure_device without the context lock once the device is bound
int apply_option(rsmi_ctx* c, const char* key, long value);  // caller holds ctx->mu

}  // namespace impl
}  // namespace rsmi
