// rsmi_core.cpp -- contexts, coding plans, kernel dispatch, options and the device-resident
// entry points of include/rsmi.h (see rsmi_impl.hpp for the file map).
#include "rsmi_impl.hpp"

#include <cassert>

#include <limits>

using namespace rsmi;
using namespace rsmi::impl;

namespace rsmi {
namespace impl {

// Page-locked host memory for the caller (rsmi_host_alloc) and for every context's staging:
// portable (mapped for every device, so a device group's members read and write one caller
// buffer in place) and placed by the calling thread's NUMA policy (hipHostMallocNumaUser): a
// device group's member threads run bound to their GPU's NUMA node (rsmi_group.cpp), so their
// staging lands in that socket's memory; other threads get the default local placement.
hipError_t pinned_alloc(void** p, size_t bytes) {
    *p = nullptr;
    hipError_t e = hipHostMalloc(p, bytes, hipHostMallocPortable | hipHostMallocNumaUser);
    if (e != hipSuccess) {  // a runtime without NUMA-user placement: portable only
        (void)hipGetLastError();
        e = hipHostMalloc(p, bytes, hipHostMallocPortable);
    }
    return e;
}

int hip_status(hipError_t e) {
    if (e == hipSuccess) return RSMI_OK;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice || e == hipErrorNoBinaryForGpu ||
        e == hipErrorInsufficientDriver)
        return RSMI_ERR_NO_DEVICE;
    return RSMI_ERR_DEVICE;
}

// Lazily bind the context to its device (caller holds ctx->mu).
int ensure_device(rsmi_ctx* c) {
    if (c->dev_ready) return RSMI_OK;
    if (c->dev_status != RSMI_OK) return c->dev_status;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0 || c->device < 0 || c->device >= count) {
        c->dev_status = RSMI_ERR_NO_DEVICE;
        return c->dev_status;
    }
    HIP_TRY(hipSetDevice(c->device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, c->device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        c->dev_status = RSMI_ERR_NO_DEVICE;  // kernels are built for gfx950 only
        return c->dev_status;
    }
    c->num_cu = prop.multiProcessorCount;
    c->staging.resize(3);
    for (auto& s : c->staging) HIP_TRY(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    c->dev_ready = true;
    c->dev_ready_flag.store(true, std::memory_order_release);
    return RSMI_OK;
}

int ensure_device_fast(rsmi_ctx* c) {
    if (c->dev_ready_flag.load(std::memory_order_acquire)) return RSMI_OK;
    std::lock_guard<std::mutex> g(c->mu);
    return ensure_device(c);
}

void set_last_kernel(rsmi_ctx* c, const std::string& label) {
    std::lock_guard<std::mutex> g(c->lk_mu);
    c->last_kernel = label;
}

CrcScratch& crc_scratch(rsmi_ctx* c, hipStream_t st) {
    // own streams: only staging[0] launches fused or flagged kernels, so a pipelined coalesced
    // batch still in flight there (ctx->mu released) and the next launch share own_scratch in
    // stream order (rsmi_impl.hpp CrcScratch)
    for (size_t i = 0; i < c->staging.size(); i++)
        if (c->staging[i].stream == st) {
            assert(i == 0 && "fused CRC scratch used on a staging stream other than staging[0]");
            return c->own_scratch;
        }
    auto it = c->stream_scratch.find(st);
    if (it != c->stream_scratch.end()) return it->second;
    // a caller that cycles through many streams: past 32 of them the device is drained once and
    // every caller stream's scratch freed (a stream the caller has destroyed cannot be
    // synchronised by itself, the device can)
    if (c->stream_scratch.size() >= 32) {
        (void)hipDeviceSynchronize();
        for (auto& e : c->stream_scratch) {
            if (e.second.d_chunks) (void)hipFree(e.second.d_chunks);
            if (e.second.d_fctr) (void)hipFree(e.second.d_fctr);
        }
        c->stream_scratch.clear();
    }
    return c->stream_scratch[st];
}

int reserve_on(uint8_t*& p, size_t& cap, size_t need, hipStream_t st) {
    if (cap >= need) return RSMI_OK;
    if (p) HIP_TRY(hipStreamSynchronize(st));
    return reserve(p, cap, need);
}

// Build the device tiles for a coefficient matrix coef (rows x K) mapping input rows
// in_rows -> output rows out_rows.
int make_plan(rsmi_ctx* c, const Matrix& coef, const std::vector<int>& in_rows, const std::vector<int>& out_rows,
              std::shared_ptr<Plan>& out) {
    auto plan = std::make_shared<Plan>();
    plan->device = c->device;
    const int K = coef.cols;
    std::unique_ptr<RsPlanDev> h(new RsPlanDev());
    for (int j0 = 0; j0 < coef.rows; j0 += kMaxMT) {
        const int MT = std::min(kMaxMT, coef.rows - j0);
        std::memset(h.get(), 0, sizeof(RsPlanDev));
        h->k = uint32_t(K);
        h->mt = uint32_t(MT);
        for (int i = 0; i < K; i++) h->in_row[i] = uint32_t(in_rows[i]);
        for (int j = 0; j < MT; j++) h->out_row[j] = uint32_t(out_rows[j0 + j]);
        for (int col = 0; col < K; col++)
            for (int j = 0; j < MT; j++) {
                uint32_t w[5];
                perm_tables(coef.at(j0 + j, col), w);
                for (int f = 0; f < 5; f++) h->tbl[col * kColDwords + f * 4 + j] = w[f];
            }
        DevTile t;
        t.K = K;
        t.MT = MT;
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&t.dev), sizeof(RsPlanDev)));
        plan->tiles.push_back(t);
        HIP_TRY(hipMemcpy(t.dev, h.get(), sizeof(RsPlanDev), hipMemcpyHostToDevice));
    }
    out = plan;
    return RSMI_OK;
}

int encode_plan(rsmi_ctx* c, std::shared_ptr<Plan>& out) {
    auto it = c->plans.find("E");
    if (it != c->plans.end()) {
        out = it->second;
        return RSMI_OK;
    }
    Matrix par(c->m, c->k);
    std::memcpy(par.v.data(), c->M.row(c->k), size_t(c->m) * c->k);
    std::vector<int> in_rows(c->k), out_rows(c->m);
    for (int i = 0; i < c->k; i++) in_rows[i] = i;
    for (int j = 0; j < c->m; j++) out_rows[j] = j;
    int rc = make_plan(c, par, in_rows, out_rows, out);
    if (rc == RSMI_OK) c->plans["E"] = out;
    return rc;
}

// Upstream reconstruct(): survivors = first k present rows; data decode rows are the
// inverse of their sub-matrix; missing parity rows are expressed directly over the
// survivors as M[i] x inverse (exact over GF(2^8), so one pass writes every missing row).
int decode_rows(const rsmi_ctx* c, const uint8_t* present, Matrix& dec, std::vector<int>& used) {
    used.clear();
    Matrix sub(c->k, c->k);
    for (int i = 0; i < c->n && int(used.size()) < c->k; i++) {
        if (!present[i]) continue;
        std::memcpy(&sub.at(int(used.size()), 0), c->M.row(i), size_t(c->k));
        used.push_back(i);
    }
    if (int(used.size()) < c->k) return RSMI_ERR_TOO_FEW_SHARDS;
    if (!mat_invert(sub, dec)) return RSMI_ERR_SINGULAR;
    return RSMI_OK;
}

// want[i]: rebuild row i (only rows that are missing are ever written)
int reconstruct_plan(rsmi_ctx* c, const uint8_t* present, const uint8_t* want, std::shared_ptr<Plan>& out) {
    std::string key = "R";
    for (int i = 0; i < c->n; i++) key.push_back(char('0' + (present[i] ? 1 : 0) + (want[i] ? 2 : 0)));
    auto it = c->plans.find(key);
    if (it != c->plans.end()) {
        out = it->second;
        return RSMI_OK;
    }
    Matrix dec;
    std::vector<int> used;
    int rc = decode_rows(c, present, dec, used);
    if (rc) return rc;
    std::vector<int> out_rows;
    std::vector<uint8_t> rows;
    for (int i = 0; i < c->k; i++)
        if (!present[i] && want[i]) {
            out_rows.push_back(i);
            rows.insert(rows.end(), dec.row(i), dec.row(i) + c->k);
        }
    for (int i = c->k; i < c->n; i++)
        if (!present[i] && want[i]) {
            Matrix r(1, c->k);
            std::memcpy(r.v.data(), c->M.row(i), size_t(c->k));
            Matrix p = mat_mul(r, dec);
            out_rows.push_back(i);
            rows.insert(rows.end(), p.v.begin(), p.v.end());
        }
    Matrix coef(int(out_rows.size()), c->k);
    std::memcpy(coef.v.data(), rows.data(), rows.size());
    rc = make_plan(c, coef, used, out_rows, out);
    if (rc == RSMI_OK) c->plans[key] = out;
    return rc;
}

// want mask of upstream ReconstructData (missing data rows) / Reconstruct (all missing)
std::vector<uint8_t> want_mask(const rsmi_ctx* c, const uint8_t* present, int data_only) {
    std::vector<uint8_t> w(size_t(c->n), 0);
    for (int i = 0; i < c->n; i++) w[i] = !present[i] && (i < c->k || !data_only);
    return w;
}

const char* kernel_label(int K, int MT, int NT, bool fast) {
    static thread_local char buf[96];
    if (fast)
        std::snprintf(buf, sizeof buf, "rs_fast_kernel<K=%d,MT=%d,NT=%d>", K, MT, NT);
    else
        std::snprintf(buf, sizeof buf, "rs_generic_kernel<K=%d,MT=%d>", K, MT);
    return buf;
}

// Cache policy per tile shape (tools/ntsweep.py, profiles/r01/ntsweep.txt): nontemporal
// loads are +5-15 % on every shape; nontemporal stores win while a tile writes a large
// share of its traffic (RS(10,4) encode +9 %, RS(4,2) encode +10 %, RS(2,1) +6 %) and lose
// once the tile reads at least 4 rows per row written (RS(10,4) 1-row reconstruct -5 %,
// 2-row -3 %, RS(16,4) 2-row -4 %, RS(4,2) 1-row -5 %; RS(16,4) encode is a tie).
int auto_cache_policy(int K, int MT) { return K >= 4 * MT ? 2 : 1; }

uintptr_t table_alignment(const BlockBases* tb, uint64_t nblocks) {
    uintptr_t a = 0;
    for (uint64_t b = 0; tb && b < nblocks; b++) a |= uintptr_t(tb->b[b]);
    return a;
}

int launch_plan(rsmi_ctx* c, const Plan& plan, const uint8_t* in, uint64_t in_rs, uint64_t in_bs, uint8_t* out,
                uint64_t out_rs, uint64_t out_bs, uint64_t S, uint64_t nblocks, hipStream_t stream,
                const CrcFuse* fuse, const BlockBases* tb, bool* armed) {
    if (armed) *armed = false;
    if (nblocks == 0 || S == 0) return RSMI_OK;
    // tb: a table of block bases (in / out are offsets from each), one launch of at most
    // kTableBlocks blocks, table kernels only (callers fall back to a launch per block)
    if (tb && (nblocks > uint64_t(kTableBlocks) || fuse)) return RSMI_ERR_INVALID_ARG;
    const uintptr_t tba = table_alignment(tb, nblocks);
    const bool aligned = ((reinterpret_cast<uintptr_t>(in) | tba) % 16 == 0) &&
                         ((reinterpret_cast<uintptr_t>(out) | tba) % 16 == 0) && in_rs % 16 == 0 && in_bs % 16 == 0 &&
                         out_rs % 16 == 0 && out_bs % 16 == 0 && in_rs >= round_up(S, 16) && out_rs >= round_up(S, 16) &&
                         S < (uint64_t(1) << 31);
    // any other layout with rows of at least 16 bytes: the unaligned-window variant (D = 1)
    const bool ua = !aligned && S >= 16 && S < (uint64_t(1) << 31) && in_rs >= S && out_rs >= S;
    if (fuse && ((!aligned && !ua) || plan.tiles.size() != 1)) return RSMI_ERR_INVALID_ARG;  // callers fall back
                                                                                              // to the separate pass
    if (tb)
        for (const DevTile& t : plan.tiles)
            if (t.K > 16 || !(aligned ? fast_kernels().fn_tb : fast_kernels().ua_tb)[t.K][t.MT] || (!aligned && !ua))
                return RSMI_ERR_INVALID_ARG;
    for (const DevTile& t : plan.tiles) {
        const int NT = auto_cache_policy(t.K, t.MT);
        void* fn = nullptr;
        if (t.K <= 16) {
            if (tb) fn = aligned ? fast_kernels().fn_tb[t.K][t.MT] : fast_kernels().ua_tb[t.K][t.MT];
            else if (fuse) fn = ua ? fast_kernels().ua_crc[t.K][t.MT] : fast_kernels().crc[t.K][t.MT];
            else if (aligned) fn = fast_kernels().fn[t.K][t.MT];
            else if (ua) fn = fast_kernels().ua[t.K][t.MT];
        }
        if (fuse && !fn) return RSMI_ERR_INVALID_ARG;
        if (fn) {
            const uint64_t cpb = (S + 15) / 16;
            const uint64_t tpb = (cpb + uint64_t(kWave) - 1) / uint64_t(kWave);
            constexpr int wpg = kFastWG / kWave;
            // One tile per wave: the hardware dispatcher hands each free slot the next workgroup,
            // which balances the launch across CUs and XCDs of uneven effective bandwidth.  A
            // persistent grid (occupancy x CUs, each wave striding over ~26 tiles) gives every CU
            // the same share and waits for the slowest: measured 9-28 % slower on every BASELINE
            // shape.  waves_per_cu > 0 caps the grid (the loop in the kernels
            // strides over the remaining tiles).
            long wg_cap = std::numeric_limits<long>::max();
            if (c->opt_waves_per_cu > 0) wg_cap = std::max(1L, long(c->num_cu) * c->opt_waves_per_cu / wpg);
            // split into launches whose tile count fits 32 bits
            const uint64_t max_blocks = std::max<uint64_t>(1, (uint64_t(1) << 31) / tpb);
            for (uint64_t b0 = 0; b0 < nblocks; b0 += max_blocks) {
                const uint64_t nb = std::min(max_blocks, nblocks - b0);
                uint32_t ntiles = uint32_t(nb * tpb);
                uint32_t S32 = uint32_t(S), cpb32 = uint32_t(cpb), tpb32 = uint32_t(tpb);
                const RsPlanDev* pd = t.dev;
                const uint8_t* inb = in + b0 * in_bs;
                uint8_t* outb = out + b0 * out_bs;
                const uint32_t* ctbl = fuse ? fuse->tbl : nullptr;
                const uint64_t rec_per_block = tpb * uint64_t((((t.K + t.MT) + 3) / 4 + 1) / 2) * kWave;
                uint32_t* crec = fuse ? fuse->rec + b0 * rec_per_block : nullptr;
                uint32_t* ctail = fuse && fuse->tail ? fuse->tail + b0 * uint64_t(t.K + t.MT) : nullptr;
                NoBases nob;
                // a table's completion flag is armed only when this one launch is the whole job
                BlockBases tbl_args;
                if (tb) {
                    tbl_args = *tb;
                    if (plan.tiles.size() != 1 || nblocks > max_blocks) tbl_args.done_flag = nullptr;
                    if (armed) *armed = tbl_args.done_flag != nullptr;
                }
                void* bases = tb ? static_cast<void*>(&tbl_args) : static_cast<void*>(&nob);
                void* args[] = {&pd,    &inb,   &outb,   &in_bs, &in_rs, &out_bs, &out_rs, &S32,
                                &cpb32, &tpb32, &ntiles, &ctbl,  &crec,  &ctail, bases};
                const uint64_t wgs = std::min<uint64_t>((ntiles + wpg - 1) / wpg, uint64_t(wg_cap));
                HIP_TRY(hipLaunchKernel(fn, dim3(uint32_t(wgs)), dim3(uint32_t(wpg * kWave)), args, 0, stream));
            }
            std::string label = kernel_label(t.K, t.MT, NT, true);
            if (ua) label += ",UA";
            if (fuse) label += ",CRC";
            if (tb) label += ",TB";
            set_last_kernel(c, label);
        } else {
            const uint64_t groups = (S + 3) / 4;
            const uint32_t gx = uint32_t(std::min<uint64_t>((groups + kWG - 1) / kWG, 4096));
            const uint32_t gy = uint32_t(std::min<uint64_t>(nblocks, 65535));
            const RsPlanDev* pd = t.dev;
            void* args[] = {&pd, &in, &out, &in_bs, &in_rs, &out_bs, &out_rs, &S, &nblocks};
            HIP_TRY(hipLaunchKernel(generic_kernel(), dim3(gx, gy), dim3(kWG), args, 0, stream));
            set_last_kernel(c, kernel_label(t.K, t.MT, 0, false));
        }
    }
    return hip_status(hipGetLastError());
}

int reserve(uint8_t*& p, size_t& cap, size_t need) {
    if (cap >= need) return RSMI_OK;
    const size_t sz = std::max(need, cap + cap / 2);
    if (p) HIP_TRY(hipFree(p));
    p = nullptr;
    cap = 0;
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&p), sz));
    cap = sz;
    return RSMI_OK;
}

int count_present(const rsmi_ctx* c, const uint8_t* present, int& np, int& dp) {
    np = dp = 0;
    for (int i = 0; i < c->n; i++)
        if (present[i]) {
            np++;
            if (i < c->k) dp++;
        }
    return RSMI_OK;
}

// quick-return / too-few checks shared by every reconstruct entry point (upstream
// reconstruct(): nothing requested missing -> no-op, then fewer than k present -> error).
// returns 1 when there is nothing to do, 0 when work is needed, or -error
int reconstruct_precheck(const rsmi_ctx* c, const uint8_t* present, const uint8_t* want) {
    int np, dp;
    count_present(c, present, np, dp);
    bool any = false;
    for (int i = 0; i < c->n; i++) any |= !present[i] && want[i];
    if (!any) return 1;
    if (np < c->k) return -RSMI_ERR_TOO_FEW_SHARDS;
    return 0;
}

int reconstruct_dev_impl(rsmi_ctx* c, uint8_t* d_shards, size_t shard_stride, size_t block_stride, size_t S,
                                size_t nblocks, const uint8_t* present, const uint8_t* want, void* stream) {
    if (!c || !d_shards || !present || !want) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    if (shard_stride < S) return RSMI_ERR_INVALID_ARG;
    int pre = reconstruct_precheck(c, present, want);
    if (pre < 0) return -pre;
    if (pre == 1) return RSMI_OK;
    std::shared_ptr<Plan> plan;
    std::lock_guard<std::mutex> g(c->mu);
    int rc = ensure_device(c);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    rc = reconstruct_plan(c, present, want, plan);
    if (rc) return rc;
    return launch_plan(c, *plan, d_shards, shard_stride, block_stride, d_shards, shard_stride, block_stride, S, nblocks,
                       static_cast<hipStream_t>(stream));
}

int exception_status() noexcept {
    // std::bad_alloc, std::system_error from a thread or mutex, or anything else a host-side
    // container throws: the call failed for want of host resources.  Unwinding released the
    // context's locks; the call's outputs are undefined, as after any failed call
    return RSMI_ERR_HOST;
}

}  // namespace impl
}  // namespace rsmi

extern "C" {

int rsmi_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int rsmi_open(int k, int m, int device, rsmi_ctx** out) try {
    if (!out) return RSMI_ERR_INVALID_ARG;
    *out = nullptr;
    if (k <= 0 || m <= 0) return RSMI_ERR_INV_SHARD_NUM;
    if (k + m > 256) return RSMI_ERR_MAX_SHARD_NUM;
    auto* c = new rsmi_ctx();
    c->k = k;
    c->m = m;
    c->n = k + m;
    c->device = device;
    c->M = build_encode_matrix(k, m);
    *out = c;
    return RSMI_OK;
} catch (...) {
    return rsmi::impl::exception_status();
}

void rsmi_close(rsmi_ctx* c) {
    if (!c) return;
    for (rsmi_ctx* l : c->lanes) rsmi_close(l);
    {
        std::lock_guard<std::mutex> g(c->mu);
        c->plans.clear();
        if (c->dev_ready) {
            (void)hipSetDevice(c->device);
            for (auto& s : c->staging) {
                if (s.stream) (void)hipStreamSynchronize(s.stream);
                if (s.d_in) (void)hipFree(s.d_in);
                if (s.d_out) (void)hipFree(s.d_out);
                if (s.d_lin) (void)hipFree(s.d_lin);
                if (s.stream) (void)hipStreamDestroy(s.stream);
            }
            if (c->h_stage) (void)hipHostFree(c->h_stage);
            if (c->h_coal) (void)hipHostFree(c->h_coal);
            if (c->h_small) (void)hipHostFree(c->h_small);
            if (c->h_raw) (void)hipHostFree(c->h_raw);
            if (c->h_done) (void)hipHostFree(c->h_done);
            if (c->d_done_ctr) (void)hipFree(c->d_done_ctr);
            for (int i = 0; i < 2; i++) {
                if (c->h_pipe[i]) (void)hipHostFree(c->h_pipe[i]);
                if (c->pipe_ev[i]) (void)hipEventDestroy(c->pipe_ev[i]);
            }
            if (c->d_crc_tbl) (void)hipFree(c->d_crc_tbl);
            if (c->d_crc) (void)hipFree(c->d_crc);
            auto free_scratch = [](CrcScratch& x) {
                if (x.d_chunks) (void)hipFree(x.d_chunks);
                if (x.d_fctr) (void)hipFree(x.d_fctr);
            };
            free_scratch(c->own_scratch);
            if (!c->stream_scratch.empty()) (void)hipDeviceSynchronize();  // caller streams may be gone
            for (auto& e : c->stream_scratch) free_scratch(e.second);
            if (c->d_crc32_tbl) (void)hipFree(c->d_crc32_tbl);
            if (c->d_crc32) (void)hipFree(c->d_crc32);
        }
    }
    delete c;
}

int rsmi_encode_matrix(const rsmi_ctx* c, uint8_t* out) try {
    if (!c || !out) return RSMI_ERR_INVALID_ARG;
    std::memcpy(out, c->M.v.data(), c->M.v.size());
    return RSMI_OK;
} catch (...) {
    return rsmi::impl::exception_status();
}

int rsmi_decode_matrix(const rsmi_ctx* c, const uint8_t* present, uint8_t* out, int* used_rows) try {
    if (!c || !present || !out) return RSMI_ERR_INVALID_ARG;
    Matrix dec;
    std::vector<int> used;
    int rc = decode_rows(c, present, dec, used);
    if (rc) return rc;
    std::memcpy(out, dec.v.data(), dec.v.size());
    if (used_rows)
        for (int i = 0; i < c->k; i++) used_rows[i] = used[i];
    return RSMI_OK;
} catch (...) {
    return rsmi::impl::exception_status();
}

int rsmi_set_option(rsmi_ctx* c, const char* key, long value) try {
    if (!c || !key) return RSMI_ERR_INVALID_ARG;
    int rc;
    {
        std::lock_guard<std::mutex> g(c->mu);
        if ((rc = apply_option(c, key, value))) return rc;
    }
    // the coalescer's lane contexts code with the same options (the test hook stays with the
    // context whose batches it fails).  A lane whose open failed (or that opened out of order)
    // leaves a null slot (lane_context): skip it.
    if (std::strcmp(key, "inject_host_fault") != 0 && std::strcmp(key, "inject_lane_fault") != 0) {
        std::lock_guard<std::mutex> g(c->lanes_mu);
        for (rsmi_ctx* l : c->lanes) {
            if (!l) continue;
            std::lock_guard<std::mutex> gl(l->mu);
            (void)apply_option(l, key, value);
        }
    }
    return RSMI_OK;
} catch (...) {
    return rsmi::impl::exception_status();
}

}  // extern "C"

namespace rsmi {
namespace impl {

int apply_option(rsmi_ctx* c, const char* key, long value) {
    if (!std::strcmp(key, "zero_copy")) {
        if (value < 0 || value > 2) return RSMI_ERR_INVALID_ARG;
        c->opt_zero_copy = int(value);
    } else if (!std::strcmp(key, "small_call_bytes")) {
        if (value < 0) return RSMI_ERR_INVALID_ARG;
        c->opt_small_bytes = value;
    } else if (!std::strcmp(key, "coalesce_us")) {
        if (value < 0 || value > 100000) return RSMI_ERR_INVALID_ARG;
        c->opt_coalesce_us = value;
    } else if (!std::strcmp(key, "coalesce_max")) {
        if (value < 1 || value > 65536) return RSMI_ERR_INVALID_ARG;
        c->opt_coalesce_max = value;
    } else if (!std::strcmp(key, "crc16_fold")) {
        if (value < 0 || value > 1) return RSMI_ERR_INVALID_ARG;
        c->opt_crc16_fold = int(value);
    } else if (!std::strcmp(key, "crc32_fold")) {
        if (value < 0 || value > 1) return RSMI_ERR_INVALID_ARG;
        c->opt_crc32_fold = int(value);
    } else if (!std::strcmp(key, "crc16_fused_fold")) {
        if (value < 0 || value > 1) return RSMI_ERR_INVALID_ARG;
        c->opt_fused_fold = int(value);
    } else if (!std::strcmp(key, "waves_per_cu")) {
        if (value < 0) return RSMI_ERR_INVALID_ARG;
        c->opt_waves_per_cu = value;
    } else if (!std::strcmp(key, "inject_host_fault")) {
        if (value < 0 || value > 1000) return RSMI_ERR_INVALID_ARG;
        c->opt_inject_host_fault.store(int(value));
    } else if (!std::strcmp(key, "inject_lane_fault")) {
        if (value < 0 || value > 1000) return RSMI_ERR_INVALID_ARG;
        c->opt_inject_lane_fault.store(int(value));
    } else if (!std::strcmp(key, "coalesce_lanes")) {
        if (value < 1 || value > 16) return RSMI_ERR_INVALID_ARG;
        c->opt_coalesce_lanes = value;
    } else if (!std::strcmp(key, "coalesce_carry")) {
        if (value < 0 || value > 16) return RSMI_ERR_INVALID_ARG;
        c->opt_coalesce_carry = value;
    } else if (!std::strcmp(key, "coalesce_pipeline")) {
        if (value < 0 || value > 1) return RSMI_ERR_INVALID_ARG;
        c->opt_coalesce_pipeline = int(value);
    } else if (!std::strcmp(key, "coalesce_flag")) {
        if (value < 0 || value > 1) return RSMI_ERR_INVALID_ARG;
        c->opt_coalesce_flag = int(value);
    } else {
        return RSMI_ERR_INVALID_ARG;
    }
    return RSMI_OK;
}

}  // namespace impl
}  // namespace rsmi

extern "C" {

// a copy per calling thread: another thread's call may relabel the context meanwhile
const char* rsmi_last_kernel(const rsmi_ctx* c) {
    static thread_local std::string copy;
    if (!c) return "";
    std::lock_guard<std::mutex> g(c->lk_mu);
    copy = c->last_kernel;
    return copy.c_str();
}

void* rsmi_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (pinned_alloc(&p, bytes) != hipSuccess) return nullptr;
    return p;
}

void rsmi_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

// ---------------------------------------------------------------- device-resident batches
int rsmi_encode_batch_dev(rsmi_ctx* c, const uint8_t* d_data, size_t data_shard_stride, size_t data_block_stride,
                          uint8_t* d_parity, size_t parity_shard_stride, size_t parity_block_stride, size_t S,
                          size_t nblocks, void* stream) try {
    if (!c || !d_data || !d_parity) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    if (data_shard_stride < S || parity_shard_stride < S) return RSMI_ERR_INVALID_ARG;
    std::shared_ptr<Plan> plan;
    {
        std::lock_guard<std::mutex> g(c->mu);
        int rc = ensure_device(c);
        if (rc) return rc;
        HIP_TRY(hipSetDevice(c->device));
        rc = encode_plan(c, plan);
        if (rc) return rc;
        return launch_plan(c, *plan, d_data, data_shard_stride, data_block_stride, d_parity, parity_shard_stride,
                           parity_block_stride, S, nblocks, static_cast<hipStream_t>(stream));
    }
} catch (...) {
    return rsmi::impl::exception_status();
}

int rsmi_reconstruct_batch_dev(rsmi_ctx* c, uint8_t* d_shards, size_t shard_stride, size_t block_stride, size_t S,
                               size_t nblocks, const uint8_t* present, int data_only, void* stream) try {
    if (!c || !present) return RSMI_ERR_INVALID_ARG;
    const std::vector<uint8_t> w = want_mask(c, present, data_only);
    return reconstruct_dev_impl(c, d_shards, shard_stride, block_stride, S, nblocks, present, w.data(), stream);
} catch (...) {
    return rsmi::impl::exception_status();
}

int rsmi_reconstruct_rows_batch_dev(rsmi_ctx* c, uint8_t* d_shards, size_t shard_stride, size_t block_stride,
                                    size_t S, size_t nblocks, const uint8_t* present, const uint8_t* required,
                                    void* stream) try {
    return reconstruct_dev_impl(c, d_shards, shard_stride, block_stride, S, nblocks, present, required, stream);
} catch (...) {
    return rsmi::impl::exception_status();
}

}  // extern "C"
