// rsmi_api.cpp -- C-ABI implementation (include/rsmi.h): contexts, coding plans, launch
// dispatch, host staging with overlapped copies.  No CPU compute path: every byte of
// parity or reconstructed data comes out of the HIP kernels in rs_kernels.hip.
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
#include "gf256.hpp"
#include "rs_plan.hpp"

using namespace rsmi;

namespace {

size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

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

}  // namespace

struct rsmi_ctx {
    int k = 0, m = 0, n = 0, device = 0;
    Matrix M;  // n x k
    std::mutex mu;
    bool dev_ready = false;
    int dev_status = RSMI_OK;
    int num_cu = 256;
    std::map<std::string, std::shared_ptr<Plan>> plans;
    std::map<void*, int> occupancy;
    std::vector<Staging> staging;  // [0] single-block calls, [0..2] batch pipeline
    uint8_t* h_stage = nullptr;    // pinned landing area for rebuilt rows (odd S)
    size_t h_stage_cap = 0;
    uint32_t* d_crc_tbl = nullptr;  // CRC-16 device tables (crc16.hpp), uploaded on first use
    uint8_t* d_crc = nullptr;       // raw row CRCs (u32) of host batch calls
    size_t crc_cap = 0;
    uint8_t* d_chunks = nullptr;    // per-chunk CRC-16 values of fused small calls (u16)
    size_t chunks_cap = 0;
    // options
    int opt_d = 1;
    int opt_nt = -1;  // cache policy, -1 = auto_cache_policy(MT) (see there)
    long opt_waves_per_cu = 0;
    int opt_prefetch = 0;
    int opt_zero_copy = 1;  // results into page-locked host buffers by kernel stores
    int opt_crc_fold = 1;   // CRC chunk fold: 1 = nibble tables, 0 = byte tables (A/B)
    int opt_tables = 0;     // 1 = split LDS/SGPR table source (A/B, RS(10,4) shapes)
    long opt_small_bytes = 2L << 20;  // host calls up to this many shard bytes run zero-copy
    uint8_t* h_small = nullptr;       // page-locked staging of small calls (pageable callers)
    size_t h_small_cap = 0;
    long opt_coalesce_us = 0;     // extra wait for more callers before a coalesced batch runs
    long opt_coalesce_max = 256;  // blocks per coalesced batch
    std::string last_kernel;
    // group commit for rsmi_encode_block_coalesced (see there)
    struct CoalReq {
        // encode: block/B in, out = (k+m)*S shards, raw optional; reconstruct: out = n*S
        // shards in place, present / want flags (group key covers S, pattern, want)
        const uint8_t* block;
        size_t B;
        uint8_t* out;
        uint32_t* raw;
        std::string key;
        int rc;
        bool done;
    };
    std::mutex q_mu;
    std::condition_variable q_cv;
    std::vector<CoalReq*> q_pending;
    bool q_executing = false;
    uint8_t* h_coal = nullptr;  // page-locked staging of the executing batch
    size_t h_coal_cap = 0;
    std::atomic<uint64_t> stat_coal_calls{0}, stat_coal_batches{0};
};

namespace {

int hip_status(hipError_t e) {
    if (e == hipSuccess) return RSMI_OK;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice || e == hipErrorNoBinaryForGpu ||
        e == hipErrorInsufficientDriver)
        return RSMI_ERR_NO_DEVICE;
    return RSMI_ERR_DEVICE;
}

#define HIP_TRY(expr)                                   \
    do {                                                \
        hipError_t _e = (expr);                         \
        if (_e != hipSuccess) return hip_status(_e);    \
    } while (0)

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
    return RSMI_OK;
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

const char* kernel_label(int K, int MT, int D, int NT, bool fast) {
    static thread_local char buf[96];
    if (fast)
        std::snprintf(buf, sizeof buf, "rs_fast_kernel<K=%d,MT=%d,D=%d,NT=%d>", K, MT, D, NT);
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

// Launch every tile of a plan over nblocks blocks.
// Fused per-chunk CRC output of a launch (rs_fast_kernel CRC variants): chunk values of every
// row the plan reads or writes, at out[(block * slots + shard) * cpb + chunk].
struct CrcFuse {
    const uint32_t* tbl = nullptr;
    uint16_t* out = nullptr;
    uint32_t slots = 0, out_slot0 = 0;
};

int launch_plan(rsmi_ctx* c, const Plan& plan, const uint8_t* in, uint64_t in_rs, uint64_t in_bs, uint8_t* out,
                uint64_t out_rs, uint64_t out_bs, uint64_t S, uint64_t nblocks, hipStream_t stream,
                const CrcFuse* fuse = nullptr) {
    if (nblocks == 0 || S == 0) return RSMI_OK;
    const bool aligned = (reinterpret_cast<uintptr_t>(in) % 16 == 0) && (reinterpret_cast<uintptr_t>(out) % 16 == 0) &&
                         in_rs % 16 == 0 && in_bs % 16 == 0 && out_rs % 16 == 0 && out_bs % 16 == 0 &&
                         in_rs >= round_up(S, 16) && out_rs >= round_up(S, 16) && S < (uint64_t(1) << 31);
    // any other layout with rows of at least 16 bytes: the unaligned-window variant (D = 1)
    const bool ua = (!aligned || fuse) && S >= 16 && S < (uint64_t(1) << 31) && in_rs >= S && out_rs >= S;
    if (fuse && !ua) return RSMI_ERR_INVALID_ARG;  // callers fall back to the separate CRC pass
    for (const DevTile& t : plan.tiles) {
        const int D = ua ? 1 : c->opt_d;
        int NT = c->opt_nt >= 0 ? c->opt_nt : auto_cache_policy(t.K, t.MT);
        if (ua && NT == 0) NT = auto_cache_policy(t.K, t.MT);  // UA variants exist for policies 1 and 2
        void* fn = nullptr;
        if (aligned && t.K <= 16) fn = fast_kernels().fn[t.K][t.MT][D][NT];
        if (ua && t.K <= 16) fn = fuse ? fast_kernels().ua_crc[t.K][t.MT] : fast_kernels().ua[t.K][t.MT][NT];
        if (fuse && !fn) return RSMI_ERR_INVALID_ARG;
        if (fuse) NT = auto_cache_policy(t.K, t.MT);  // the one policy the fused variants have
        int pf_label = 0, ts_label = 0;
        if (fn && !ua && c->opt_prefetch && t.K == 10 && (t.MT == 4 || t.MT == 1) && D == 1 && NT == 1) {
            const int pi = c->opt_prefetch == 4 ? 0 : c->opt_prefetch == 8 ? 1 : 2;
            fn = exp_kernels().fn[t.MT == 4 ? 0 : 1][pi];
            pf_label = c->opt_prefetch;
        } else if (fn && !ua && c->opt_tables >= 1 && t.K == 10 && D == 1 &&
                   ((t.MT == 4 && NT == 1) || (t.MT == 1 && NT == 2))) {
            fn = exp_kernels().fn[t.MT == 4 ? 0 : 1][c->opt_tables == 1 ? 3 : 4];
            ts_label = c->opt_tables;
        }
        if (fn) {
            const uint64_t cpb = (S + 15) / 16;
            const uint64_t tpb = (cpb + uint64_t(kWave * D) - 1) / uint64_t(kWave * D);
            int& occ = c->occupancy[fn];  // queried once per kernel, not per launch
            if (occ <= 0) {
                HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, kWG, 0));
                if (occ <= 0) occ = 1;
            }
            long wg_cap = long(c->num_cu) * occ;
            if (c->opt_waves_per_cu > 0) wg_cap = std::max(1L, long(c->num_cu) * c->opt_waves_per_cu / (kWG / kWave));
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
                uint16_t* cout = fuse ? fuse->out + b0 * fuse->slots * tpb * kWave : nullptr;
                uint32_t cslots = fuse ? fuse->slots : 0, cslot0 = fuse ? fuse->out_slot0 : 0;
                void* args[] = {&pd,    &inb,    &outb,  &in_bs, &in_rs, &out_bs, &out_rs, &S32,
                                &cpb32, &tpb32, &ntiles, &ctbl,  &cout,  &cslots, &cslot0};
                const uint64_t wgs = std::min<uint64_t>((ntiles + 3) / 4, uint64_t(wg_cap));
                HIP_TRY(hipLaunchKernel(fn, dim3(uint32_t(wgs)), dim3(kWG), args, 0, stream));
            }
            c->last_kernel = kernel_label(t.K, t.MT, D, NT, true);
            if (ua) c->last_kernel += ",UA";
            if (fuse) c->last_kernel += ",CRC";
            if (pf_label) c->last_kernel += ",PF=" + std::to_string(pf_label);
            if (ts_label) c->last_kernel += ts_label == 1 ? ",TS=1" : ",SH64";
        } else {
            const uint64_t groups = (S + 3) / 4;
            const uint32_t gx = uint32_t(std::min<uint64_t>((groups + kWG - 1) / kWG, 4096));
            const uint32_t gy = uint32_t(std::min<uint64_t>(nblocks, 65535));
            const RsPlanDev* pd = t.dev;
            void* args[] = {&pd, &in, &out, &in_bs, &in_rs, &out_bs, &out_rs, &S, &nblocks};
            HIP_TRY(hipLaunchKernel(generic_kernel(), dim3(gx, gy), dim3(kWG), args, 0, stream));
            c->last_kernel = kernel_label(t.K, t.MT, 0, 0, false);
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

}  // namespace

// ====================================================================== C-ABI
extern "C" {

int rsmi_abi_version(void) { return RSMI_ABI_VERSION; }

const char* rsmi_status_string(int s) {
    switch (s) {
        case RSMI_OK: return "ok";
        case RSMI_ERR_SHORT_DATA: return "not enough data to fill the number of requested shards";
        case RSMI_ERR_TOO_FEW_SHARDS: return "too few shards given";
        case RSMI_ERR_SHARD_NO_DATA: return "no shard data";
        case RSMI_ERR_SHARD_SIZE: return "shard sizes do not match";
        case RSMI_ERR_INV_SHARD_NUM: return "cannot create Encoder with less than one data shard or less than zero parity shards";
        case RSMI_ERR_MAX_SHARD_NUM: return "cannot create Encoder with more than 256 data+parity shards";
        case RSMI_ERR_SINGULAR: return "matrix is singular";
        case RSMI_ERR_INVALID_ARG: return "invalid argument";
        case RSMI_ERR_DEVICE: return "HIP device error";
        case RSMI_ERR_NO_DEVICE: return "no usable gfx950 device";
        default: return "unknown status";
    }
}

int rsmi_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int rsmi_open(int k, int m, int device, rsmi_ctx** out) {
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
}

void rsmi_close(rsmi_ctx* c) {
    if (!c) return;
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
            if (c->d_crc_tbl) (void)hipFree(c->d_crc_tbl);
            if (c->d_crc) (void)hipFree(c->d_crc);
            if (c->d_chunks) (void)hipFree(c->d_chunks);
        }
    }
    delete c;
}

size_t rsmi_recommended_pitch(size_t S) {
    if (S == 0) return 0;
    size_t p = 16;
    while (p < S) p <<= 1;
    // Measured on MI355X (tools/pitchsweep*.py, DESIGN.md "Layout"): a power-of-two row
    // pitch is +13% for S = 26215 (32 KiB) and best for S = 262144 (itself a power of
    // two), but the worst choice for S = 104858 (128 KiB: -4% vs 4 KiB granules).  Use
    // powers of two for shards up to 64 KiB (padding <= 50%) and exact powers; otherwise
    // 4 KiB granules.
    if (p == S || p <= 4096) return p;
    if (S <= 65536 && p <= S + S / 2) return p;
    return round_up(S, 4096);
}

size_t rsmi_shard_size(size_t block_size, int k) {
    if (k <= 0) return 0;
    return (block_size + size_t(k) - 1) / size_t(k);
}

int rsmi_encode_matrix(const rsmi_ctx* c, uint8_t* out) {
    if (!c || !out) return RSMI_ERR_INVALID_ARG;
    std::memcpy(out, c->M.v.data(), c->M.v.size());
    return RSMI_OK;
}

int rsmi_check_shards(int n, const size_t* lens, int nil_ok, size_t* S_out) {
    if (!lens || n <= 0) return RSMI_ERR_INVALID_ARG;
    size_t S = 0;
    for (int i = 0; i < n; i++)
        if (lens[i]) {
            S = lens[i];
            break;
        }
    if (S_out) *S_out = S;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    for (int i = 0; i < n; i++)
        if (lens[i] != S && (lens[i] != 0 || !nil_ok)) return RSMI_ERR_SHARD_SIZE;
    return RSMI_OK;
}

int rsmi_decode_matrix(const rsmi_ctx* c, const uint8_t* present, uint8_t* out, int* used_rows) {
    if (!c || !present || !out) return RSMI_ERR_INVALID_ARG;
    Matrix dec;
    std::vector<int> used;
    int rc = decode_rows(c, present, dec, used);
    if (rc) return rc;
    std::memcpy(out, dec.v.data(), dec.v.size());
    if (used_rows)
        for (int i = 0; i < c->k; i++) used_rows[i] = used[i];
    return RSMI_OK;
}

int rsmi_set_option(rsmi_ctx* c, const char* key, long value) {
    if (!c || !key) return RSMI_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    if (!std::strcmp(key, "chunks_per_lane")) {
        if (value != 1 && value != 2) return RSMI_ERR_INVALID_ARG;
        c->opt_d = int(value);
    } else if (!std::strcmp(key, "nontemporal")) {
        if (value < -1 || value > 2) return RSMI_ERR_INVALID_ARG;
        c->opt_nt = int(value);
    } else if (!std::strcmp(key, "prefetch")) {
        // 4/8/10 = rows in flight (A/B only; RS(10,4) encode and 1-row reconstruct, NT=1)
        if (value != 0 && value != 4 && value != 8 && value != 10)
            return RSMI_ERR_INVALID_ARG;
        c->opt_prefetch = int(value);
    } else if (!std::strcmp(key, "zero_copy")) {
        if (value < 0 || value > 2) return RSMI_ERR_INVALID_ARG;
        c->opt_zero_copy = int(value);
    } else if (!std::strcmp(key, "tables")) {
        if (value < 0 || value > 2) return RSMI_ERR_INVALID_ARG;
        c->opt_tables = int(value);
    } else if (!std::strcmp(key, "small_call_bytes")) {
        if (value < 0) return RSMI_ERR_INVALID_ARG;
        c->opt_small_bytes = value;
    } else if (!std::strcmp(key, "coalesce_us")) {
        if (value < 0 || value > 100000) return RSMI_ERR_INVALID_ARG;
        c->opt_coalesce_us = value;
    } else if (!std::strcmp(key, "coalesce_max")) {
        if (value < 1 || value > 65536) return RSMI_ERR_INVALID_ARG;
        c->opt_coalesce_max = value;
    } else if (!std::strcmp(key, "crc_fold")) {
        if (value != 0 && value != 1) return RSMI_ERR_INVALID_ARG;
        c->opt_crc_fold = int(value);
    } else if (!std::strcmp(key, "waves_per_cu")) {
        if (value < 0) return RSMI_ERR_INVALID_ARG;
        c->opt_waves_per_cu = value;
    } else {
        return RSMI_ERR_INVALID_ARG;
    }
    return RSMI_OK;
}

const char* rsmi_last_kernel(const rsmi_ctx* c) { return c ? c->last_kernel.c_str() : ""; }

void* rsmi_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
    return p;
}

void rsmi_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

// ---------------------------------------------------------------- device-resident batches
int rsmi_encode_batch_dev(rsmi_ctx* c, const uint8_t* d_data, size_t data_shard_stride, size_t data_block_stride,
                          uint8_t* d_parity, size_t parity_shard_stride, size_t parity_block_stride, size_t S,
                          size_t nblocks, void* stream) {
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
}

static int reconstruct_dev_impl(rsmi_ctx* c, uint8_t* d_shards, size_t shard_stride, size_t block_stride, size_t S,
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

int rsmi_reconstruct_batch_dev(rsmi_ctx* c, uint8_t* d_shards, size_t shard_stride, size_t block_stride, size_t S,
                               size_t nblocks, const uint8_t* present, int data_only, void* stream) {
    if (!c || !present) return RSMI_ERR_INVALID_ARG;
    const std::vector<uint8_t> w = want_mask(c, present, data_only);
    return reconstruct_dev_impl(c, d_shards, shard_stride, block_stride, S, nblocks, present, w.data(), stream);
}

int rsmi_reconstruct_rows_batch_dev(rsmi_ctx* c, uint8_t* d_shards, size_t shard_stride, size_t block_stride,
                                    size_t S, size_t nblocks, const uint8_t* present, const uint8_t* required,
                                    void* stream) {
    return reconstruct_dev_impl(c, d_shards, shard_stride, block_stride, S, nblocks, present, required, stream);
}

// ---------------------------------------------------------------- host memory, one block
int rsmi_encode(rsmi_ctx* c, const uint8_t* data, uint8_t* parity, size_t S) {
    if (!c || !data || !parity) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    return rsmi_encode_batch_host(c, data, size_t(c->k) * S, parity, size_t(c->m) * S, S, 1);
}

int rsmi_encode_block(rsmi_ctx* c, const uint8_t* block, size_t B, uint8_t* shards_out) {
    if (!c) return RSMI_ERR_INVALID_ARG;
    if (B == 0) return RSMI_ERR_SHORT_DATA;  // upstream Split checks this first
    if (!block || !shards_out) return RSMI_ERR_INVALID_ARG;
    const size_t S = rsmi_shard_size(B, c->k);
    std::memcpy(shards_out, block, B);
    std::memset(shards_out + B, 0, size_t(c->k) * S - B);  // Split zero-padding
    return rsmi_encode(c, shards_out, shards_out + size_t(c->k) * S, S);
}

int rsmi_reconstruct(rsmi_ctx* c, uint8_t* shards, size_t S, const uint8_t* present, int data_only) {
    if (!c || !shards || !present) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    return rsmi_reconstruct_batch_host(c, shards, size_t(c->n) * S, S, 1, present, data_only);
}

}  // extern "C"

// ---------------------------------------------------------------- host memory, batches
// Pipeline: chunks of blocks round-robin over 3 streams, each with its own device
// buffers: H2D -> kernel -> D2H.  When S is a multiple of 8 the DMA engines move rows
// straight between the contiguous host layout (pitch S) and the pitched device layout with
// 2-D copies at full PCIe rate.  Odd-width 2-D copies crawl (3-9 GB/s measured,
// tools/copyprobe.py), so for other S the PCIe copies stay linear and rs_repitch_kernel
// re-lays rows out on the device (HBM-speed, ~1% of the PCIe time).
namespace {

bool dma_2d_ok(size_t S) { return S % 8 == 0; }

int repitch(uint8_t* dst, size_t dpitch, const uint8_t* src, size_t spitch, size_t width, size_t rows,
            hipStream_t stream) {
    if (!rows || !width) return RSMI_OK;
    uint64_t sp = spitch, dp = dpitch, w = width, r = rows;
    const uint64_t dwords = ((w + 6) / 4 + 1) * r;
    const uint32_t grid = uint32_t(std::min<uint64_t>((dwords + kWG - 1) / kWG, 8192));
    void* args[] = {&src, &sp, &dst, &dp, &w, &r};
    HIP_TRY(hipLaunchKernel(repitch_kernel(), dim3(grid), dim3(kWG), args, 0, stream));
    return RSMI_OK;
}

// Device-visible alias of the page-locked host range [p, p + len) (hipHostMalloc /
// rsmi_host_alloc memory), or nullptr when the range is pageable memory.  On the odd-S
// (linear copy) path, results bound for such a range are written by the repitch kernel
// straight over PCIe: the copy engines were measured running the linear host->device and
// device->host transfers one after the other, and taking the write-back off them lets it
// overlap the next chunk's upload (tools/hostsweep.py, RS(10,4) 256 KiB: encode 41.7 -> 47.6
// GiB/s).  Reconstruct also uploads by kernel loads from such memory (below).  With 2-D
// DMA rows (S % 8 == 0) the engines already overlap, so that path keeps its copies.
uint8_t* host_alias(void* p, size_t len) {
    auto alias = [](void* q) -> uint8_t* {
        hipPointerAttribute_t a{};
        if (hipPointerGetAttributes(&a, q) != hipSuccess) {
            (void)hipGetLastError();  // pageable memory: not an error for the caller
            return nullptr;
        }
        if (a.type != hipMemoryTypeHost || !a.devicePointer || !a.hostPointer) return nullptr;
        return static_cast<uint8_t*>(a.devicePointer) + (static_cast<uint8_t*>(q) - static_cast<uint8_t*>(a.hostPointer));
    };
    uint8_t* first = alias(p);
    if (!first || len == 0) return first;
    uint8_t* last = alias(static_cast<uint8_t*>(p) + len - 1);
    return last == first + (len - 1) ? first : nullptr;  // one allocation end to end
}

// CRC-16 device tables, uploaded once per context (caller holds ctx->mu)
int ensure_crc_tables(rsmi_ctx* c) {
    if (c->d_crc_tbl) return RSMI_OK;
    const Crc16Tables& t = crc16_tables();
    static_assert(sizeof(t.P) + sizeof(t.U) + sizeof(t.N) == size_t(kCrcTableWords) * 4, "CRC table layout");
    std::vector<uint16_t> h(size_t(kCrcTableWords) * 2);
    std::memcpy(h.data(), t.P, sizeof(t.P));
    std::memcpy(h.data() + kCrcPWords * 2, t.U, sizeof(t.U));
    std::memcpy(h.data() + (kCrcPWords + kCrcUWords) * 2, t.N, sizeof(t.N));
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&c->d_crc_tbl), h.size() * 2));
    HIP_TRY(hipMemcpy(c->d_crc_tbl, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    return RSMI_OK;
}

// R(row) of nrows rows per block into out[b*out_bs + r] (zeroed first), stream-ordered.
int launch_crc(rsmi_ctx* c, const uint8_t* base, uint64_t rpitch, uint64_t bstride, uint32_t nrows, uint64_t S,
               uint64_t nblocks, uint32_t* out, uint64_t out_bs, hipStream_t stream, bool zero = true) {
    if (!nblocks || !nrows) return RSMI_OK;
    int rc = ensure_crc_tables(c);
    if (rc) return rc;
    if (zero) HIP_TRY(hipMemset2DAsync(out, out_bs * 4, 0, size_t(nrows) * 4, nblocks, stream));
    if (S == 0) return RSMI_OK;  // R(empty) = 0
    const bool aligned = reinterpret_cast<uintptr_t>(base) % 16 == 0 && rpitch % 16 == 0 && bstride % 16 == 0;
    void* fn = crc16_rows_kernel(aligned, c->opt_crc_fold);
    const uint64_t tile = uint64_t(kWave) * 16;
    uint32_t tpb = uint32_t((S + tile - 1) / tile);
    uint32_t nseg = (tpb + kCrcSegTiles - 1) / kCrcSegTiles;
    uint64_t nitems = nblocks * nrows * nseg;
    int& occ = c->occupancy[fn];
    if (occ <= 0) {
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, kWG, 0));
        if (occ <= 0) occ = 1;
    }
    const uint64_t wgs = std::min<uint64_t>((nitems + 3) / 4, uint64_t(c->num_cu) * uint64_t(occ));
    const uint32_t* tb = c->d_crc_tbl;
    void* args[] = {&tb, &base, &bstride, &rpitch, &nrows, &S, &tpb, &nseg, &nitems, &out, &out_bs};
    HIP_TRY(hipLaunchKernel(fn, dim3(uint32_t(wgs)), dim3(kWG), args, 0, stream));
    return RSMI_OK;
}

}  // namespace

extern "C" {

// ---------------------------------------------------------------- small host calls
// A per-block call (DagNode.Put / Get, one 256 KiB block) is latency-bound: the copy-engine
// path pays a DMA setup on each side of the kernel.  Small calls instead run ONE kernel that
// reads its input rows from page-locked host memory and writes its output rows back over
// PCIe (the unaligned-window kernels take the Split layout's odd row pitch as is).  Pageable
// callers (Go slices over cgo) are staged through a page-locked buffer by CPU copies.
// Caller holds ctx->mu.
static uint8_t* small_stage(rsmi_ctx* c, size_t need) {
    if (c->h_small_cap >= need) return c->h_small;
    if (c->h_small) (void)hipHostFree(c->h_small);
    c->h_small = nullptr;
    c->h_small_cap = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(&c->h_small), std::max<size_t>(need, 1 << 20), hipHostMallocDefault) !=
        hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    c->h_small_cap = std::max<size_t>(need, 1 << 20);
    return c->h_small;
}

// Encode with fused per-chunk CRCs, then R(row) of all k+m rows of every block into
// raw[b * (k+m) + row] (device or page-locked host memory).  Needs S >= 16 and k <= 16.
static int launch_encode_crc(rsmi_ctx* c, const Plan& plan, const uint8_t* in, size_t in_rs, size_t in_bs, uint8_t* out,
                             size_t out_rs, size_t out_bs, size_t S, size_t nblocks, uint32_t* raw, hipStream_t st) {
    const size_t k = size_t(c->k), n = size_t(c->n);
    const size_t cpb = (S + 15) / 16, pitch = (cpb + kWave - 1) / kWave * kWave;
    int rc;
    if ((rc = ensure_crc_tables(c))) return rc;
    if ((rc = reserve(c->d_chunks, c->chunks_cap, nblocks * n * pitch * 2))) return rc;
    CrcFuse fz;
    fz.tbl = c->d_crc_tbl;
    fz.out = reinterpret_cast<uint16_t*>(c->d_chunks);
    fz.slots = uint32_t(n);
    fz.out_slot0 = uint32_t(k);
    if ((rc = launch_plan(c, plan, in, in_rs, in_bs, out, out_rs, out_bs, S, nblocks, st, &fz))) return rc;
    const uint16_t* ch = fz.out;
    uint32_t cpb32 = uint32_t(cpb), pitch32 = uint32_t(pitch);
    uint64_t S64 = S, rows = nblocks * n;
    const uint32_t* tb = c->d_crc_tbl;
    void* args[] = {&tb, &ch, &cpb32, &pitch32, &S64, &rows, &raw};
    const uint32_t grid = uint32_t(std::min<uint64_t>((rows + 3) / 4, uint64_t(c->num_cu) * 4));
    HIP_TRY(hipLaunchKernel(crc16_combine_kernel(), dim3(grid), dim3(kWG), args, 0, st));
    return RSMI_OK;
}

static int encode_small(rsmi_ctx* c, const Plan& plan, const uint8_t* data, size_t dbs, uint8_t* parity, size_t pbs,
                        size_t S, size_t nblocks, uint32_t* raw_out) {
    const size_t k = size_t(c->k), m = size_t(c->m), n = k + m;
    hipStream_t st = c->staging[0].stream;
    const uint8_t* in = host_alias(const_cast<uint8_t*>(data), (nblocks - 1) * dbs + k * S);
    uint8_t* out = host_alias(parity, (nblocks - 1) * pbs + m * S);
    size_t in_bs = dbs, out_bs = pbs;
    // page-locked staging, only the parts needed: [data rows | parity rows | raw CRCs]
    const bool stage_in = in == nullptr, stage_out = out == nullptr;
    const size_t in_sz = stage_in ? nblocks * k * S : 0, out_sz = stage_out ? nblocks * m * S : 0;
    const size_t raw_sz = raw_out ? nblocks * n * 4 : 0;
    uint8_t* hs = nullptr;
    if (in_sz + out_sz + raw_sz) {
        hs = small_stage(c, in_sz + out_sz + raw_sz);
        if (!hs) return RSMI_ERR_DEVICE;
    }
    if (stage_in) {
        for (size_t b = 0; b < nblocks; b++) std::memcpy(hs + b * k * S, data + b * dbs, k * S);
        in = host_alias(hs, in_sz);
        in_bs = k * S;
    }
    uint8_t* hout = hs ? hs + in_sz : nullptr;
    if (stage_out) {
        out = host_alias(hout, out_sz);
        out_bs = m * S;
    }
    uint32_t* hraw = raw_out ? reinterpret_cast<uint32_t*>(hs + in_sz + out_sz) : nullptr;
    if (!in || !out) return RSMI_ERR_DEVICE;
    int rc;
    if (raw_out && S >= 16 && k <= 16) {
        // fused: the encode stores per-chunk CRCs of every row it reads and writes (the shard
        // bytes cross PCIe once), then one wave per row combines them into R(row) and stores
        // it straight into the page-locked staging
        uint32_t* draw = reinterpret_cast<uint32_t*>(host_alias(hraw, raw_sz));
        if (!draw) return RSMI_ERR_DEVICE;
        if ((rc = launch_encode_crc(c, plan, in, S, in_bs, out, S, out_bs, S, nblocks, draw, st))) return rc;
    } else {
        if ((rc = launch_plan(c, plan, in, S, in_bs, out, S, out_bs, S, nblocks, st))) return rc;
        if (raw_out) {  // S < 16 or k > 16: a separate CRC pass over the rows where they lie
            if ((rc = reserve(c->d_crc, c->crc_cap, raw_sz))) return rc;
            uint32_t* cr = reinterpret_cast<uint32_t*>(c->d_crc);
            HIP_TRY(hipMemsetAsync(cr, 0, raw_sz, st));
            if ((rc = launch_crc(c, in, S, in_bs, uint32_t(k), S, nblocks, cr, n, st, false))) return rc;
            if ((rc = launch_crc(c, out, S, out_bs, uint32_t(m), S, nblocks, cr + k, n, st, false))) return rc;
            if ((rc = repitch(host_alias(hraw, raw_sz), raw_sz, reinterpret_cast<uint8_t*>(cr), raw_sz, raw_sz, 1,
                              st)))
                return rc;
        }
    }
    HIP_TRY(hipStreamSynchronize(st));
    if (stage_out)
        for (size_t b = 0; b < nblocks; b++) std::memcpy(parity + b * pbs, hout + b * m * S, m * S);
    if (raw_out) std::memcpy(raw_out, hraw, raw_sz);
    return RSMI_OK;
}

static int encode_host_impl(rsmi_ctx* c, const uint8_t* data, size_t data_block_stride, uint8_t* parity,
                            size_t parity_block_stride, size_t S, size_t nblocks, uint32_t* raw_out) {
    if (!c || !data || !parity) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    if (data_block_stride < size_t(c->k) * S || parity_block_stride < size_t(c->m) * S) return RSMI_ERR_INVALID_ARG;
    if (nblocks == 0) return RSMI_OK;
    std::lock_guard<std::mutex> g(c->mu);
    int rc = ensure_device(c);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    std::shared_ptr<Plan> plan;
    rc = encode_plan(c, plan);
    if (rc) return rc;
    const size_t k = size_t(c->k), m = size_t(c->m);
    // One zero-copy kernel (encode_small) when both sides are page-locked, whatever the size
    // (tools/hostsweep.py "direct": equal to the copy-engine pipeline for encode, +8-18% for
    // reconstruct), or when the call is small; pageable input is staged by CPU copies, and
    // above half the small-call limit the copy engines win (tools/latency.cpp, 1 MiB blocks:
    // 107 us staged against 99 us).
    const size_t total = nblocks * (k + m) * S;
    const bool in_pinned = host_alias(const_cast<uint8_t*>(data), (nblocks - 1) * data_block_stride + k * S);
    const bool pinned = in_pinned && host_alias(parity, (nblocks - 1) * parity_block_stride + m * S);
    if ((c->opt_zero_copy && pinned) ||
        (total <= size_t(c->opt_small_bytes) && (2 * total <= size_t(c->opt_small_bytes) || in_pinned)))
        return encode_small(c, *plan, data, data_block_stride, parity, parity_block_stride, S, nblocks, raw_out);
    const size_t Sp = rsmi_recommended_pitch(S);
    const size_t in_bs = k * Sp, out_bs = m * Sp;
    const bool d2 = dma_2d_ok(S);
    const size_t chunk = std::max<size_t>(1, (size_t(64) << 20) / (in_bs + out_bs));
    const int ns = nblocks > chunk ? 3 : 1;
    // odd S: parity straight into page-locked host memory when it is one contiguous
    // [block][row][S] run (host_alias); 2-D DMA rows stay faster than kernel stores
    uint8_t* zc = c->opt_zero_copy && !d2 ? host_alias(parity, (nblocks - 1) * parity_block_stride + m * S) : nullptr;
    // zero_copy 2 (A/B only): the upload by kernel loads too (RS(10,4) 256 KiB: 47.6 -> 34.6
    // GiB/s; the copy engine uploads a whole data block faster than kernel loads do)
    const uint8_t* zin = c->opt_zero_copy == 2 && !d2
                             ? host_alias(const_cast<uint8_t*>(data), (nblocks - 1) * data_block_stride + k * S)
                             : nullptr;
    const size_t n = k + m;
    if (raw_out && (rc = reserve(c->d_crc, c->crc_cap, nblocks * n * 4))) return rc;
    for (size_t b0 = 0, i = 0; b0 < nblocks; b0 += chunk, i++) {
        Staging& st = c->staging[i % ns];
        const size_t nb = std::min(chunk, nblocks - b0);
        if ((rc = reserve(st.d_in, st.in_cap, nb * in_bs))) return rc;
        if ((rc = reserve(st.d_out, st.out_cap, nb * out_bs))) return rc;
        if (!d2 && !zin && (rc = reserve(st.d_lin, st.lin_cap, nb * k * S))) return rc;
        const uint8_t* src = data + b0 * data_block_stride;
        uint8_t* dst = parity + b0 * parity_block_stride;
        // host -> device
        if (zin) {
            for (size_t r = 0; r < k; r++)
                if ((rc = repitch(st.d_in + r * Sp, in_bs, zin + b0 * data_block_stride + r * S, data_block_stride, S,
                                  nb, st.stream)))
                    return rc;
        } else if (d2 && data_block_stride == k * S) {
            HIP_TRY(hipMemcpy2DAsync(st.d_in, Sp, src, S, S, nb * k, hipMemcpyHostToDevice, st.stream));
        } else if (d2) {
            for (size_t b = 0; b < nb; b++)
                HIP_TRY(hipMemcpy2DAsync(st.d_in + b * in_bs, Sp, src + b * data_block_stride, S, S, k,
                                         hipMemcpyHostToDevice, st.stream));
        } else {
            if (data_block_stride == k * S)
                HIP_TRY(hipMemcpyAsync(st.d_lin, src, nb * k * S, hipMemcpyHostToDevice, st.stream));
            else
                for (size_t b = 0; b < nb; b++)
                    HIP_TRY(hipMemcpyAsync(st.d_lin + b * k * S, src + b * data_block_stride, k * S,
                                           hipMemcpyHostToDevice, st.stream));
            if ((rc = repitch(st.d_in, Sp, st.d_lin, S, S, nb * k, st.stream))) return rc;
        }
        if ((rc = launch_plan(c, *plan, st.d_in, Sp, in_bs, st.d_out, Sp, out_bs, S, nb, st.stream))) return rc;
        if (raw_out) {  // R(shard) of the k data rows and the m parity rows, [block][row]
            uint32_t* cr = reinterpret_cast<uint32_t*>(c->d_crc) + b0 * n;
            HIP_TRY(hipMemsetAsync(cr, 0, nb * n * 4, st.stream));
            if ((rc = launch_crc(c, st.d_in, Sp, in_bs, uint32_t(k), S, nb, cr, n, st.stream, false))) return rc;
            if ((rc = launch_crc(c, st.d_out, Sp, out_bs, uint32_t(m), S, nb, cr + k, n, st.stream, false)))
                return rc;
        }
        // device -> host
        if (zc && parity_block_stride == m * S) {
            if ((rc = repitch(zc + b0 * m * S, S, st.d_out, Sp, S, nb * m, st.stream))) return rc;
        } else if (zc) {
            for (size_t r = 0; r < m; r++)
                if ((rc = repitch(zc + b0 * parity_block_stride + r * S, parity_block_stride, st.d_out + r * Sp, out_bs,
                                  S, nb, st.stream)))
                    return rc;
        } else if (d2 && parity_block_stride == m * S) {
            HIP_TRY(hipMemcpy2DAsync(dst, S, st.d_out, Sp, S, nb * m, hipMemcpyDeviceToHost, st.stream));
        } else if (d2) {
            for (size_t b = 0; b < nb; b++)
                HIP_TRY(hipMemcpy2DAsync(dst + b * parity_block_stride, S, st.d_out + b * out_bs, Sp, S, m,
                                         hipMemcpyDeviceToHost, st.stream));
        } else {
            // reuse d_lin (its H2D contents are consumed by the repitch above, in stream order)
            if ((rc = repitch(st.d_lin, S, st.d_out, Sp, S, nb * m, st.stream))) return rc;
            if (parity_block_stride == m * S)
                HIP_TRY(hipMemcpyAsync(dst, st.d_lin, nb * m * S, hipMemcpyDeviceToHost, st.stream));
            else
                for (size_t b = 0; b < nb; b++)
                    HIP_TRY(hipMemcpyAsync(dst + b * parity_block_stride, st.d_lin + b * m * S, m * S,
                                           hipMemcpyDeviceToHost, st.stream));
        }
    }
    for (int s = 0; s < ns; s++) HIP_TRY(hipStreamSynchronize(c->staging[s].stream));
    if (raw_out) HIP_TRY(hipMemcpy(raw_out, c->d_crc, nblocks * n * 4, hipMemcpyDeviceToHost));
    return RSMI_OK;
}

int rsmi_encode_batch_host(rsmi_ctx* c, const uint8_t* data, size_t data_block_stride, uint8_t* parity,
                           size_t parity_block_stride, size_t S, size_t nblocks) {
    return encode_host_impl(c, data, data_block_stride, parity, parity_block_stride, S, nblocks, nullptr);
}

int rsmi_encode_batch_host_crc(rsmi_ctx* c, const uint8_t* data, size_t data_block_stride, uint8_t* parity,
                               size_t parity_block_stride, size_t S, size_t nblocks, uint32_t* raw_out) {
    if (!raw_out) return RSMI_ERR_INVALID_ARG;
    return encode_host_impl(c, data, data_block_stride, parity, parity_block_stride, S, nblocks, raw_out);
}

int rsmi_encode_block_crc(rsmi_ctx* c, const uint8_t* block, size_t B, uint8_t* shards_out, uint32_t* raw_out) {
    if (!c) return RSMI_ERR_INVALID_ARG;
    if (B == 0) return RSMI_ERR_SHORT_DATA;
    if (!block || !shards_out || !raw_out) return RSMI_ERR_INVALID_ARG;
    const size_t S = rsmi_shard_size(B, c->k);
    std::memcpy(shards_out, block, B);
    std::memset(shards_out + B, 0, size_t(c->k) * S - B);  // Split zero-padding
    return encode_host_impl(c, shards_out, size_t(c->k) * S, shards_out + size_t(c->k) * S, size_t(c->m) * S, S, 1,
                            raw_out);
}

// ---------------------------------------------------------------- coalesced single blocks
// DagNode.Put hands the engine one block per call (node.go:358-408), from many goroutines at
// once.  Group commit turns those calls into GPU batches without a thread of our own: a
// caller that finds no batch executing becomes the executor, takes every block queued so
// far (optionally waiting coalesce_us for more), runs them as rsmi_encode_batch_host(_crc)
// calls grouped by shard size, and wakes their callers.  Blocks that arrive while a batch
// runs queue up and form the next batch.  A lone caller never waits: its batch is itself.
static int reconstruct_host_impl(rsmi_ctx* c, uint8_t* shards, size_t block_stride, size_t S, size_t nblocks,
                                 const uint8_t* present, const uint8_t* want);

// page-locked staging of the executing batch (only the executor touches it)
static uint8_t* coal_stage(rsmi_ctx* c, size_t need) {
    if (c->h_coal_cap >= need) return c->h_coal;
    if (c->h_coal) (void)hipHostFree(c->h_coal);
    c->h_coal = nullptr;
    c->h_coal_cap = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(&c->h_coal), need, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    c->h_coal_cap = need;
    return c->h_coal;
}

// One group of a coalesced batch: same request key, i.e. same kind and shard size (and,
// for reconstruct, the same survivor pattern and requested rows).
static void run_coalesced_group(rsmi_ctx* c, rsmi_ctx::CoalReq* const* rq, size_t nb) {
    const size_t k = size_t(c->k), m = size_t(c->m), n = k + m;
    const std::string& key = rq[0]->key;
    const size_t S = std::stoull(key.substr(1, key.find(':') - 1));
    uint8_t* h = coal_stage(c, nb * n * S);
    if (!h) {
        for (size_t j = 0; j < nb; j++) rq[j]->rc = RSMI_ERR_DEVICE;
        return;
    }
    if (key[0] == 'E') {
        bool want_raw = false;
        for (size_t j = 0; j < nb; j++) {
            uint8_t* dst = h + j * n * S;
            std::memcpy(dst, rq[j]->block, rq[j]->B);
            std::memset(dst + rq[j]->B, 0, k * S - rq[j]->B);  // Split zero-padding
            want_raw |= rq[j]->raw != nullptr;
        }
        std::vector<uint32_t> raw(want_raw ? nb * n : 0);
        const int rc = encode_host_impl(c, h, n * S, h + k * S, n * S, S, nb, want_raw ? raw.data() : nullptr);
        for (size_t j = 0; j < nb; j++) {
            rq[j]->rc = rc;
            if (rc) continue;
            std::memcpy(rq[j]->out, h + j * n * S, n * S);
            if (rq[j]->raw) std::memcpy(rq[j]->raw, raw.data() + j * n, n * 4);
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

static void run_coalesced(rsmi_ctx* c, std::vector<rsmi_ctx::CoalReq*>& batch) {
    const size_t n = size_t(c->n);
    std::map<std::string, std::vector<rsmi_ctx::CoalReq*>> groups;
    for (auto* r : batch) groups[r->key].push_back(r);
    for (auto& g : groups) {
        const std::string& key = g.first;
        const size_t S = std::stoull(key.substr(1, key.find(':') - 1));
        const size_t chunk = std::max<size_t>(1, (size_t(64) << 20) / (n * S));
        for (size_t j0 = 0; j0 < g.second.size(); j0 += chunk)
            run_coalesced_group(c, g.second.data() + j0, std::min(chunk, g.second.size() - j0));
    }
}

// Queue a request and either wait for the executor or become it (group commit).
static int coalesce(rsmi_ctx* c, rsmi_ctx::CoalReq& req) {
    {
        std::lock_guard<std::mutex> g(c->mu);
        int rc = ensure_device(c);
        if (rc) return rc;
    }
    c->stat_coal_calls++;
    std::unique_lock<std::mutex> lk(c->q_mu);
    c->q_pending.push_back(&req);
    c->q_cv.notify_all();  // an executor waiting out coalesce_us may now have enough
    while (!req.done) {
        if (c->q_executing) {
            c->q_cv.wait(lk);
            continue;
        }
        c->q_executing = true;
        const size_t cap = size_t(c->opt_coalesce_max);
        if (c->opt_coalesce_us > 0 && c->q_pending.size() < cap)
            c->q_cv.wait_for(lk, std::chrono::microseconds(c->opt_coalesce_us),
                             [&] { return c->q_pending.size() >= cap; });
        const size_t take = std::min(cap, c->q_pending.size());
        std::vector<rsmi_ctx::CoalReq*> batch(c->q_pending.begin(), c->q_pending.begin() + take);
        c->q_pending.erase(c->q_pending.begin(), c->q_pending.begin() + take);
        lk.unlock();
        run_coalesced(c, batch);
        c->stat_coal_batches++;
        lk.lock();
        for (auto* r : batch) r->done = true;
        c->q_executing = false;
        c->q_cv.notify_all();
    }
    return req.rc;
}

int rsmi_encode_block_coalesced(rsmi_ctx* c, const uint8_t* block, size_t B, uint8_t* shards_out,
                                uint32_t* raw_out) {
    if (!c) return RSMI_ERR_INVALID_ARG;
    if (B == 0) return RSMI_ERR_SHORT_DATA;
    if (!block || !shards_out) return RSMI_ERR_INVALID_ARG;
    rsmi_ctx::CoalReq req{block, B, shards_out, raw_out, "E" + std::to_string(rsmi_shard_size(B, c->k)) + ":",
                          RSMI_OK, false};
    return coalesce(c, req);
}

int rsmi_reconstruct_coalesced(rsmi_ctx* c, uint8_t* shards, size_t S, const uint8_t* present, int data_only) {
    if (!c || !shards || !present) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    const std::vector<uint8_t> want = want_mask(c, present, data_only);
    int pre = reconstruct_precheck(c, present, want.data());
    if (pre < 0) return -pre;
    if (pre == 1) return RSMI_OK;
    std::string key = "R" + std::to_string(S) + ":";
    for (int i = 0; i < c->n; i++) key.push_back(present[i] ? '1' : '0');
    for (int i = 0; i < c->n; i++) key.push_back(want[i] ? '1' : '0');
    rsmi_ctx::CoalReq req{nullptr, 0, shards, nullptr, std::move(key), RSMI_OK, false};
    return coalesce(c, req);
}

long rsmi_get_stat(const rsmi_ctx* c, const char* key) {
    if (!c || !key) return -1;
    if (!std::strcmp(key, "coalesced_calls")) return long(c->stat_coal_calls.load());
    if (!std::strcmp(key, "coalesced_batches")) return long(c->stat_coal_batches.load());
    return -1;
}

int rsmi_encode_batch_dev_crc(rsmi_ctx* c, const uint8_t* d_data, size_t data_shard_stride, size_t data_block_stride,
                              uint8_t* d_parity, size_t parity_shard_stride, size_t parity_block_stride, size_t S,
                              size_t nblocks, uint32_t* d_raw_out, void* stream) {
    if (!c || !d_data || !d_parity || !d_raw_out) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    if (data_shard_stride < S || parity_shard_stride < S) return RSMI_ERR_INVALID_ARG;
    if (nblocks == 0) return RSMI_OK;
    std::lock_guard<std::mutex> g(c->mu);
    int rc = ensure_device(c);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    std::shared_ptr<Plan> plan;
    if ((rc = encode_plan(c, plan))) return rc;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const size_t k = size_t(c->k), m = size_t(c->m), n = k + m;
    if (S >= 16 && k <= 16)
        return launch_encode_crc(c, *plan, d_data, data_shard_stride, data_block_stride, d_parity, parity_shard_stride,
                                 parity_block_stride, S, nblocks, d_raw_out, st);
    // S < 16 or k > 16: the encode, then the CRC pass over both row sets
    if ((rc = launch_plan(c, *plan, d_data, data_shard_stride, data_block_stride, d_parity, parity_shard_stride,
                          parity_block_stride, S, nblocks, st)))
        return rc;
    HIP_TRY(hipMemsetAsync(d_raw_out, 0, nblocks * n * 4, st));
    if ((rc = launch_crc(c, d_data, data_shard_stride, data_block_stride, uint32_t(k), S, nblocks, d_raw_out, n, st,
                         false)))
        return rc;
    return launch_crc(c, d_parity, parity_shard_stride, parity_block_stride, uint32_t(m), S, nblocks, d_raw_out + k, n,
                      st, false);
}

int rsmi_crc16_rows_dev(rsmi_ctx* c, const uint8_t* d_rows, size_t shard_stride, size_t block_stride, int nrows,
                        size_t S, size_t nblocks, uint32_t* d_raw_out, size_t out_block_stride, void* stream) {
    if (!c || !d_rows || !d_raw_out || nrows < 0 || out_block_stride < size_t(nrows)) return RSMI_ERR_INVALID_ARG;
    if (nrows > 1 && shard_stride < S) return RSMI_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    int rc = ensure_device(c);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    rc = launch_crc(c, d_rows, shard_stride, block_stride, uint32_t(nrows), S, nblocks, d_raw_out, out_block_stride,
                    static_cast<hipStream_t>(stream));
    if (rc) return rc;
    c->last_kernel = "rs_crc16_rows_kernel";
    return hip_status(hipGetLastError());
}

uint16_t rsmi_crc16_ibm(const uint8_t* p, size_t n) { return crc16_checksum(p, n); }

uint16_t rsmi_crc16_entry(const uint8_t* head, size_t head_len, uint32_t raw, size_t data_len) {
    return crc16_entry(head, head_len, raw, data_len);
}

// Small reconstruct calls in place over PCIe (see encode_small): page-locked shards are
// read and rebuilt where they lie; pageable ones are staged (survivor rows in, rebuilt rows
// back).  Caller holds ctx->mu.
static int reconstruct_small(rsmi_ctx* c, const Plan& plan, uint8_t* shards, size_t bs, size_t S, size_t nblocks,
                             const uint8_t* present, const uint8_t* want) {
    const size_t n = size_t(c->n);
    hipStream_t st = c->staging[0].stream;
    uint8_t* dev = host_alias(shards, (nblocks - 1) * bs + n * S);
    size_t dbs = bs;
    uint8_t* hs = nullptr;
    if (!dev) {
        hs = small_stage(c, nblocks * n * S);
        if (!hs) return RSMI_ERR_DEVICE;
        for (size_t b = 0; b < nblocks; b++)
            for (size_t i = 0; i < n; i++)
                if (present[i]) std::memcpy(hs + (b * n + i) * S, shards + b * bs + i * S, S);
        dev = host_alias(hs, nblocks * n * S);
        dbs = n * S;
        if (!dev) return RSMI_ERR_DEVICE;
    }
    int rc = launch_plan(c, plan, dev, S, dbs, dev, S, dbs, S, nblocks, st);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(st));
    if (hs)
        for (size_t b = 0; b < nblocks; b++)
            for (size_t i = 0; i < n; i++)
                if (!present[i] && want[i]) std::memcpy(shards + b * bs + i * S, hs + (b * n + i) * S, S);
    return RSMI_OK;
}

static int reconstruct_host_impl(rsmi_ctx* c, uint8_t* shards, size_t block_stride, size_t S, size_t nblocks,
                                 const uint8_t* present, const uint8_t* want) {
    if (!c || !shards || !present || !want) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    if (block_stride < size_t(c->n) * S) return RSMI_ERR_INVALID_ARG;
    int pre = reconstruct_precheck(c, present, want);
    if (pre < 0) return -pre;
    if (pre == 1 || nblocks == 0) return RSMI_OK;
    std::lock_guard<std::mutex> g(c->mu);
    int rc = ensure_device(c);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    std::shared_ptr<Plan> plan;
    rc = reconstruct_plan(c, present, want, plan);
    if (rc) return rc;
    // zero-copy in place when the shards are page-locked (hostsweep "direct": +8-18% over the
    // pipeline) or the call is small (see encode_host_impl)
    if ((c->opt_zero_copy && host_alias(shards, (nblocks - 1) * block_stride + size_t(c->n) * S)) ||
        nblocks * size_t(c->n) * S <= size_t(c->opt_small_bytes))
        return reconstruct_small(c, *plan, shards, block_stride, S, nblocks, present, want);
    // rows to ship: the k survivors in; the missing rows the plan writes, out
    std::vector<int> in_rows, out_rows;
    for (int i = 0; i < c->n && int(in_rows.size()) < c->k; i++)
        if (present[i]) in_rows.push_back(i);
    for (int i = 0; i < c->n; i++)
        if (!present[i] && want[i]) out_rows.push_back(i);
    const size_t n = size_t(c->n), nr = out_rows.size();
    const size_t Sp = rsmi_recommended_pitch(S);
    const size_t bs = n * Sp;
    const bool d2 = dma_2d_ok(S);
    const size_t chunk = std::max<size_t>(1, (size_t(64) << 20) / bs);
    const int ns = nblocks > chunk ? 3 : 1;
    // odd S: rebuilt rows straight into page-locked host memory (see host_alias)
    uint8_t* zc = c->opt_zero_copy && !d2 ? host_alias(shards, (nblocks - 1) * block_stride + size_t(c->n) * S)
                                          : nullptr;
    // the upload by kernel loads too: only the k rows the plan reads cross PCIe, where the
    // linear copy would ship whole blocks (RS(10,4) 256 KiB batches: 35.5 -> 42.9 GiB/s).
    // One launch per row, so small calls keep the single linear copy (tools/latency.cpp:
    // a 4 KiB block took 59 us this way against 26 us with the copy).
    const uint8_t* zin = nblocks * size_t(c->n) * S >= (size_t(4) << 20) ? zc : nullptr;
    if (!d2 && !zc) {  // pinned landing area for the rebuilt rows, scattered on the host at the end
        const size_t need = nblocks * nr * S;
        if (c->h_stage_cap < need) {
            if (c->h_stage) HIP_TRY(hipHostFree(c->h_stage));
            c->h_stage = nullptr;
            c->h_stage_cap = 0;
            HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->h_stage), need, hipHostMallocDefault));
            c->h_stage_cap = need;
        }
    }
    for (size_t b0 = 0, i = 0; b0 < nblocks; b0 += chunk, i++) {
        Staging& st = c->staging[i % ns];
        const size_t nb = std::min(chunk, nblocks - b0);
        if ((rc = reserve(st.d_in, st.in_cap, nb * bs))) return rc;
        uint8_t* h = shards + b0 * block_stride;
        if (zin) {  // only the k rows the plan reads cross PCIe
            for (int r : in_rows)
                if ((rc = repitch(st.d_in + size_t(r) * Sp, bs, zin + b0 * block_stride + size_t(r) * S, block_stride, S,
                                  nb, st.stream)))
                    return rc;
        } else if (d2) {
            for (int r : in_rows)
                HIP_TRY(hipMemcpy2DAsync(st.d_in + size_t(r) * Sp, bs, h + size_t(r) * S, block_stride, S, nb,
                                         hipMemcpyHostToDevice, st.stream));
        } else {
            // whole blocks move linearly (missing rows ride along as don't-care bytes)
            if ((rc = reserve(st.d_lin, st.lin_cap, nb * n * S))) return rc;
            if (block_stride == n * S)
                HIP_TRY(hipMemcpyAsync(st.d_lin, h, nb * n * S, hipMemcpyHostToDevice, st.stream));
            else
                for (size_t b = 0; b < nb; b++)
                    HIP_TRY(hipMemcpyAsync(st.d_lin + b * n * S, h + b * block_stride, n * S, hipMemcpyHostToDevice,
                                           st.stream));
            if ((rc = repitch(st.d_in, Sp, st.d_lin, S, S, nb * n, st.stream))) return rc;
        }
        if ((rc = launch_plan(c, *plan, st.d_in, Sp, bs, st.d_in, Sp, bs, S, nb, st.stream))) return rc;
        if (zc) {
            for (int r : out_rows)
                if ((rc = repitch(zc + b0 * block_stride + size_t(r) * S, block_stride, st.d_in + size_t(r) * Sp, bs, S,
                                  nb, st.stream)))
                    return rc;
        } else if (d2) {
            for (int r : out_rows)
                HIP_TRY(hipMemcpy2DAsync(h + size_t(r) * S, block_stride, st.d_in + size_t(r) * Sp, bs, S, nb,
                                         hipMemcpyDeviceToHost, st.stream));
        } else {
            // gather rebuilt rows compactly as [row][block][S], then one linear D2H
            for (size_t j = 0; j < nr; j++)
                if ((rc = repitch(st.d_lin + j * nb * S, S, st.d_in + size_t(out_rows[j]) * Sp, bs, S, nb,
                                  st.stream)))
                    return rc;
            HIP_TRY(hipMemcpyAsync(c->h_stage + b0 * nr * S, st.d_lin, nb * nr * S, hipMemcpyDeviceToHost,
                                   st.stream));
        }
    }
    for (int s = 0; s < ns; s++) HIP_TRY(hipStreamSynchronize(c->staging[s].stream));
    if (!d2 && !zc) {
        for (size_t b0 = 0; b0 < nblocks; b0 += chunk) {
            const size_t nb = std::min(chunk, nblocks - b0);
            const uint8_t* hs = c->h_stage + b0 * nr * S;
            for (size_t j = 0; j < nr; j++)
                for (size_t b = 0; b < nb; b++)
                    std::memcpy(shards + (b0 + b) * block_stride + size_t(out_rows[j]) * S, hs + (j * nb + b) * S, S);
        }
    }
    return RSMI_OK;
}

int rsmi_reconstruct_batch_host(rsmi_ctx* c, uint8_t* shards, size_t block_stride, size_t S, size_t nblocks,
                                const uint8_t* present, int data_only) {
    if (!c || !present) return RSMI_ERR_INVALID_ARG;
    const std::vector<uint8_t> w = want_mask(c, present, data_only);
    return reconstruct_host_impl(c, shards, block_stride, S, nblocks, present, w.data());
}

int rsmi_reconstruct_rows_batch_host(rsmi_ctx* c, uint8_t* shards, size_t block_stride, size_t S, size_t nblocks,
                                     const uint8_t* present, const uint8_t* required) {
    return reconstruct_host_impl(c, shards, block_stride, S, nblocks, present, required);
}

}  // extern "C"
