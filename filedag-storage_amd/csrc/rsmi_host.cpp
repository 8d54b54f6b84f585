// rsmi_host.cpp -- host-memory entry points of include/rsmi.h (see rsmi_impl.hpp).
//
// Host-memory calls.  Page-locked buffers of any size, and small pageable calls staged by CPU
// copies, run as one unaligned-window kernel in place over PCIe (encode_small /
// reconstruct_small).  Larger pageable calls take the copy-engine pipeline: chunks of blocks
// round-robin over 3 streams, each with its own device buffers: H2D -> kernel -> D2H.  When S
// is a multiple of 8 the DMA engines move rows straight between the contiguous host layout
// (pitch S) and the pitched device layout with 2-D copies at full PCIe rate.  Odd-width 2-D
// copies crawl (3-9 GB/s measured, tools/copyprobe.py), so for other S the PCIe copies stay
// linear and rs_repitch_kernel re-lays rows out on the device (HBM-speed, ~1% of the PCIe
// time).

#include "rsmi_impl.hpp"
#include <new>

using namespace rsmi;
using namespace rsmi::impl;

namespace rsmi {
namespace impl {

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

// ---------------------------------------------------------------- small host calls
// A per-block call (DagNode.Put / Get, one 256 KiB block) is latency-bound: the copy-engine
// path pays a DMA setup on each side of the kernel.  Small calls instead run ONE kernel that
// reads its input rows from page-locked host memory and writes its output rows back over
// PCIe (the unaligned-window kernels take the Split layout's odd row pitch as is).  Pageable
// callers (Go slices over cgo) are staged through a page-locked buffer by CPU copies.
// Caller holds ctx->mu.
uint8_t* small_stage(rsmi_ctx* c, size_t need) {
    if (c->h_small_cap >= need) return c->h_small;
    if (c->h_small) (void)hipHostFree(c->h_small);
    c->h_small = nullptr;
    c->h_small_cap = 0;
    if (pinned_alloc(reinterpret_cast<void**>(&c->h_small), std::max<size_t>(need, 1 << 20)) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    c->h_small_cap = std::max<size_t>(need, 1 << 20);
    return c->h_small;
}

// Row CRCs (device buffers d16 / d32, sz bytes each, either may be null) to the host: a copy
// kernel per buffer into the context's page-locked read-back area, in stream order, so they
// arrive with the call's own stream synchronisation instead of a blocking hipMemcpy after it (a second
// round trip).  h16 / h32 are where they land; read them after that synchronisation.
// The context's page-locked read-back area, at least `bytes` long (caller holds ctx->mu, and no
// kernel of an earlier call still writes it: every call synchronises before it returns).
uint8_t* raw_area(rsmi_ctx* c, size_t bytes) {
    if (c->h_raw_cap < bytes) {
        if (c->h_raw) (void)hipHostFree(c->h_raw);
        c->h_raw = nullptr;
        c->h_raw_cap = 0;
        const size_t cap = std::max<size_t>(bytes, 64 << 10);
        if (pinned_alloc(reinterpret_cast<void**>(&c->h_raw), cap) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        c->h_raw_cap = cap;
    }
    return c->h_raw;
}

int readback(rsmi_ctx* c, const uint32_t* d16, const uint32_t* d32, size_t sz, hipStream_t st, const uint32_t*& h16,
             const uint32_t*& h32) {
    h16 = h32 = nullptr;
    if (!sz || (!d16 && !d32)) return RSMI_OK;
    if (!raw_area(c, 2 * sz)) return RSMI_ERR_DEVICE;
    uint8_t* dev = host_alias(c->h_raw, 2 * sz);
    if (!dev) return RSMI_ERR_DEVICE;
    int rc;
    if (d16) {
        if ((rc = repitch(dev, sz, reinterpret_cast<const uint8_t*>(d16), sz, sz, 1, st))) return rc;
        h16 = reinterpret_cast<const uint32_t*>(c->h_raw);
    }
    if (d32) {
        if ((rc = repitch(dev + sz, sz, reinterpret_cast<const uint8_t*>(d32), sz, sz, 1, st))) return rc;
        h32 = reinterpret_cast<const uint32_t*>(c->h_raw + sz);
    }
    return RSMI_OK;
}

int encode_small(rsmi_ctx* c, const Plan& plan, const uint8_t* data, size_t dbs, uint8_t* parity, size_t pbs,
                        size_t S, size_t nblocks, uint32_t* raw_out, uint32_t* raw32_out) {
    const size_t k = size_t(c->k), m = size_t(c->m), n = k + m;
    hipStream_t st = c->staging[0].stream;
    const uint8_t* in = host_alias(const_cast<uint8_t*>(data), (nblocks - 1) * dbs + k * S);
    uint8_t* out = host_alias(parity, (nblocks - 1) * pbs + m * S);
    size_t in_bs = dbs, out_bs = pbs;
    // page-locked staging, only the parts needed: [data rows | parity rows | raw CRCs | CRC-32s]
    const bool stage_in = in == nullptr, stage_out = out == nullptr;
    const size_t in_sz = stage_in ? nblocks * k * S : 0, out_sz = stage_out ? nblocks * m * S : 0;
    const size_t raw_sz = raw_out ? nblocks * n * 4 : 0, raw32_sz = raw32_out ? nblocks * n * 4 : 0;
    uint8_t* hs = nullptr;
    if (in_sz + out_sz + raw_sz + raw32_sz) {
        hs = small_stage(c, in_sz + out_sz + raw_sz + raw32_sz);
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
    uint32_t* hraw32 = raw32_out ? reinterpret_cast<uint32_t*>(hs + in_sz + out_sz + raw_sz) : nullptr;
    if (!in || !out) return RSMI_ERR_DEVICE;
    int rc;
    uint32_t seq = 0;
    bool armed = false;
    if (raw_out && S >= 16 && k <= 16 && m <= 4) {
        // fused: the encode folds every row it reads and writes into per-tile CRC records (the
        // shard bytes cross PCIe once), then one wave per block combines them into R(row) and
        // stores it straight into the page-locked staging
        uint32_t* draw = reinterpret_cast<uint32_t*>(host_alias(hraw, raw_sz));
        if (!draw) return RSMI_ERR_DEVICE;
        // one block (a lone DagNode.Put): the table form with a single zero base (in / out stay
        // absolute) and its completion flag, polled below instead of synchronising the stream
        if (nblocks == 1 && !raw32_out && c->opt_coalesce_flag) {
            BlockBases tb;
            tb.b[0] = 0;
            if ((rc = arm_flag(c, st, tb, seq))) return rc;
            rc = launch_plan_crc(c, plan, in, S, in_bs, out, S, out_bs, S, 1, draw, st, &tb, &armed);
            if (rc == RSMI_ERR_INVALID_ARG) rc = launch_encode_crc(c, plan, in, S, in_bs, out, S, out_bs, S, 1, draw, st);
            if (rc) return rc;
        } else if ((rc = launch_encode_crc(c, plan, in, S, in_bs, out, S, out_bs, S, nblocks, draw, st))) {
            return rc;
        }
    } else {
        if ((rc = launch_plan(c, plan, in, S, in_bs, out, S, out_bs, S, nblocks, st))) return rc;
        if (raw_out) {  // S < 16, k > 16 or m > 4: a separate CRC pass over the rows where they lie
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
    if (raw32_out) {  // CRC-32 R(row): a second read of the rows where they lie
        if ((rc = reserve(c->d_crc32, c->crc32_cap, raw32_sz))) return rc;
        uint32_t* cr = reinterpret_cast<uint32_t*>(c->d_crc32);
        HIP_TRY(hipMemsetAsync(cr, 0, raw32_sz, st));
        if ((rc = launch_crc32(c, in, S, in_bs, uint32_t(k), S, nblocks, cr, n, st))) return rc;
        if ((rc = launch_crc32(c, out, S, out_bs, uint32_t(m), S, nblocks, cr + k, n, st))) return rc;
        uint8_t* d32 = host_alias(reinterpret_cast<uint8_t*>(hraw32), raw32_sz);
        if (!d32) return RSMI_ERR_DEVICE;
        if ((rc = repitch(d32, raw32_sz, reinterpret_cast<uint8_t*>(cr), raw32_sz, raw32_sz, 1, st))) return rc;
    }
    // a one-block call (a lone DagNode.Put): the calling thread's wait hook runs while the kernel
    // codes the block (rsmi_set_wait_hook)
    if (nblocks == 1) run_pending_wait_hook();
    if (armed) {
        if ((rc = wait_flag(done_flag(c, seq), seq, st, nullptr))) {
            (void)hipStreamSynchronize(st);
            return rc;
        }
    } else {
        HIP_TRY(hipStreamSynchronize(st));
    }
    if (stage_out)
        for (size_t b = 0; b < nblocks; b++) std::memcpy(parity + b * pbs, hout + b * m * S, m * S);
    if (raw_out) std::memcpy(raw_out, hraw, raw_sz);
    if (raw32_out) std::memcpy(raw32_out, hraw32, raw32_sz);
    return RSMI_OK;
}

// The encode of nblocks blocks whose rows lie at in / out (device addresses: device memory or
// aliases of page-locked host memory), stream-ordered, no synchronisation: R(row) of every row
// into d16[b*n + r] (the CRC fused into the encode where the plan allows it, else a separate
// pass over the rows) and R32(row) into d32, either may be null (device buffers, b*n + r).
int launch_encode_rows(rsmi_ctx* c, const Plan& plan, const uint8_t* in, size_t in_bs, uint8_t* out, size_t out_bs,
                       size_t S, size_t nblocks, uint32_t* d16, uint32_t* d32, hipStream_t st) {
    const size_t k = size_t(c->k), m = size_t(c->m), n = k + m;
    int rc;
    if (d16 && S >= 16 && k <= 16 && m <= 4) {
        if ((rc = launch_encode_crc(c, plan, in, S, in_bs, out, S, out_bs, S, nblocks, d16, st))) return rc;
    } else {
        if ((rc = launch_plan(c, plan, in, S, in_bs, out, S, out_bs, S, nblocks, st))) return rc;
        if (d16) {
            HIP_TRY(hipMemsetAsync(d16, 0, nblocks * n * 4, st));
            if ((rc = launch_crc(c, in, S, in_bs, uint32_t(k), S, nblocks, d16, n, st, false))) return rc;
            if ((rc = launch_crc(c, out, S, out_bs, uint32_t(m), S, nblocks, d16 + k, n, st, false))) return rc;
        }
    }
    if (d32) {
        HIP_TRY(hipMemsetAsync(d32, 0, nblocks * n * 4, st));
        if ((rc = launch_crc32(c, in, S, in_bs, uint32_t(k), S, nblocks, d32, n, st))) return rc;
        if ((rc = launch_crc32(c, out, S, out_bs, uint32_t(m), S, nblocks, d32 + k, n, st))) return rc;
    }
    return RSMI_OK;
}

int encode_host_impl(rsmi_ctx* c, const uint8_t* data, size_t data_block_stride, uint8_t* parity,
                            size_t parity_block_stride, size_t S, size_t nblocks, uint32_t* raw_out, uint32_t* raw32_out) {
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
        return encode_small(c, *plan, data, data_block_stride, parity, parity_block_stride, S, nblocks, raw_out,
                            raw32_out);
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
    if (raw32_out && (rc = reserve(c->d_crc32, c->crc32_cap, nblocks * n * 4))) return rc;
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
        // one chunk (a latency-bound call): the encode with the CRC-16 fused in, one launch plus
        // the combine, instead of the encode and two rows passes.  Several chunks run on three
        // streams; the fused path's record buffer is one per context, so they keep the rows
        // passes (which the PCIe copies hide).
        const bool fused = raw_out && ns == 1 && S >= 16 && k <= 16 && m <= 4;
        if (fused) {
            uint32_t* cr = reinterpret_cast<uint32_t*>(c->d_crc) + b0 * n;
            rc = launch_encode_crc(c, *plan, st.d_in, Sp, in_bs, st.d_out, Sp, out_bs, S, nb, cr, st.stream);
            if (rc) return rc;
        } else if ((rc = launch_plan(c, *plan, st.d_in, Sp, in_bs, st.d_out, Sp, out_bs, S, nb, st.stream))) {
            return rc;
        }
        if (raw_out && !fused) {  // R(shard) of the k data rows and the m parity rows, [block][row]
            uint32_t* cr = reinterpret_cast<uint32_t*>(c->d_crc) + b0 * n;
            HIP_TRY(hipMemsetAsync(cr, 0, nb * n * 4, st.stream));
            if ((rc = launch_crc(c, st.d_in, Sp, in_bs, uint32_t(k), S, nb, cr, n, st.stream, false))) return rc;
            if ((rc = launch_crc(c, st.d_out, Sp, out_bs, uint32_t(m), S, nb, cr + k, n, st.stream, false)))
                return rc;
        }
        if (raw32_out) {
            uint32_t* cr = reinterpret_cast<uint32_t*>(c->d_crc32) + b0 * n;
            HIP_TRY(hipMemsetAsync(cr, 0, nb * n * 4, st.stream));
            if ((rc = launch_crc32(c, st.d_in, Sp, in_bs, uint32_t(k), S, nb, cr, n, st.stream))) return rc;
            if ((rc = launch_crc32(c, st.d_out, Sp, out_bs, uint32_t(m), S, nb, cr + k, n, st.stream))) return rc;
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
    if (raw32_out) HIP_TRY(hipMemcpy(raw32_out, c->d_crc32, nblocks * n * 4, hipMemcpyDeviceToHost));
    return RSMI_OK;
}

// Small reconstruct calls in place over PCIe (see encode_small): page-locked shards are
// read and rebuilt where they lie; pageable ones are staged (survivor rows in, rebuilt rows
// back).  Caller holds ctx->mu.
int reconstruct_small(rsmi_ctx* c, const Plan& plan, uint8_t* shards, size_t bs, size_t S, size_t nblocks,
                             const uint8_t* present, const uint8_t* want, uint32_t* raw16, uint32_t* raw32) {
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
    int rc;
    uint32_t seq = 0;
    bool armed = false;
    if (nblocks == 1 && !raw16 && !raw32 && c->opt_coalesce_flag) {
        // one block, no checksums (a lone repair or degraded read): the table form with a single
        // zero base and its completion flag, polled below instead of synchronising the stream
        BlockBases tb;
        tb.b[0] = 0;
        if ((rc = arm_flag(c, st, tb, seq))) return rc;
        rc = launch_plan(c, plan, dev, S, dbs, dev, S, dbs, S, 1, st, nullptr, &tb, &armed);
        if (rc == RSMI_ERR_INVALID_ARG) rc = launch_plan(c, plan, dev, S, dbs, dev, S, dbs, S, nblocks, st);
    } else {
        rc = launch_plan(c, plan, dev, S, dbs, dev, S, dbs, S, nblocks, st);
    }
    if (rc) return rc;
    const size_t raw_sz = nblocks * n * 4;
    if (raw16 && (rc = reserve(c->d_crc, c->crc_cap, raw_sz))) return rc;
    if (raw32 && (rc = reserve(c->d_crc32, c->crc32_cap, raw_sz))) return rc;
    uint32_t* d16 = raw16 ? reinterpret_cast<uint32_t*>(c->d_crc) : nullptr;
    uint32_t* d32 = raw32 ? reinterpret_cast<uint32_t*>(c->d_crc32) : nullptr;
    if ((raw16 || raw32) && (rc = launch_rebuilt_crcs(c, dev, S, dbs, S, nblocks, present, want, d16, d32, st)))
        return rc;
    const uint32_t *h16, *h32;
    if ((rc = readback(c, d16, d32, raw_sz, st, h16, h32))) return rc;
    // a one-block call (a lone degraded DagNode.Get): the calling thread's wait hook runs while the
    // kernel rebuilds the block (rsmi_set_wait_hook)
    if (nblocks == 1) run_pending_wait_hook();
    if (armed) {
        if ((rc = wait_flag(done_flag(c, seq), seq, st, nullptr))) {
            (void)hipStreamSynchronize(st);
            return rc;
        }
    } else {
        HIP_TRY(hipStreamSynchronize(st));
    }
    if (raw16) std::memcpy(raw16, h16, raw_sz);
    if (raw32) std::memcpy(raw32, h32, raw_sz);
    if (hs)
        for (size_t b = 0; b < nblocks; b++)
            for (size_t i = 0; i < n; i++)
                if (!present[i] && want[i]) std::memcpy(shards + b * bs + i * S, hs + (b * n + i) * S, S);
    return RSMI_OK;
}

int reconstruct_host_impl(rsmi_ctx* c, uint8_t* shards, size_t block_stride, size_t S, size_t nblocks,
                                 const uint8_t* present, const uint8_t* want, uint32_t* raw16, uint32_t* raw32) {
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
        return reconstruct_small(c, *plan, shards, block_stride, S, nblocks, present, want, raw16, raw32);
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
            HIP_TRY(pinned_alloc(reinterpret_cast<void**>(&c->h_stage), need));
            c->h_stage_cap = need;
        }
    }
    if (raw16 && (rc = reserve(c->d_crc, c->crc_cap, nblocks * n * 4))) return rc;
    if (raw32 && (rc = reserve(c->d_crc32, c->crc32_cap, nblocks * n * 4))) return rc;
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
        if ((raw16 || raw32) &&
            (rc = launch_rebuilt_crcs(c, st.d_in, Sp, bs, S, nb, present, want,
                                      raw16 ? reinterpret_cast<uint32_t*>(c->d_crc) + b0 * n : nullptr,
                                      raw32 ? reinterpret_cast<uint32_t*>(c->d_crc32) + b0 * n : nullptr, st.stream)))
            return rc;
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
    if (raw16) HIP_TRY(hipMemcpy(raw16, c->d_crc, nblocks * n * 4, hipMemcpyDeviceToHost));
    if (raw32) HIP_TRY(hipMemcpy(raw32, c->d_crc32, nblocks * n * 4, hipMemcpyDeviceToHost));
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

}  // namespace impl
}  // namespace rsmi

extern "C" {

// ---------------------------------------------------------------- host memory, one block
int rsmi_encode(rsmi_ctx* c, const uint8_t* data, uint8_t* parity, size_t S) try {
    if (!c || !data || !parity) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    return rsmi_encode_batch_host(c, data, size_t(c->k) * S, parity, size_t(c->m) * S, S, 1);
} catch (...) {
    return rsmi::impl::exception_status();
}

int rsmi_encode_block(rsmi_ctx* c, const uint8_t* block, size_t B, uint8_t* shards_out) try {
    if (!c) return RSMI_ERR_INVALID_ARG;
    if (B == 0) return RSMI_ERR_SHORT_DATA;  // upstream Split checks this first
    if (!block || !shards_out) return RSMI_ERR_INVALID_ARG;
    const size_t S = rsmi_shard_size(B, c->k);
    std::memcpy(shards_out, block, B);
    std::memset(shards_out + B, 0, size_t(c->k) * S - B);  // Split zero-padding
    return rsmi_encode(c, shards_out, shards_out + size_t(c->k) * S, S);
} catch (...) {
    return rsmi::impl::exception_status();
}

int rsmi_reconstruct(rsmi_ctx* c, uint8_t* shards, size_t S, const uint8_t* present, int data_only) try {
    if (!c || !shards || !present) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    return rsmi_reconstruct_batch_host(c, shards, size_t(c->n) * S, S, 1, present, data_only);
} catch (...) {
    return rsmi::impl::exception_status();
}

namespace {
// test hook (option "inject_host_fault"): a direct host encode fails as a host allocation would,
// as the coalesced batches do (rsmi_coalesce.cpp)
void direct_fault_hook(rsmi_ctx* c) {
    if (!c) return;
    for (int v = c->opt_inject_host_fault.load(); v > 0;)
        if (c->opt_inject_host_fault.compare_exchange_weak(v, v - 1)) throw std::bad_alloc();
}
}  // namespace

int rsmi_encode_batch_host(rsmi_ctx* c, const uint8_t* data, size_t data_block_stride, uint8_t* parity,
                           size_t parity_block_stride, size_t S, size_t nblocks) try {
    direct_fault_hook(c);
    return encode_host_impl(c, data, data_block_stride, parity, parity_block_stride, S, nblocks, nullptr);
} catch (...) {
    return rsmi::impl::exception_status();
}

int rsmi_encode_batch_host_crc(rsmi_ctx* c, const uint8_t* data, size_t data_block_stride, uint8_t* parity,
                               size_t parity_block_stride, size_t S, size_t nblocks, uint32_t* raw_out) try {
    if (!raw_out) return RSMI_ERR_INVALID_ARG;
    direct_fault_hook(c);
    return encode_host_impl(c, data, data_block_stride, parity, parity_block_stride, S, nblocks, raw_out);
} catch (...) {
    return rsmi::impl::exception_status();
}

int rsmi_encode_batch_host_crcs(rsmi_ctx* c, const uint8_t* data, size_t data_block_stride, uint8_t* parity,
                                size_t parity_block_stride, size_t S, size_t nblocks, uint32_t* raw16_out,
                                uint32_t* raw32_out) try {
    direct_fault_hook(c);
    return encode_host_impl(c, data, data_block_stride, parity, parity_block_stride, S, nblocks, raw16_out,
                            raw32_out);
} catch (...) {
    return rsmi::impl::exception_status();
}

int rsmi_encode_block_crc(rsmi_ctx* c, const uint8_t* block, size_t B, uint8_t* shards_out, uint32_t* raw_out) try {
    if (!c) return RSMI_ERR_INVALID_ARG;
    if (B == 0) return RSMI_ERR_SHORT_DATA;
    if (!block || !shards_out || !raw_out) return RSMI_ERR_INVALID_ARG;
    const size_t S = rsmi_shard_size(B, c->k);
    std::memcpy(shards_out, block, B);
    std::memset(shards_out + B, 0, size_t(c->k) * S - B);  // Split zero-padding
    return encode_host_impl(c, shards_out, size_t(c->k) * S, shards_out + size_t(c->k) * S, size_t(c->m) * S, S, 1,
                            raw_out);
} catch (...) {
    return rsmi::impl::exception_status();
}

int rsmi_reconstruct_batch_host(rsmi_ctx* c, uint8_t* shards, size_t block_stride, size_t S, size_t nblocks,
                                const uint8_t* present, int data_only) try {
    if (!c || !present) return RSMI_ERR_INVALID_ARG;
    const std::vector<uint8_t> w = want_mask(c, present, data_only);
    return reconstruct_host_impl(c, shards, block_stride, S, nblocks, present, w.data());
} catch (...) {
    return rsmi::impl::exception_status();
}

int rsmi_reconstruct_rows_batch_host(rsmi_ctx* c, uint8_t* shards, size_t block_stride, size_t S, size_t nblocks,
                                     const uint8_t* present, const uint8_t* required) try {
    return reconstruct_host_impl(c, shards, block_stride, S, nblocks, present, required);
} catch (...) {
    return rsmi::impl::exception_status();
}

int rsmi_reconstruct_rows_batch_host_crcs(rsmi_ctx* c, uint8_t* shards, size_t block_stride, size_t S,
                                          size_t nblocks, const uint8_t* present, const uint8_t* required,
                                          uint32_t* raw16_out, uint32_t* raw32_out) try {
    if (!c) return RSMI_ERR_INVALID_ARG;
    if (raw16_out) std::memset(raw16_out, 0, nblocks * size_t(c->n) * 4);
    if (raw32_out) std::memset(raw32_out, 0, nblocks * size_t(c->n) * 4);
    return reconstruct_host_impl(c, shards, block_stride, S, nblocks, present, required, raw16_out, raw32_out);
} catch (...) {
    return rsmi::impl::exception_status();
}

int rsmi_reconstruct_batch_host_verify(rsmi_ctx* c, uint8_t* shards, size_t block_stride, size_t S, size_t nblocks,
                                       const uint8_t* present, int data_only, uint32_t* raw16_in) try {
    if (!c || !shards || !present || !raw16_in) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    if (block_stride < size_t(c->n) * S) return RSMI_ERR_INVALID_ARG;
    const size_t k = size_t(c->k), n = size_t(c->n);
    std::vector<int> used;
    for (int i = 0; i < c->n && used.size() < k; i++)
        if (present[i]) used.push_back(i);
    if (used.size() < k) return RSMI_ERR_TOO_FEW_SHARDS;
    if (nblocks == 0) return RSMI_OK;
    const std::vector<uint8_t> want = want_mask(c, present, data_only);
    {
        std::lock_guard<std::mutex> g(c->mu);
        int rc = ensure_device(c);
        if (rc) return rc;
        HIP_TRY(hipSetDevice(c->device));
        uint8_t* dev = host_alias(shards, (nblocks - 1) * block_stride + n * S);
        std::shared_ptr<Plan> plan;
        if (dev && c->opt_zero_copy && reconstruct_precheck(c, present, want.data()) == 0 &&
            (rc = reconstruct_plan(c, present, want.data(), plan)) == RSMI_OK) {
            // one kernel reads every survivor once, in place over PCIe, for both the rebuild and
            // its R(row); the combine lands R of the K inputs and MT outputs per block
            const size_t nsh = size_t(plan->tiles.empty() ? 0 : plan->tiles[0].K + plan->tiles[0].MT);
            if ((rc = reserve(c->d_crc, c->crc_cap, nblocks * nsh * 4))) return rc;
            hipStream_t st = c->staging[0].stream;
            const uint32_t *all = nullptr, *unused;
            uint32_t seq = 0;
            bool armed = false;
            rc = RSMI_ERR_INVALID_ARG;
            if (nblocks == 1 && c->opt_coalesce_flag) {
                // one block (a lone degraded read): the table form with a single zero base, R(row)
                // stored straight into the page-locked area by the in-kernel combine, and the
                // completion flag polled below instead of a read-back kernel and a synchronisation
                uint8_t* h = raw_area(c, nsh * 4);
                uint32_t* hd = h ? reinterpret_cast<uint32_t*>(host_alias(h, nsh * 4)) : nullptr;
                BlockBases tb;
                tb.b[0] = 0;
                if (hd && (rc = arm_flag(c, st, tb, seq)) == RSMI_OK)
                    rc = launch_plan_crc(c, *plan, dev, S, block_stride, dev, S, block_stride, S, 1, hd, st, &tb, &armed);
                else if (!hd)
                    rc = RSMI_ERR_INVALID_ARG;
                if (rc == RSMI_OK && !armed) rc = hip_status(hipStreamSynchronize(st));  // R landed by a second launch
                if (rc == RSMI_OK) all = reinterpret_cast<const uint32_t*>(h);
            }
            if (rc == RSMI_ERR_INVALID_ARG && !armed) {
                uint32_t* d = reinterpret_cast<uint32_t*>(c->d_crc);
                rc = launch_plan_crc(c, *plan, dev, S, block_stride, dev, S, block_stride, S, nblocks, d, st);
                if (rc == RSMI_OK) rc = readback(c, d, nullptr, nblocks * nsh * 4, st, all, unused);
            }
            if (rc == RSMI_OK) {
                if (armed) {
                    if ((rc = wait_flag(done_flag(c, seq), seq, st, nullptr))) {
                        (void)hipStreamSynchronize(st);
                        return rc;
                    }
                } else {
                    HIP_TRY(hipStreamSynchronize(st));
                }
                for (size_t b = 0; b < nblocks; b++)
                    std::memcpy(raw16_in + b * k, all + b * nsh, k * 4);
                return RSMI_OK;
            }
            if (rc != RSMI_ERR_INVALID_ARG) return rc;
        }
    }
    // any other layout or plan: the rebuild, then a CRC pass over each survivor row
    int rc = rsmi_reconstruct_batch_host(c, shards, block_stride, S, nblocks, present, data_only);
    if (rc) return rc;
    std::vector<uint32_t> r(nblocks);
    for (size_t j = 0; j < k; j++) {
        if ((rc = rsmi_crc_rows_host(c, shards + size_t(used[j]) * S, block_stride, nblocks, S, r.data(), nullptr)))
            return rc;
        for (size_t b = 0; b < nblocks; b++) raw16_in[b * k + j] = r[b];
    }
    return RSMI_OK;
} catch (...) {
    return rsmi::impl::exception_status();
}

}  // extern "C"
