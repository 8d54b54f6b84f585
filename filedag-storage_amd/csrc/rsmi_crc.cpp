// rsmi_crc.cpp -- the datanode entry checksum (dag/node/datanode/server.go:58-75) on the GPU:
// the R(row) pass, the encode with the CRC fused in, and the host-side header fold
// (crc16.hpp has the algebra; rsmi_impl.hpp the file map); and the mutcask value checksum
// (CRC-32 IEEE, kv/mutcask/cask.go:73-97; crc32.hpp) as an R(row) pass.
#include "rsmi_impl.hpp"

using namespace rsmi;
using namespace rsmi::impl;

namespace rsmi {
namespace impl {

// CRC-16 device tables, uploaded once per context (caller holds ctx->mu)
int ensure_crc_tables(rsmi_ctx* c) {
    if (c->d_crc_tbl) return RSMI_OK;
    const Crc16Tables& t = crc16_tables();
    static_assert(sizeof(t.P) + sizeof(t.N) + sizeof(t.Q) + sizeof(t.G) + sizeof(t.P4) + sizeof(t.MW) +
                          sizeof(t.FW) ==
                      size_t(kCrcTableWords) * 4,
                  "CRC table layout");
    std::vector<uint16_t> h(size_t(kCrcTableWords) * 2);
    std::memcpy(h.data(), t.P, sizeof(t.P));
    std::memcpy(h.data() + kCrcPWords * 2, t.N, sizeof(t.N));
    std::memcpy(h.data() + kCrcQOff * 2, t.Q, sizeof(t.Q));
    std::memcpy(h.data() + kCrcGOff * 2, t.G, sizeof(t.G));
    std::memcpy(h.data() + kCrcP4Off * 2, t.P4, sizeof(t.P4));
    std::memcpy(h.data() + kCrcMWOff * 2, t.MW, sizeof(t.MW));
    std::memcpy(h.data() + kCrcFWOff * 2, t.FW, sizeof(t.FW));
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&c->d_crc_tbl), h.size() * 2));
    HIP_TRY(hipMemcpy(c->d_crc_tbl, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    return RSMI_OK;
}

// R(row) of nrows rows per block into out[b*out_bs + r] (zeroed first), stream-ordered.
int launch_crc(rsmi_ctx* c, const uint8_t* base, uint64_t rpitch, uint64_t bstride, uint32_t nrows, uint64_t S,
               uint64_t nblocks, uint32_t* out, uint64_t out_bs, hipStream_t stream, bool zero) {
    if (!nblocks || !nrows) return RSMI_OK;
    int rc = ensure_crc_tables(c);
    if (rc) return rc;
    if (zero) HIP_TRY(hipMemset2DAsync(out, out_bs * 4, 0, size_t(nrows) * 4, nblocks, stream));
    if (S == 0) return RSMI_OK;  // R(empty) = 0
    const bool aligned = reinterpret_cast<uintptr_t>(base) % 16 == 0 && rpitch % 16 == 0 && bstride % 16 == 0;
    // the fold on the matrix cores for any layout (unaligned rows: aligned loads funnel-shifted),
    // option crc16_fold 0: the nibble-table passes
    void* fn = c->opt_crc16_fold == 1 ? crc16_rows_mfma_kernel(aligned) : crc16_rows_kernel(aligned);
    const uint64_t tile = uint64_t(kWave) * 16;
    // the matrix-core pass folds unaligned rows on the memory's 16-byte grid, where a row spans
    // its misalignment (< 16) + S bytes
    const uint64_t span = S + (c->opt_crc16_fold == 1 && !aligned ? 15 : 0);
    uint32_t tpb = uint32_t((span + tile - 1) / tile);
    constexpr uint32_t kSup = kCrcSupGroups * kCrcSegTiles;
    uint32_t nsup = (tpb + kSup - 1) / kSup;
    uint64_t nitems = nblocks * nrows * nsup;
    // A^E, E = S - (end of the last item, counted in whole 8-tile groups), mod 32767
    const uint64_t last_end = (uint64_t(tpb) + kCrcSegTiles - 1) / kCrcSegTiles * kCrcSegTiles * tile;
    const int64_t E = ((int64_t(S) - int64_t(last_end)) % int64_t(kCrcOrder) + kCrcOrder) % kCrcOrder;
    Crc16Shift sh;
    for (int b = 0; b < 16; b++) sh.col[b] = crc16_tables().shift(uint16_t(1u << b), uint64_t(E));
    // 96 waves per CU: several dispatch rounds, so the hardware balances CUs (items differ in
    // length at a row's end), while each workgroup still amortizes its LDS table staging over
    // a few items per wave.  Level with 48 and 64 at 26 KB rows, +10 % at 256 KB rows
    // (profiles/r02/crc/crc_rows_grid.txt).
    uint64_t cap = uint64_t(c->num_cu) * 96 / 4;
    if (c->opt_waves_per_cu > 0) cap = std::max<uint64_t>(1, uint64_t(c->num_cu) * uint64_t(c->opt_waves_per_cu) / 4);
    const uint64_t wgs = std::min<uint64_t>((nitems + 3) / 4, cap);
    const uint32_t* tb = c->d_crc_tbl;
    void* args[] = {&tb, &base, &bstride, &rpitch, &nrows, &S, &tpb, &nsup, &nitems, &out, &out_bs, &sh};
    HIP_TRY(hipLaunchKernel(fn, dim3(uint32_t(wgs)), dim3(kWG), args, 0, stream));
    return RSMI_OK;
}

// CRC-32 device tables (crc32.hpp), uploaded once per context (caller holds ctx->mu)
int ensure_crc32_tables(rsmi_ctx* c) {
    if (c->d_crc32_tbl) return RSMI_OK;
    const Crc32Tables& t = crc32_tables();
    static_assert(sizeof(t.NT) + sizeof(t.SN) + sizeof(t.SG) + sizeof(t.SC) + sizeof(t.MW) + sizeof(t.SG4) ==
                      size_t(kCrc32TableWords) * 4,
                  "CRC-32 table layout");
    static_assert(sizeof(t.MW) == size_t(kCrc32MWWords) * 4, "CRC-32 MFMA weights");
    std::vector<uint32_t> h(static_cast<size_t>(kCrc32TableWords));
    std::memcpy(h.data(), t.NT, sizeof(t.NT));
    std::memcpy(h.data() + kCrc32FoldWords, t.SN, sizeof(t.SN));
    std::memcpy(h.data() + kCrc32FoldWords + 6 * kCrc32PowWords, t.SG, sizeof(t.SG));
    std::memcpy(h.data() + kCrc32LdsWords, t.SC, sizeof(t.SC));
    std::memcpy(h.data() + kCrc32MWOff, t.MW, sizeof(t.MW));
    std::memcpy(h.data() + kCrc32SG4Off, t.SG4, sizeof(t.SG4));
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&c->d_crc32_tbl), h.size() * 4));
    HIP_TRY(hipMemcpy(c->d_crc32_tbl, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    return RSMI_OK;
}

// CRC-32 R(row) of nrows rows per block, XORed into out[b*out_bs + r] (the caller zeroes
// it), stream-ordered.  Rows may lie in device or page-locked host memory.

int launch_crc32(rsmi_ctx* c, const uint8_t* base, uint64_t rpitch, uint64_t bstride, uint32_t nrows, uint64_t S,
                 uint64_t nblocks, uint32_t* out, uint64_t out_bs, hipStream_t stream) {
    if (!nblocks || !nrows || S == 0) return RSMI_OK;  // R(empty) = 0
    int rc = ensure_crc32_tables(c);
    if (rc) return rc;
    const bool aligned = reinterpret_cast<uintptr_t>(base) % 16 == 0 && rpitch % 16 == 0 && bstride % 16 == 0;
    const bool mfma = c->opt_crc32_fold == 1;
    void* fn = mfma ? crc32_rows_mfma_kernel(aligned) : crc32_rows_kernel(aligned);
    const uint64_t tile = uint64_t(kWave) * 16, span = tile * kCrc32SegTiles;
    if (S / span >= (uint64_t(1) << kCrc32SegPowers)) return RSMI_ERR_INVALID_ARG;  // rows below 4 GiB
    // unaligned rows fold on the memory's 16-byte grid, where a row spans its misalignment + S bytes
    uint32_t tpb = uint32_t((S + (aligned ? 0 : 15) + tile - 1) / tile);
    uint32_t nseg = (tpb + kCrc32SegTiles - 1) / kCrc32SegTiles;
    uint32_t nsup = (nseg + kCrc32SupGroups - 1) / kCrc32SupGroups;
    // the per-launch shift to the row's end (crc32.hpp), cached for the last S
    if (c->crc32_shift_S != S) {
        crc32_tables().shift_columns(S % span, c->crc32_shift.col);
        c->crc32_shift_S = S;
    }
    Crc32Shift sh = c->crc32_shift;
    uint64_t nitems = nblocks * nrows * nsup;
    // 96 waves per CU as for the CRC-16 pass
    // (the matrix-core pass: workgroups of 8 waves, 2 resident per CU by its 66 KiB of LDS, each
    // staging the 64 KiB of weights: 48 waves per CU, three rounds, measured best of 16-96,
    // profiles/r03/crc/crc32_mfma_wpc.txt)
    const uint64_t wpg = mfma ? uint64_t(kCrc32MfmaWG) / kWave : 4;
    uint64_t cap = uint64_t(c->num_cu) * (mfma && !kCrc32MfmaHalf ? 48 : 96) / wpg;
    if (c->opt_waves_per_cu > 0) cap = std::max<uint64_t>(1, uint64_t(c->num_cu) * uint64_t(c->opt_waves_per_cu) / wpg);
    const uint64_t wgs = std::min<uint64_t>((nitems + wpg - 1) / wpg, cap);
    const uint32_t* tb = c->d_crc32_tbl;
    void* args[] = {&tb, &base, &bstride, &rpitch, &nrows, &S, &tpb, &nseg, &nsup, &nitems, &out, &out_bs, &sh};
    HIP_TRY(hipLaunchKernel(fn, dim3(uint32_t(wgs)), dim3(uint32_t(wpg * kWave)), args, 0, stream));
    return RSMI_OK;
}

int launch_rebuilt_crcs(rsmi_ctx* c, const uint8_t* base, uint64_t rpitch, uint64_t bstride, uint64_t S,
                        uint64_t nblocks, const uint8_t* present, const uint8_t* want, uint32_t* d16, uint32_t* d32,
                        hipStream_t stream) {
    const uint64_t n = uint64_t(c->n);
    if (d16) HIP_TRY(hipMemsetAsync(d16, 0, nblocks * n * 4, stream));
    if (d32) HIP_TRY(hipMemsetAsync(d32, 0, nblocks * n * 4, stream));
    int rc;
    for (uint64_t r = 0; r < n; r++) {
        if (present[r] || !want[r]) continue;
        const uint8_t* row = base + r * rpitch;
        if (d16 && (rc = launch_crc(c, row, rpitch, bstride, 1, S, nblocks, d16 + r, n, stream, false))) return rc;
        if (d32 && (rc = launch_crc32(c, row, rpitch, bstride, 1, S, nblocks, d32 + r, n, stream))) return rc;
    }
    return RSMI_OK;
}

// Any single-tile plan with the CRC-16 fused in (rs_fast_kernel CRC variants), then R(row) of
// its K input rows and MT output rows into raw[b * (K + MT) + r] (input row c at r = c, output
// row j at r = K + j; device or page-locked host memory).  Needs K <= 16, one plan tile
// (MT <= 4) and either an aligned layout or S >= 16; returns RSMI_ERR_INVALID_ARG otherwise
// (callers then run the separate pass).
int launch_plan_crc(rsmi_ctx* c, const Plan& plan, const uint8_t* in, size_t in_rs, size_t in_bs, uint8_t* out,
                    size_t out_rs, size_t out_bs, size_t S, size_t nblocks, uint32_t* raw, hipStream_t st,
                    const BlockBases* tb, bool* armed) {
    if (armed) *armed = false;
    if (plan.tiles.size() != 1 || plan.tiles[0].K > 16) return RSMI_ERR_INVALID_ARG;
    // tb: a table of block bases (in / out are offsets from each), one launch of at most
    // kTableBlocks blocks on the matrix-core fold; callers fall back to a launch per block
    if (tb && (nblocks > size_t(kTableBlocks) || c->opt_fused_fold != 1)) return RSMI_ERR_INVALID_ARG;
    const DevTile& tile = plan.tiles[0];
    const size_t nsh = size_t(tile.K + tile.MT);
    const size_t cpb = (S + 15) / 16, tpb = (cpb + kWave - 1) / kWave;
    int rc;
    if ((rc = ensure_crc_tables(c))) return rc;
    const uintptr_t tba = table_alignment(tb, nblocks);
    const bool aligned = (reinterpret_cast<uintptr_t>(in) | tba) % 16 == 0 &&
                         (reinterpret_cast<uintptr_t>(out) | tba) % 16 == 0 && in_rs % 16 == 0 && in_bs % 16 == 0 &&
                         out_rs % 16 == 0 && out_bs % 16 == 0 && in_rs >= round_up(S, 16) && out_rs >= round_up(S, 16) &&
                         S < (size_t(1) << 31);
    // unaligned-window layouts (the Split layout, page-locked host rows at pitch S): S >= 16
    const bool ua = !aligned && S >= 16 && S < (size_t(1) << 31) && in_rs >= S && out_rs >= S;
    const FastKernelTable& kt = fast_kernels();
    void* mfma_fn = aligned ? (tb ? kt.fused_tb : kt.fused)[tile.K][tile.MT]
                            : ua ? (tb ? kt.fused_ua_tb : kt.fused_ua)[tile.K][tile.MT] : nullptr;
    // some table shapes exist only in the in-kernel-combine form (a lone verified reconstruct)
    void* tb_inl = !tb ? nullptr : aligned ? kt.fused_inl_tb[tile.K][tile.MT] : ua ? kt.fused_ua_inl_tb[tile.K][tile.MT] : nullptr;
    if (tb && !mfma_fn && !tb_inl) return RSMI_ERR_INVALID_ARG;
    if ((mfma_fn || tb_inl) && c->opt_fused_fold == 1) {
        // the fold on the matrix cores (rs_fused_mfma_kernel): a unit of 4 tiles per workgroup,
        // then the records' combine
        const size_t upb = (tpb + kFusedUnitTiles - 1) / kFusedUnitTiles;
        const size_t nacc = (nsh + 1) / 2;  // two-shard accumulators: a record byte per lane each
        const size_t rec_per_block = upb * nacc * kWave;
        CrcScratch& sc = crc_scratch(c, st);
        if ((rc = reserve_on(sc.d_chunks, sc.chunks_cap, nblocks * rec_per_block, st))) return rc;
        uint8_t* rec = sc.d_chunks;
        void* fn = mfma_fn;
        const RsPlanDev* pd = tile.dev;
        uint32_t S32 = uint32_t(S), cpb32 = uint32_t(cpb), tpb32 = uint32_t(tpb), upb32 = uint32_t(upb);
        const uint32_t* ctb = c->d_crc_tbl;
        uint64_t ibs = in_bs, irs = in_rs, obs = out_bs, ors = out_rs;
        // A^e moves a row's value from the end of its last unit to the row's end
        const int64_t unit_bytes = int64_t(kFusedUnitTiles) * kWave * 16;
        const uint64_t e = uint64_t(((int64_t(S) - int64_t(upb) * unit_bytes) % int64_t(kCrcOrder) + kCrcOrder) % kCrcOrder);
        Crc16Shift sh;
        for (int b = 0; b < 16; b++) sh.col[b] = crc16_tables().shift(uint16_t(1u << b), e);
        // a launch of a few units (the per-block calls of DagNode.Put) combines in the kernel: one
        // launch instead of two; big ones keep the separate combine (rs_fused_mfma_kernel INL)
        void* inl_fn = aligned ? (tb ? kt.fused_inl_tb : kt.fused_inl)[tile.K][tile.MT]
                               : (tb ? kt.fused_ua_inl_tb : kt.fused_ua_inl)[tile.K][tile.MT];
        const bool inline_combine = RSMI_FUSED_COOP && inl_fn && nblocks * upb <= kFusedInlineUnits;
        if (inline_combine) fn = inl_fn;
        if (!fn) return RSMI_ERR_INVALID_ARG;  // a table shape without the two-launch form, too big to combine inside
        // per-block unit counters of the inline combine: zeroed once when allocated, and every
        // launch leaves them at zero again (atomicInc wraps at the block's last unit)
        if (inline_combine && sc.fctr_cap < nblocks) {
            if (sc.d_fctr) {
                HIP_TRY(hipStreamSynchronize(st));  // the last launch on this stream may still count
                HIP_TRY(hipFree(sc.d_fctr));
            }
            sc.d_fctr = nullptr;
            sc.fctr_cap = 0;
            HIP_TRY(hipMalloc(reinterpret_cast<void**>(&sc.d_fctr), nblocks * 4));
            HIP_TRY(hipMemsetAsync(sc.d_fctr, 0, nblocks * 4, st));
            sc.fctr_cap = nblocks;
        }
        // launches of at most 2^31 units (32-bit unit index)
        const uint64_t max_blocks = std::max<uint64_t>(1, (uint64_t(1) << 31) / upb);
        for (uint64_t b0 = 0; b0 < nblocks; b0 += max_blocks) {
            const uint64_t nb = std::min<uint64_t>(max_blocks, nblocks - b0);
            uint32_t nunits = uint32_t(nb * upb);
            const uint8_t* inb = in + b0 * in_bs;
            uint8_t* outb = out + b0 * out_bs;
            uint8_t* rb = rec + b0 * rec_per_block;
            uint32_t* cb = inline_combine ? sc.d_fctr + b0 : nullptr;
            uint32_t* rw = raw + b0 * nsh;
            NoBases nob;
            // a table's completion flag is armed only when this one launch is the whole job (the
            // combine inside): a separate combine launch would still be writing R after it
            BlockBases tbl_args;
            if (tb) {
                tbl_args = *tb;
                if (!inline_combine || nblocks > max_blocks) tbl_args.done_flag = nullptr;
                if (armed) *armed = tbl_args.done_flag != nullptr;
            }
            void* bases = tb ? static_cast<void*>(&tbl_args) : static_cast<void*>(&nob);
            void* args[] = {&pd,    &inb,   &outb,   &ibs, &irs, &obs, &ors, &S32, &cpb32,
                            &tpb32, &upb32, &nunits, &ctb, &rb,  &cb,  &rw,  &sh,  bases};
            const uint32_t wgs = RSMI_FUSED_COOP ? nunits : (nunits + kWG / kWave - 1) / (kWG / kWave);
            HIP_TRY(hipLaunchKernel(fn, dim3(wgs), dim3(kWG), args, 0, st));
        }
        if (!inline_combine) {
            uint32_t nacc32 = uint32_t(nacc), nsh32 = uint32_t(nsh);
            uint64_t nb64 = nblocks;
            const uint8_t* crec = rec;
            void* cargs[] = {&ctb, &crec, &upb32, &nacc32, &nsh32, &sh, &nb64, &raw};
            // a persistent grid of up to 8 workgroups per CU, 4 waves each, over (block, 4-row group) items
            const uint64_t items = nblocks * ((nsh + 3) / 4);
#ifndef RSMI_COMBINE_WGS_PER_CU
#define RSMI_COMBINE_WGS_PER_CU 8
#endif
            const uint32_t grid = uint32_t(std::max<uint64_t>(
                1, std::min<uint64_t>((items + 3) / 4, uint64_t(c->num_cu) * RSMI_COMBINE_WGS_PER_CU)));
            HIP_TRY(hipLaunchKernel(crc16_combine_mfma_kernel(), dim3(grid), dim3(kWG), cargs, 0, st));
        }
        char buf[96];
        std::snprintf(buf, sizeof buf, "rs_fused_mfma_kernel<K=%d,MT=%d,NT=%d>%s%s%s", tile.K, tile.MT,
                      auto_cache_policy(tile.K, tile.MT), aligned ? "" : ",UA", inline_combine ? ",INL" : "",
                      tb ? ",TB" : "");
        set_last_kernel(c, buf);
        return hip_status(hipGetLastError());
    }
    const size_t ns2 = ((nsh + 3) / 4 + 1) / 2;
    const size_t rec_bytes = nblocks * tpb * ns2 * kWave * 4, tail_bytes = nblocks * nsh * 4;
    CrcScratch& sc = crc_scratch(c, st);
    if ((rc = reserve_on(sc.d_chunks, sc.chunks_cap, rec_bytes + tail_bytes, st))) return rc;
    if (!aligned && S < 16) return RSMI_ERR_INVALID_ARG;
    CrcFuse fz;
    fz.tbl = c->d_crc_tbl;
    fz.rec = reinterpret_cast<uint32_t*>(sc.d_chunks);
    fz.tail = aligned ? nullptr : reinterpret_cast<uint32_t*>(sc.d_chunks + rec_bytes);
    if ((rc = launch_plan(c, plan, in, in_rs, in_bs, out, out_rs, out_bs, S, nblocks, st, &fz))) return rc;
    const uint32_t* ctb = c->d_crc_tbl;
    const uint32_t* rec = fz.rec;
    const uint32_t* tail = fz.tail;
    uint32_t tpb32 = uint32_t(tpb), nsh32 = uint32_t(nsh);
    uint64_t S64 = S, nb64 = nblocks;
    void* args[] = {&ctb, &rec, &tail, &tpb32, &nsh32, &S64, &nb64, &raw};
    // one wave per block, a persistent grid of up to 8 workgroups per CU (the nibble-sliced
    // power tables take 1.9 KiB of LDS per workgroup)
    const uint32_t grid = uint32_t(std::max<uint64_t>(1, std::min<uint64_t>((nblocks + 3) / 4, uint64_t(c->num_cu) * 8)));
    void* fn = crc16_combine_kernel(int(ns2));
    if (!fn) return RSMI_ERR_INVALID_ARG;
    HIP_TRY(hipLaunchKernel(fn, dim3(grid), dim3(kWG), args, 0, st));
    return RSMI_OK;
}

// Encode with the CRC-16 fused in: raw[b * (k+m) + row] = R(row) of all k+m rows.
int launch_encode_crc(rsmi_ctx* c, const Plan& plan, const uint8_t* in, size_t in_rs, size_t in_bs, uint8_t* out,
                      size_t out_rs, size_t out_bs, size_t S, size_t nblocks, uint32_t* raw, hipStream_t st) {
    return launch_plan_crc(c, plan, in, in_rs, in_bs, out, out_rs, out_bs, S, nblocks, raw, st);
}

}  // namespace impl
}  // namespace rsmi

extern "C" {

int rsmi_encode_batch_dev_crc(rsmi_ctx* c, const uint8_t* d_data, size_t data_shard_stride, size_t data_block_stride,
                              uint8_t* d_parity, size_t parity_shard_stride, size_t parity_block_stride, size_t S,
                              size_t nblocks, uint32_t* d_raw_out, void* stream) try {
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
    rc = launch_encode_crc(c, *plan, d_data, data_shard_stride, data_block_stride, d_parity, parity_shard_stride,
                           parity_block_stride, S, nblocks, d_raw_out, st);
    if (rc != RSMI_ERR_INVALID_ARG) return rc;
    // k > 16, m > 4, or S < 16 in an unaligned layout: the encode, then the CRC pass over both
    // row sets
    if ((rc = launch_plan(c, *plan, d_data, data_shard_stride, data_block_stride, d_parity, parity_shard_stride,
                          parity_block_stride, S, nblocks, st)))
        return rc;
    HIP_TRY(hipMemsetAsync(d_raw_out, 0, nblocks * n * 4, st));
    if ((rc = launch_crc(c, d_data, data_shard_stride, data_block_stride, uint32_t(k), S, nblocks, d_raw_out, n, st,
                         false)))
        return rc;
    return launch_crc(c, d_parity, parity_shard_stride, parity_block_stride, uint32_t(m), S, nblocks, d_raw_out + k, n,
                      st, false);
} catch (...) {
    return rsmi::impl::exception_status();
}

int rsmi_crc16_rows_dev(rsmi_ctx* c, const uint8_t* d_rows, size_t shard_stride, size_t block_stride, int nrows,
                        size_t S, size_t nblocks, uint32_t* d_raw_out, size_t out_block_stride, void* stream) try {
    if (!c || !d_rows || !d_raw_out || nrows < 0 || out_block_stride < size_t(nrows)) return RSMI_ERR_INVALID_ARG;
    if (nrows > 1 && shard_stride < S) return RSMI_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    int rc = ensure_device(c);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    rc = launch_crc(c, d_rows, shard_stride, block_stride, uint32_t(nrows), S, nblocks, d_raw_out, out_block_stride,
                    static_cast<hipStream_t>(stream));
    if (rc) return rc;
    const bool aligned = reinterpret_cast<uintptr_t>(d_rows) % 16 == 0 && shard_stride % 16 == 0 && block_stride % 16 == 0;
    set_last_kernel(c, c->opt_crc16_fold == 1 ? (aligned ? "rs_crc16_rows_kernel,MFMA" : "rs_crc16_rows_kernel,MFMA,UA")
                                              : "rs_crc16_rows_kernel");
    return hip_status(hipGetLastError());
} catch (...) {
    return rsmi::impl::exception_status();
}

int rsmi_crc32_rows_dev(rsmi_ctx* c, const uint8_t* d_rows, size_t shard_stride, size_t block_stride, int nrows,
                        size_t S, size_t nblocks, uint32_t* d_raw_out, size_t out_block_stride, void* stream) try {
    if (!c || !d_rows || !d_raw_out || nrows < 0 || out_block_stride < size_t(nrows)) return RSMI_ERR_INVALID_ARG;
    if (nrows > 1 && shard_stride < S) return RSMI_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    int rc = ensure_device(c);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (nblocks && nrows)
        HIP_TRY(hipMemset2DAsync(d_raw_out, out_block_stride * 4, 0, size_t(nrows) * 4, nblocks, st));
    rc = launch_crc32(c, d_rows, shard_stride, block_stride, uint32_t(nrows), S, nblocks, d_raw_out, out_block_stride,
                      st);
    if (rc) return rc;
    set_last_kernel(c, c->opt_crc32_fold == 1 ? "rs_crc32_rows_kernel,MFMA" : "rs_crc32_rows_kernel");
    return hip_status(hipGetLastError());
} catch (...) {
    return rsmi::impl::exception_status();
}

int rsmi_crc_rows_host(rsmi_ctx* c, const uint8_t* rows, size_t row_stride, size_t nrows, size_t S,
                       uint32_t* raw16_out, uint32_t* raw32_out) try {
    if (!c || !rows || (!raw16_out && !raw32_out) || (nrows > 1 && row_stride < S)) return RSMI_ERR_INVALID_ARG;
    if (nrows == 0) return RSMI_OK;
    std::lock_guard<std::mutex> g(c->mu);
    int rc = ensure_device(c);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t st = c->staging[0].stream;
    // page-locked rows are read in place over PCIe; pageable ones through the small-call staging
    const uint8_t* dev = host_alias(const_cast<uint8_t*>(rows), (nrows - 1) * row_stride + S);
    size_t stride = row_stride;
    if (!dev) {
        uint8_t* hs = small_stage(c, nrows * S);
        if (!hs) return RSMI_ERR_DEVICE;
        for (size_t r = 0; r < nrows; r++) std::memcpy(hs + r * S, rows + r * row_stride, S);
        dev = host_alias(hs, nrows * S);
        stride = S;
        if (!dev) return RSMI_ERR_DEVICE;
    }
    const size_t sz = nrows * 4;
    if (raw16_out) {
        if ((rc = reserve(c->d_crc, c->crc_cap, sz))) return rc;
        if ((rc = launch_crc(c, dev, stride, stride, 1, S, nrows, reinterpret_cast<uint32_t*>(c->d_crc), 1, st))) return rc;
    }
    if (raw32_out) {
        if ((rc = reserve(c->d_crc32, c->crc32_cap, sz))) return rc;
        HIP_TRY(hipMemsetAsync(c->d_crc32, 0, sz, st));
        if ((rc = launch_crc32(c, dev, stride, stride, 1, S, nrows, reinterpret_cast<uint32_t*>(c->d_crc32), 1, st)))
            return rc;
    }
    const uint32_t *h16, *h32;
    if ((rc = readback(c, raw16_out ? reinterpret_cast<const uint32_t*>(c->d_crc) : nullptr,
                       raw32_out ? reinterpret_cast<const uint32_t*>(c->d_crc32) : nullptr, sz, st, h16, h32)))
        return rc;
    HIP_TRY(hipStreamSynchronize(st));
    if (raw16_out) std::memcpy(raw16_out, h16, sz);
    if (raw32_out) std::memcpy(raw32_out, h32, sz);
    return RSMI_OK;
} catch (...) {
    return rsmi::impl::exception_status();
}

}  // extern "C"
