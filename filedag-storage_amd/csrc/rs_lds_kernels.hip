// rs_lds_kernels.hip -- the coding kernel with its input rows staged by LDS-DMA.
//
// Same arithmetic and layout contract as rs_fast_kernel (rs_kernels.hip: aligned rows, a
// wave owns a tile of 64 x 16-byte chunks of one block, D = 1), different streaming.  The
// register-ring kernel keeps at most its ring's 6 rows in flight while a wave computes, and
// drains it at the end of every tile.  Here every wave owns K row slots of 1 KiB in LDS:
// as soon as row c of the current tile has been read out of its slot, the wave refills that
// slot with row c of its next tile by global_load_lds_dwordx4 (HBM -> LDS, no VGPRs held),
// so about K rows stay in flight through the whole tile and across tile boundaries.
//
// Waits.  Vector memory operations of a wave retire in issue order (loads, LDS-DMA loads and
// stores alike), so "row r of this tile has landed" is `s_waitcnt vmcnt(n)` with n = the
// number of vector memory instructions issued after it.  When row r is waited for, those are
// rows r+1..K-1 of this tile, the previous tile's stores (>= MT instructions: at least lane 0
// of every tile holds a chunk, and the partial-chunk path only adds stores) and the next
// tile's rows 0..r-2 (the refill of slot r-1 is issued after column r-1's math).  A smaller n
// only waits longer, so the immediates below take the lower bounds:
//   steady state   r = 0: K-1+MT,   r >= 1: K-2+MT
//   first tile     r = 0: K-1,      r >= 1: K-2        (no stores before it)
//   last tile      K-1-r                                (nothing refilled)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>
#include <utility>

#include "rs_device.hpp"
#include "rs_plan.hpp"

namespace rsmi {

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
// f(integral_constant<0>), ..., f(integral_constant<N-1>), in order
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// 16 bytes per lane from g into LDS at byte offset lds + 16 * lane (global_load_lds_dwordx4,
// nontemporal).  Issued from asm so the compiler's waitcnt pass does not see an LDS write:
// its LDS-DMA tracking cannot tell the ring's slots apart and put a vmcnt(0) at the start of
// every tile, which drains the very queue this kernel keeps full.  All waits on these loads
// are explicit (wait_vmcnt); the loop issues no compiler-tracked vector loads.
__device__ __forceinline__ void dma16_nt(const void* g, uint32_t lds) {
    // M0 is compiler-reserved: saved and restored inside the statement that writes it; the
    // s_nop covers the M0 write -> LDS-DMA read of M0 (one wait state on gfx9)
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off nt\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(g), "s"(lds)
        : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits on gfx9");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// acc[j] ^= coef[j][c] (x) x over one 16-byte chunk: 3 v_perm_b32 per (output, dword) on the
// bit fields 0-2, 3-5, 6-7, XORs paired across columns (rs_fast_kernel has the derivation).
template <int K, int MT>
__device__ __forceinline__ void gf_mac_col(int c, const u32x4& x4, const u32x4 (&T)[5], uint32_t (&acc)[MT][4],
                                           uint32_t (&pend)[MT][4]) {
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const uint32_t x = u4get(x4, w);
        const uint32_t s1 = x & 0x07070707u, s2 = (x >> 3) & 0x07070707u, s3 = (x >> 6) & 0x03030303u;
#pragma unroll
        for (int j = 0; j < MT; j++) {
            const uint32_t p1 = __builtin_amdgcn_perm(u4get(T[1], j), u4get(T[0], j), s1);
            const uint32_t p2 = __builtin_amdgcn_perm(u4get(T[3], j), u4get(T[2], j), s2);
            const uint32_t p3 = __builtin_amdgcn_perm(u4get(T[4], j), u4get(T[4], j), s3);
            uint32_t& a = acc[j][w];
            uint32_t& q = pend[j][w];
            if (c == 0 && K == 1) {
                a = xor3(p1, p2, p3);
            } else if (c == 0) {
                a = p1 ^ p2;
                q = p3;
            } else if (c & 1) {
                a = xor3(a, p1, p2);
                a = xor3(a, p3, q);
            } else if (c == K - 1) {
                a = xor3(a, p1, p2);
                a ^= p3;
            } else {
                a = xor3(a, p1, p2);
                q = p3;
            }
        }
    }
}

}  // namespace

// K inputs, MT (<= 4) outputs, NT cache policy as rs_fast_kernel (loads always nontemporal;
// 1 = nontemporal stores, 2 = default stores), WPG waves per workgroup.  Same argument list
// as rs_fast_kernel (the CRC and tile-order arguments are unused), so the launcher treats
// both alike.
template <int K, int MT, int NT, int WPG>
__global__ __launch_bounds__(WPG * kWave) void rs_lds_kernel(const RsPlanDev* __restrict__ plan,
                                                             const uint8_t* __restrict__ in,
                                                             uint8_t* __restrict__ out, uint64_t in_bs,
                                                             uint64_t in_rs, uint64_t out_bs, uint64_t out_rs,
                                                             uint32_t S, uint32_t cpb, uint32_t tpb, uint32_t ntiles,
                                                             const uint32_t*, uint16_t*, uint32_t, uint32_t,
                                                             uint32_t) {
    static_assert(K >= 2 && K - 1 + MT < 64, "vmcnt immediates");
    __shared__ u32x4 s_tbl[K * kColDwords / 4];
    __shared__ u32x4 s_ring[WPG][K][kWave];  // per wave: one 1 KiB slot per input row
    {
        const uint32_t* src = plan->tbl;
        uint32_t* dst = reinterpret_cast<uint32_t*>(s_tbl);
        for (int i = threadIdx.x; i < K * kColDwords; i += WPG * kWave) dst[i] = src[i];
    }
    __syncthreads();

    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint32_t nw = gridDim.x * WPG;
    uint32_t t = blockIdx.x * WPG + wid;
    if (t >= ntiles) return;

    uint64_t in_off[K], out_off[MT];
#pragma unroll
    for (int c = 0; c < K; c++) in_off[c] = uint64_t(plan->in_row[c]) * in_rs;
#pragma unroll
    for (int j = 0; j < MT; j++) out_off[j] = uint64_t(plan->out_row[j]) * out_rs;

    u32x4(&ring)[K][kWave] = s_ring[wid];
    const uint32_t ring_lds =
        __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>((lds_ptr_t)(&ring[0][0]))));
    // row c of tile (blk, tib) -> slot c; lanes past the block's end clamp to its last chunk
    auto refill = [&](uint32_t b, uint32_t tb, int c) {
        uint32_t ch = tb * kWave + lane;
        ch = ch < cpb ? ch : cpb - 1;
        const uint8_t* p = in + uint64_t(b) * in_bs + in_off[c] + uint64_t(ch) * 16u;
        dma16_nt(p, ring_lds + uint32_t(c) * (kWave * 16u));
    };

    uint32_t blk = t / tpb;
    uint32_t tib = t - blk * tpb;
    const uint32_t step_b = nw / tpb, step_t = nw - step_b * tpb;
#pragma unroll
    for (int c = 0; c < K; c++) refill(blk, tib, c);

    const u32x4* tbl = s_tbl;
    // one tile; MODE 0 = first tile with a next one, 1 = steady state, 2 = last tile
    auto tile = [&](auto mode) {
        constexpr int MODE = decltype(mode)::value;
        uint32_t nblk = blk + step_b, ntib = tib + step_t;
        if (ntib >= tpb) {
            ntib -= tpb;
            nblk++;
        }
        uint32_t acc[MT][4], pend[MT][4];
        u32x4 xc, xn, Tc[5], Tn[5];
        if constexpr (MODE == 0) wait_vmcnt<K - 1>();
        else if constexpr (MODE == 1) wait_vmcnt<K - 1 + MT>();
        else wait_vmcnt<K - 1>();
        xc = ring[0][lane];
#pragma unroll
        for (int f = 0; f < 5; f++) Tc[f] = tbl[f];
        static_for<K>([&](auto ci) {
            constexpr int c = decltype(ci)::value;
            if constexpr (c + 1 < K) {
                if constexpr (MODE == 0) wait_vmcnt<K - 2>();
                else if constexpr (MODE == 1) wait_vmcnt<K - 2 + MT>();
                else wait_vmcnt<K - 2 - c>();
                xn = ring[c + 1][lane];
#pragma unroll
                for (int f = 0; f < 5; f++) Tn[f] = tbl[(c + 1) * 5 + f];
            }
            gf_mac_col<K, MT>(c, xc, Tc, acc, pend);
            // xc was consumed above, so slot c is free: refill it with the next tile's row
            if constexpr (MODE != 2) refill(nblk, ntib, c);
            xc = xn;
#pragma unroll
            for (int f = 0; f < 5; f++) Tc[f] = Tn[f];
            __builtin_amdgcn_sched_barrier(0);
        });
#pragma unroll
        for (int j = 0; j < MT; j++)
#pragma unroll
            for (int w = 0; w < 4; w++) asm volatile("" : "+v"(acc[j][w]));

        uint8_t* ob = out + uint64_t(blk) * out_bs;
        const uint32_t ch = tib * kWave + lane;
        if (ch < cpb) {
            const uint32_t boff = ch * 16u;
            if (boff + 16u <= S) {
#pragma unroll
                for (int j = 0; j < MT; j++) {
                    const u32x4 o = u32x4{acc[j][0], acc[j][1], acc[j][2], acc[j][3]};
                    if constexpr (NT == 1)
                        __builtin_nontemporal_store(o, reinterpret_cast<u32x4*>(ob + out_off[j]) + ch);
                    else
                        *(reinterpret_cast<u32x4*>(ob + out_off[j]) + ch) = o;
                }
            } else {
                // the row's last, partial chunk (1..15 bytes): whole dwords, then bytes
#pragma unroll
                for (int j = 0; j < MT; j++) {
                    uint8_t* p = ob + out_off[j] + boff;
#pragma unroll
                    for (int w = 0; w < 4; w++) {
                        const uint32_t val = acc[j][w];
                        const uint32_t o = boff + 4u * w;
                        if (o + 4u <= S) {
                            *reinterpret_cast<uint32_t*>(p + 4 * w) = val;
                        } else if (o < S) {
                            p[4 * w] = uint8_t(val);
                            if (o + 1u < S) p[4 * w + 1] = uint8_t(val >> 8);
                            if (o + 2u < S) p[4 * w + 2] = uint8_t(val >> 16);
                        }
                    }
                }
            }
        }
        blk = nblk;
        tib = ntib;
    };

    if (t + nw < ntiles) {
        tile(std::integral_constant<int, 0>{});
        t += nw;
        for (; t + nw < ntiles; t += nw) tile(std::integral_constant<int, 1>{});
    }
    tile(std::integral_constant<int, 2>{});
    // nothing may be left in flight into LDS when the wave ends
    wait_vmcnt<0>();
}

// rsmi_set_option("lds_dma", 1): aligned RS(10,4) encode (K=10, MT=4) and 1-row reconstruct
// (K=10, MT=1) shapes; [k][mt] for those, WPG = 4.
const LdsKernelTable& lds_kernels() {
    static const LdsKernelTable t = [] {
        LdsKernelTable x{};
        x.fn[0] = reinterpret_cast<void*>(&rs_lds_kernel<10, 4, 1, 4>);
        x.fn[1] = reinterpret_cast<void*>(&rs_lds_kernel<10, 1, 2, 4>);
        x.fn[2] = reinterpret_cast<void*>(&rs_lds_kernel<10, 4, 1, 2>);
        x.fn[3] = reinterpret_cast<void*>(&rs_lds_kernel<10, 1, 2, 2>);
        x.wpg[0] = x.wpg[1] = 4;
        x.wpg[2] = x.wpg[3] = 2;
        return x;
    }();
    return t;
}

}  // namespace rsmi
