// rs_device.hpp -- device helpers shared by the coding kernels (rs_kernels.hip,
// rs_lds_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace rsmi {

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));  // any byte alignment
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));  // dword alignment

__device__ __forceinline__ uint32_t u4get(const u32x4& v, int i) { return v[i]; }

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const u32x4* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
// Byte-aligned 16-byte access: the ROCm runtime runs gfx9+ in unaligned access mode, so this
// is still one global_load/store_dwordx4 (the memory pipeline splits it as needed).
template <bool NT>
__device__ __forceinline__ u32x4 ld16u(const uint8_t* p) {
    if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4u*>(p));
    else return *reinterpret_cast<const u32x4u*>(p);
}
template <bool NT>
__device__ __forceinline__ void st16u(uint8_t* p, u32x4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4u*>(p));
    else *reinterpret_cast<u32x4u*>(p) = v;
}

// 16 bytes of a row at byte offset off; bytes at or past S read as zero (CRC passes: zero
// bytes past the end only move the reference point, which the caller's shift accounts for)
template <bool ALIGNED>
__device__ __forceinline__ u32x4 crc_chunk_load(const uint8_t* row, uint64_t off, uint64_t S) {
    u32x4 v = {0, 0, 0, 0};
    if (off >= S) return v;
    if constexpr (ALIGNED) {
        v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(row + off));
        if (off + 16 > S) {
            const int valid = int(S - off);
#pragma unroll
            for (int w = 0; w < 4; w++) {
                const int nb = valid - 4 * w;
                const uint32_t mask = nb >= 4 ? ~0u : nb <= 0 ? 0u : (1u << (8 * nb)) - 1u;
                v[w] &= mask;
            }
        }
    } else if (off + 16 <= S) {
        v = ld16u<true>(row + off);  // byte-aligned 16-byte load (also over PCIe from host memory)
    } else {
#pragma unroll
        for (int q = 0; q < 16; q++)
            if (off + q < S) v[q >> 2] |= uint32_t(row[off + q]) << (8 * (q & 3));
    }
    return v;
}

}  // namespace rsmi
