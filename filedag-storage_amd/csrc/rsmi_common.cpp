// rsmi_common.cpp -- the entry points of include/rsmi.h that need no device: status strings,
// shard geometry, the shard-length checks, the host halves of the split checksums, and the
// device groups' partition and key routing.  Plain C++ (no HIP), so the host mirror's
// sanitizer builds (tests/cpp) link exactly this code.
#include <algorithm>
#include <cstring>

#include "../../include/rsmi.h"
#include "crc16.hpp"
#include "crc32.hpp"
#include "host/datanode.hpp"
#include "wait_hook.hpp"

using namespace rsmi;

namespace {
inline size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
thread_local WaitHook t_wait_hook;  // rsmi_set_wait_hook: this thread's pending hook
}  // namespace

namespace rsmi {
WaitHook take_wait_hook() {
    const WaitHook h = t_wait_hook;
    t_wait_hook = WaitHook{};
    return h;
}
}  // namespace rsmi

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
        case RSMI_ERR_HOST: return "host resources exhausted (memory or threads)";
        default: return "unknown status";
    }
}

size_t rsmi_recommended_pitch(size_t S) {
    if (S == 0) return 0;
    size_t p = 16;
    while (p < S) p <<= 1;
    // Measured on MI355X (tools/pitchsweep*.py; in bench.py's own context with --pitch,
    // profiles/r01/pitch_ab.txt): a power-of-two row pitch is best for S = 26215 (32 KiB, far
    // ahead of every 4 KiB step) and for S = 262144 (itself a power of two), and the worst
    // choice for S = 104858 (128 KiB).  There 11/8 S in 4 KiB granules (144 KiB) is +7% over
    // the 4 KiB-rounded 104 KiB (1 MiB RS(10,4) blocks: 6.14 against 5.72 TB/s).  Use powers
    // of two for shards up to 64 KiB (padding <= 50%) and exact powers, 11/8 S between 96 and
    // 128 KiB, and 4 KiB granules otherwise.
    if (p == S || p <= 4096) return p;
    if (S <= 65536 && p <= S + S / 2) return p;
    if (S > 98304 && S < 131072) return round_up(S * 11 / 8, 4096);
    return round_up(S, 4096);
}

size_t rsmi_shard_size(size_t block_size, int k) {
    if (k <= 0) return 0;
    return (block_size + size_t(k) - 1) / size_t(k);
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

// the datanode's host CRCs: carry-less-multiply folding from 256 bytes (host/crc_clmul.hpp)
uint16_t rsmi_crc16_ibm(const uint8_t* p, size_t n) { return host::crc16_ibm(p, n); }

uint32_t rsmi_crc32_ieee(const uint8_t* p, size_t n) { return host::crc32_ieee(p, n); }

uint32_t rsmi_crc32_entry(const uint8_t* head, size_t head_len, uint32_t raw, size_t data_len) {
    return crc32_entry(head, head_len, raw, data_len);
}

uint16_t rsmi_crc16_entry(const uint8_t* head, size_t head_len, uint32_t raw, size_t data_len) {
    return crc16_entry(head, head_len, raw, data_len);
}

int rsmi_partition(size_t nblocks, int parts, int i, size_t* start, size_t* count) {
    if (parts <= 0 || i < 0 || i >= parts || !start || !count) return RSMI_ERR_INVALID_ARG;
    // contiguous ranges, sizes differ by at most one block (rsmi/multi.py partition_blocks)
    const size_t base = nblocks / size_t(parts), extra = nblocks % size_t(parts), ii = size_t(i);
    *start = ii * base + std::min(ii, extra);
    *count = base + (ii < extra ? 1 : 0);
    return RSMI_OK;
}

void rsmi_set_wait_hook(void (*fn)(void*), void* arg) { t_wait_hook = WaitHook{fn, fn ? arg : nullptr}; }

int rsmi_run_wait_hook(void) {
    const WaitHook h = take_wait_hook();
    if (!h) return 0;
    h();
    return 1;
}

int rsmi_key_slot(const uint8_t* key, size_t len) {
    if (!key && len) return -1;
    return int(crc16_checksum(key, len) & 0x3FFF);  // keyHashSlot, hash_slot.go:20-22
}

}  // extern "C"
