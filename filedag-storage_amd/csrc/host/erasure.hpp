// erasure.hpp -- C++ mirror of dag/node/dagnode/erasure.go over the rsmi C-ABI.
//
// Same method set and semantics as the Go type: NewErasure validation (erasure.go:16-24),
// EncodeData = Split + Encode with the empty-block short-circuit (:51-65),
// DecodeDataBlocks with the isZero/break quirk (:70-83), DecodeDataAndParityBlocks
// (:87-93), ShardSize = ceilFrac(B, k) (:96-98).  A shard is a byte vector; an empty
// vector is a missing shard (Go: nil / zero-length slice).  Every coded byte comes from
// the gfx950 kernels behind include/rsmi.h; there is no CPU fallback.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../../include/rsmi.h"
#include "datanode.hpp"

namespace rsmi {
namespace host {

// upstream sentinel texts (reedsolomon.Err*), so callers can match on them
Status rsmi_status(int rc);
int64_t ceil_frac(int64_t numerator, int64_t denominator);  // utils.go:6-21

// Process-wide context per (k, m, device, replica): NewErasure runs per block in the reference
// (node.go:277,376) but the matrix / device plans are built once.  `replica` tells apart the
// members of a Dag Node's device list that name the same device (DagNode::New with a device list:
// every member has contexts, group-commit queue and coalescing lanes of its own).
rsmi_ctx* shared_context(int k, int m, int device, int* rc, int replica = 0);
// Per-block calls from concurrent threads (Erasure's encodes and reconstructs) go to kCallLanes
// contexts per (k, m, device), one per calling thread in turn; lane 0 is the shared context.  One
// (the default) keeps every caller in one group-commit queue, whose batches the context codes on
// its own coalescing lanes (option "coalesce_lanes", include/rsmi.h), so concurrent Puts become
// a few launches over tables of blocks instead of a launch per block (round 4 spread the callers
// over 4 contexts instead, each queue then holding ~1 block per batch: 2,048 calls in 1,744-2,048
// groups, profiles/r04/af).
#ifndef RSMI_HOST_CALL_LANES
#define RSMI_HOST_CALL_LANES 1
#endif
constexpr int kCallLanes = RSMI_HOST_CALL_LANES;
rsmi_ctx* call_context(int k, int m, int device, int* rc, int replica = 0);
// rsmi_get_stat summed over the lanes of (k, m, device, replica) (the coalescing counters)
long lane_stat(int k, int m, int device, const char* key, int replica = 0);
// Bring up every lane's device resources (streams, plans, CRC tables) with one tiny encode each,
// so the first concurrent calls do not pay for them (a Dag Node does this when it starts);
// errors are left to the real calls, which fail loudly.
void warm_contexts(int k, int m, int device, int replica = 0);
// Close every shared context (process shutdown, with no call in flight).
void release_shared_contexts();

// Host staging for the batch calls: page-locked (rsmi_host_alloc) so the batch copies run
// as DMA at full PCIe rate instead of bouncing through the runtime's own pinned pool.
// Grown on demand and reused; contents are not cleared.  If page-locking fails (no
// device) it holds ordinary memory and the rsmi call itself reports the device error.
class PinnedBuf {
public:
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf&) = delete;
    PinnedBuf& operator=(const PinnedBuf&) = delete;
    ~PinnedBuf() { release(); }
    uint8_t* reserve(size_t bytes);
    uint8_t* data() const { return p_; }
    size_t capacity() const { return cap_; }

private:
    void release();
    uint8_t* p_ = nullptr;
    size_t cap_ = 0;
    bool pinned_ = false;
};

// Page-locking costs tens of ms per 100 MB, so the batch paths share one staging buffer per
// thread, kept for the thread's life, and cut their batches to at most kStagingBytes.
constexpr size_t kStagingBytes = size_t(64) << 20;
PinnedBuf& thread_staging();
// The calling thread's page-locked scratch for one block's rows (single-block encodes and
// reconstructs), separate from thread_staging; grown on demand, contents not cleared.  A thread
// that ends hands its scratch to a process-wide pool (by NUMA node), and a new thread takes one
// placed on its own node, so short-lived callers do not page-lock fresh memory each
// (page-locking holds the process's memory-map lock, which stalls every other thread's page
// faults meanwhile).
uint8_t* block_scratch(size_t bytes);
// n bytes into page-locked staging on the calling thread; from 1 MiB with streaming stores, which
// skip the destination's read-for-ownership and leave no dirty lines for the GPU's zero-copy
// reads to snoop (tools/latency.cpp: a 4 MiB Split copy + in-place encode 278-297 -> 252-255 us;
// level at 256 KiB)
void copy_to_staging(uint8_t* dst, const uint8_t* src, size_t n);
void copy_streaming(uint8_t* dst, const uint8_t* src, size_t n);  // always streaming stores
inline size_t staging_blocks(size_t block_bytes) {
    return block_bytes >= kStagingBytes ? 1 : kStagingBytes / block_bytes;
}

class Erasure {
public:
    static Status New(int data_blocks, int parity_blocks, int64_t block_size, Erasure* out, int device = 0,
                      int replica = 0);
    // through rsmi_encode_block_coalesced: concurrent Puts on one process-wide context are
    // batched on the GPU (group commit); a lone caller runs alone, unchanged
    Status EncodeData(const Bytes& data, std::vector<Bytes>* shards) const;
    // EncodeData plus R(shard) of every shard from the GPU (include/rsmi.h, datanode CRC-16);
    // raw is left empty for an empty block
    Status EncodeDataWithCrc(const Bytes& data, std::vector<Bytes>* shards, std::vector<uint32_t>* raw) const;
    // ... and, when raw32 is not null, R32(shard) for the mutcask value checksum (CRC-32)
    Status EncodeDataWithCrcs(const Bytes& data, std::vector<Bytes>* shards, std::vector<uint32_t>* raw,
                              std::vector<uint32_t>* raw32) const;
    // EncodeData into one caller buffer of (k+m) * ShardSize() bytes, shard i at i * ShardSize():
    // the Go slices Split returns alias one buffer, so the shards need no copies of their own.
    // raw / raw32 (k+m entries each, may be null): R(shard) / R32(shard) as EncodeDataWithCrcs.
    // flat should be page-locked (block_scratch): the block is Split into it on the calling
    // thread, and the call (alone or in a coalesced group) codes it in place.
    Status EncodeDataFlat(const Bytes& data, uint8_t* flat, uint32_t* raw, uint32_t* raw32) const;
    // EncodeDataFlat of a block of B bytes the caller has already copied to the start of flat
    Status EncodeSplitFlat(size_t B, uint8_t* flat, uint32_t* raw, uint32_t* raw32) const;
    Status DecodeDataBlocks(std::vector<Bytes>& shards) const;
    Status DecodeDataAndParityBlocks(std::vector<Bytes>& shards) const;
    int64_t ShardSize() const { return ceil_frac(block_size_, data_blocks_); }
    int data_blocks() const { return data_blocks_; }
    int parity_blocks() const { return parity_blocks_; }

private:
    Status reconstruct(std::vector<Bytes>& shards, bool data_only) const;
    int data_blocks_ = 0, parity_blocks_ = 0, device_ = 0, replica_ = 0;
    int64_t block_size_ = 0;
};

}  // namespace host
}  // namespace rsmi
