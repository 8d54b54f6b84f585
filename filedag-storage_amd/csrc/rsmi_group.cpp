// rsmi_group.cpp -- one process driving several GPUs (include/rsmi.h "device groups").
//
// The reference's Dag Pool hosts every DagNode of the cluster in one process
// (dag/pool/poolservice/cluster.go:28-41) and routes each key to a node by its hash slot
// (hash_slot.go:20-22: crc16(key) & 0x3FFF).  Blocks are coded independently
// (dag/node/dagnode/node.go:358-408), so a group of per-device contexts spreads a host batch over
// the node's GPUs as contiguous block ranges, each range on its own context (own HIP streams
// and page-locked staging) from its own host thread; no data crosses devices and no collective
// runs.  The caller's buffers are written in place, so results need no reordering.
#include "rsmi_impl.hpp"

#include <thread>

using namespace rsmi;
using namespace rsmi::impl;

struct rsmi_group {
    int k = 0, m = 0;
    std::vector<rsmi_ctx*> ctx;  // one per entry of the device list (a device may repeat)
};

namespace {

constexpr int kClusterSlots = 16384;  // dag/slotsmgr/slots_mgr.go:8

// Run f(i, start, count) for every non-empty part on its own thread (part 0 on the caller's);
// the first failing part's status in part order, so results do not depend on timing.
template <class F>
int run_parts(const rsmi_group* s, size_t nblocks, F f) {
    const size_t parts = s->ctx.size();
    std::vector<int> rc(parts, RSMI_OK);
    std::vector<std::thread> th;
    for (size_t i = 1; i < parts; i++) {
        size_t st, cnt;
        rsmi_partition(nblocks, int(parts), int(i), &st, &cnt);
        if (cnt) th.emplace_back([&, i, st, cnt] { rc[i] = f(i, st, cnt); });
    }
    size_t st0, cnt0;
    rsmi_partition(nblocks, int(parts), 0, &st0, &cnt0);
    if (cnt0) rc[0] = f(size_t(0), st0, cnt0);
    for (auto& t : th) t.join();
    for (int r : rc)
        if (r != RSMI_OK) return r;
    return RSMI_OK;
}

}  // namespace

extern "C" {

int rsmi_group_open(int k, int m, const int* devices, int ndev, rsmi_group** out) {
    if (!out) return RSMI_ERR_INVALID_ARG;
    *out = nullptr;
    if (k <= 0 || m <= 0) return RSMI_ERR_INV_SHARD_NUM;
    if (k + m > 256) return RSMI_ERR_MAX_SHARD_NUM;
    if (!devices || ndev <= 0 || ndev > 1024) return RSMI_ERR_INVALID_ARG;
    auto* s = new rsmi_group();
    s->k = k;
    s->m = m;
    for (int i = 0; i < ndev; i++) {
        rsmi_ctx* c = nullptr;
        const int rc = rsmi_open(k, m, devices[i], &c);
        if (rc != RSMI_OK) {
            rsmi_group_close(s);
            return rc;
        }
        s->ctx.push_back(c);
    }
    *out = s;
    return RSMI_OK;
}

void rsmi_group_close(rsmi_group* s) {
    if (!s) return;
    for (rsmi_ctx* c : s->ctx) rsmi_close(c);
    delete s;
}

int rsmi_group_size(const rsmi_group* s) { return s ? int(s->ctx.size()) : 0; }

rsmi_ctx* rsmi_group_context(rsmi_group* s, int i) {
    if (!s || i < 0 || size_t(i) >= s->ctx.size()) return nullptr;
    return s->ctx[size_t(i)];
}

int rsmi_group_member_of_key(const rsmi_group* s, const uint8_t* key, size_t len) {
    if (!s || s->ctx.empty()) return -1;
    const int slot = rsmi_key_slot(key, len);
    if (slot < 0) return -1;
    // contiguous slot ranges per member, like DagNodes owning SlotPairs (slotsmgr)
    return int(size_t(slot) * s->ctx.size() / kClusterSlots);
}

int rsmi_group_encode_batch_host(rsmi_group* s, const uint8_t* data, size_t data_block_stride, uint8_t* parity,
                               size_t parity_block_stride, size_t S, size_t nblocks) {
    if (!s || !data || !parity) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    return run_parts(s, nblocks, [&](size_t i, size_t st, size_t cnt) {
        return rsmi_encode_batch_host(s->ctx[i], data + st * data_block_stride, data_block_stride,
                                      parity + st * parity_block_stride, parity_block_stride, S, cnt);
    });
}

int rsmi_group_encode_batch_host_crcs(rsmi_group* s, const uint8_t* data, size_t data_block_stride, uint8_t* parity,
                                    size_t parity_block_stride, size_t S, size_t nblocks, uint32_t* raw16_out,
                                    uint32_t* raw32_out) {
    if (!s || !data || !parity) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    const size_t n = size_t(s->k + s->m);
    return run_parts(s, nblocks, [&](size_t i, size_t st, size_t cnt) {
        return rsmi_encode_batch_host_crcs(s->ctx[i], data + st * data_block_stride, data_block_stride,
                                           parity + st * parity_block_stride, parity_block_stride, S, cnt,
                                           raw16_out ? raw16_out + st * n : nullptr,
                                           raw32_out ? raw32_out + st * n : nullptr);
    });
}

int rsmi_group_reconstruct_batch_host(rsmi_group* s, uint8_t* shards, size_t block_stride, size_t S, size_t nblocks,
                                    const uint8_t* present, int data_only) {
    if (!s || !shards || !present) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    return run_parts(s, nblocks, [&](size_t i, size_t st, size_t cnt) {
        return rsmi_reconstruct_batch_host(s->ctx[i], shards + st * block_stride, block_stride, S, cnt, present,
                                           data_only);
    });
}

int rsmi_group_reconstruct_rows_batch_host(rsmi_group* s, uint8_t* shards, size_t block_stride, size_t S,
                                         size_t nblocks, const uint8_t* present, const uint8_t* required) {
    if (!s || !shards || !present || !required) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    return run_parts(s, nblocks, [&](size_t i, size_t st, size_t cnt) {
        return rsmi_reconstruct_rows_batch_host(s->ctx[i], shards + st * block_stride, block_stride, S, cnt, present,
                                                required);
    });
}

}  // extern "C"
