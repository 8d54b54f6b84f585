// dagnode.hpp -- C++ mirror of dag/node/dagnode's DagNode (the erasure set).
//
// Same public surface the Dag Pool calls: NewDagNode, Put, Get, GetSize,
// Has, DeleteBlock, PutMany, the slot methods, GetConfig / GetDataNodeState, the
// heartbeat and repair loops and RepairDataNode.  Semantics follow node.go and
// data_recovery.go line by line where they are observable:
//   * Meta{BlockSize int32} stored as 4 bytes little-endian with every shard (node.go:48-50,367-374);
//   * write quorum k (k+1 when k == m), read quorum k (entryQuorum, node.go:439-446);
//   * meta quorum via reduceQuorumErrs + findMetaInQuorum, including "quorum < 2 fails"
//     (node.go:334-355, :491-533; error.go:30-82);
//   * Get fetches shards with cancel-others after k successes, decodes the data shards,
//     queues a read-repair for shards that failed on online nodes (queue of 10000, drops
//     when full) and truncates to BlockSize (node.go:220-326);
//   * repairBlock / RepairDataNode (data_recovery.go:16-167).
// Fan-out is sequential over in-process datanodes; the success / failure quorum rules of
// paralleltask.Wait (parallel_task.go:59-84) decide the outcome exactly as in Go, and the
// Get fan-out returns after the first k successes in node order.
//
// Additions for the GPU engine (results identical to the per-block path):
//   * PutMany batches equal-size blocks through one rsmi_encode_batch_host call;
//   * RepairDataNodeBatched rebuilds only the repaired node's row for many keys at once
//     with rsmi_reconstruct_rows_batch_host;
//   * GetMany decodes the blocks that need it in GPU batches (8(f) rank 3);
//   * MigrateBlocks moves blocks between erasure sets as batched decode + encode (rank 4);
//   * Put writes its block-only data shards, and a lone degraded Get copies its present data rows
//     into the block, while the codec call is in flight (rsmi_set_wait_hook).
#pragma once
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "datanode.hpp"
#include "erasure.hpp"
#include "fanout.hpp"

namespace rsmi {
namespace host {

struct DagNodeConfig {  // dag/config/config.go:24-29
    std::string name;
    std::vector<std::string> nodes;
    int data_blocks = 0;
    int parity_blocks = 0;
};

struct Meta {
    int32_t block_size = 0;
};

extern const char* const kErrReadQuorum;   // error.go:12
extern const char* const kErrNodeNotFound;  // error.go:9

struct StorageNode {
    std::shared_ptr<DataNodeClient> client;
    bool state = false;  // set by the heartbeat (node.go:127-157)
};

class DagNode {
public:
    static constexpr int kClusterSlots = 16384;  // slotsmgr.ClusterSlots
    static constexpr size_t kRepairQueueCap = 10000;

    // node.go:53-73 (clients replace the gRPC dial of datanode.NewClient)
    static Status New(const DagNodeConfig& cfg, std::vector<std::shared_ptr<DataNodeClient>> clients,
                      std::unique_ptr<DagNode>* out, int device = 0);
    // ... coding on a list of GPUs (members; a device may repeat).  Every per-key call (Put, Get,
    // the read-repair, RepairDataNode's rebuilds) runs on the member that owns the key: the Dag
    // Pool's hash slot crc16(key) & 0x3FFF (hash_slot.go:20-22) in contiguous ranges of
    // 16384 / members slots per member, as rsmi_group_member_of_key.  Each member has contexts,
    // group-commit queue and coalescing lanes of its own, so concurrent callers spread over the
    // members' PCIe links.  The batch calls (PutMany, GetMany's decode, RepairDataNodeBatched)
    // order each chunk's blocks by member and code the members' ranges concurrently.  Stored
    // entries and returned blocks are identical to the one-device node's.
    static Status New(const DagNodeConfig& cfg, std::vector<std::shared_ptr<DataNodeClient>> clients,
                      std::unique_ptr<DagNode>* out, const std::vector<int>& devices);
    ~DagNode();

    Status Put(const std::string& key, const Bytes& block);
    Status PutMany(const std::vector<std::string>& keys, const std::vector<Bytes>& blocks);
    Status Get(const std::string& key, Bytes* block);
    Status GetSize(const std::string& key, int* size);
    Status Has(const std::string& key, bool* has);
    Status DeleteBlock(const std::string& key);

    // Get for many keys: blocks whose data shards all arrived are assembled directly, the
    // rest are decoded on the GPU in batches grouped by (block size, survivor pattern)
    // (SURVEY.md 8(f) rank 3).  statuses[i] is what Get(keys[i]) would return.
    void GetMany(const std::vector<std::string>& keys, std::vector<Bytes>* blocks, std::vector<Status>* statuses,
                 size_t batch = 256);

    // RepairDataNode runs the batched form (kRepairBatch keys per flush at most); the per-key
    // loop of data_recovery.go stays as RepairDataNodePerKey (A/B legs, tools/bench_dagnode)
    static constexpr size_t kRepairBatch = 256;
    Status RepairDataNode(int from_index, int repair_index);
    Status RepairDataNodePerKey(int from_index, int repair_index);
    // batched: keys needing repair are grouped by (block size, survivor pattern) and rebuilt
    // `batch` at a time on the GPU
    Status RepairDataNodeBatched(int from_index, int repair_index, size_t batch, size_t* repaired = nullptr);

    // heartbeat: one health-check round (node.go:132-144); the ticker loop is the caller's
    void HealthCheckAll();
    // drain queued read-repairs synchronously; returns how many ran (RunRepairTask body)
    size_t RunRepairTasks();
    void StartRepairWorker();  // RunRepairTask goroutine
    void Close();

    bool AddSlot(uint64_t slot);
    bool ClearSlot(uint64_t slot);
    bool GetSlot(uint64_t slot) const;
    int GetNumSlots() const { return num_slots_; }
    const DagNodeConfig& GetConfig() const { return config_; }
    int Members() const { return int(devices_.size()); }
    int MemberOfKey(const std::string& key) const;  // the member coding key's per-key calls
    int MemberDevice(int member) const { return devices_.at(size_t(member)); }
    int MemberReplica(int member) const { return replicas_.at(size_t(member)); }
    bool GetDataNodeState(int set_index) const;
    void SetDataNodeState(int set_index, bool v) { nodes_.at(set_index).state = v; }
    // Put / PutMany compute each shard's datanode entry checksum on the GPU, from the rows
    // the encode already holds, and send it with the shard (DataNodeClient::PutWithChecksum)
    // instead of leaving the byte-serial CRC to the datanode.  On by
    // default; the stored entries are byte-identical either way.
    void SetGpuChecksums(bool v) { gpu_checksums_ = v; }
    // With SetGpuChecksums, also compute the mutcask value CRC-32 (cask.go:73-79) on the GPU
    // (a separate rows pass after the encode).  Off by default: the datanode's own
    // carry-less-multiply fold (crc_clmul.hpp, ~30 GiB/s per core, run in the datanode calls'
    // fan-out) measured faster than the extra GPU pass.  Stored values are
    // byte-identical either way.
    void SetGpuValueChecksums(bool v) { gpu_value_checksums_ = v; }
    // Get / GetMany read shards with DataNodeClient::GetForVerify and check the stored entry
    // (and mutcask value) checksums on the GPU, one call per fetch wave, instead of each
    // datanode checking its own (server.go:93-97, cask.go:250).  A shard that fails is
    // treated exactly like a failed fetch: missing, on the repair list, the next node
    // fetched.  Off by default (it needs the datanode RPC that skips the check).
    void SetGpuVerifiedReads(bool v) { gpu_verified_reads_ = v; }
    // The k+m datanode calls of one block run concurrently, like node.go's goroutine per
    // datanode (fanout.hpp); results are replayed in node order, so every quorum outcome,
    // repair list and error equals the sequential one.  On by default.
    void SetParallelFanout(bool v) { parallel_ = v; }
    // ... but only where it pays: a lone caller (concurrent callers already keep the cores
    // busy) and shards of at least this many bytes (in-process datanode calls on small
    // shards cost less than a thread hand-off).  Default 128 KiB (tools/bench_dagnode).
    void SetFanoutMinBytes(size_t v) { fanout_min_ = v; }
    // A lone caller's per-block Put, degraded Get and per-key RepairDataNode code the block in
    // place in the page-locked block scratch (Split copy, one zero-copy kernel, the datanodes or
    // the block reading views of it) instead of through Erasure's shard vectors and the engine's
    // group commit.  On by default; the stored entries and returned blocks are identical either
    // way (off: tools/bench_dagnode's A/B legs).
    void SetLoneCallerPaths(bool v) { lone_paths_ = v; }
    std::pair<int, int> EntryQuorum() const;  // (read, write)
    size_t RepairQueueLen();
    // Per-phase host time of Put / PutMany / RepairDataNodeBatched (diagnostic, off by default):
    // seconds spent fetching shards (window fetches of the batched repair), staging rows into
    // page-locked memory, in the codec call, and writing to the datanodes, summed over the
    // calling and helper threads since the last ResetPhases (overlapped phases both count).
    enum class Phase { Fetch = 0, Stage = 1, Codec = 2, Put = 3 };
    void SetPhaseTiming(bool v) { phase_on_ = v; }
    std::array<double, 4> PhaseSeconds() const;
    void ResetPhases();
    // With phase timing on, also keep every phase interval (phase, thread, start and end in
    // seconds since ResetPhases) for a timeline of the overlap (diagnostic, tools/bench_dagnode)
    struct PhaseEvent {
        int phase;
        uint64_t thread;
        double t0, t1;
    };
    void SetPhaseTrace(bool v) { trace_on_ = v; }
    static constexpr int kTraceWaitFetch = 4, kTraceWaitWrites = 5;  // trace-only ids: waits on helpers
    std::vector<PhaseEvent> PhaseEvents();

private:
    using PhaseClock = std::chrono::steady_clock;
    void phase_add(Phase p, PhaseClock::time_point t0);
    void trace_add(int id, PhaseClock::time_point t0, PhaseClock::time_point t1);
    std::atomic<bool> phase_on_{false};
    std::atomic<uint64_t> phase_ns_[4] = {};
    std::atomic<bool> trace_on_{false};
    std::mutex trace_mu_;
    std::vector<PhaseEvent> trace_;
    PhaseClock::time_point trace_epoch_ = PhaseClock::now();
    struct Fetched {
        Meta meta;
        std::vector<Bytes> shards;
        std::vector<int> repair;
        // deferred verification (GetMany): the accepted shards' entry metas and stored checksums
        std::vector<Bytes> metas;
        std::vector<DataNodeClient::Stored> stored;
        bool assembled = false;  // GetMany: the block was taken from the batch decode's staging
        int member = 0;          // the key's member (a device list)
    };
    // defer_verify: with GPU-verified reads on, accept the first wave's shards unchecked and keep
    // their stored checksums in f, for one batched check across many keys (verify_fetched)
    Status fetch_for_get(const std::string& key, Fetched* f, bool defer_verify = false);
    // the batched check of deferred fetches: one GPU call per shard size over every key's
    // accepted shards; bad[q] is set for keys with a shard that fails
    void verify_fetched(std::vector<Fetched>& fs, const std::vector<Status>& st, const std::vector<char>& skip,
                        std::vector<char>* bad);
    Status finish_get(const std::string& key, Fetched& f, Bytes* block);
    Status decode_into_block(const std::string& key, Fetched& f, size_t S, Bytes* block, bool* done);
    Status repair_row_in_place(const std::string& key, int size, const std::vector<Bytes>& shards, int to, bool* done);
    Status get_meta_info(const std::string& key, Meta* meta, std::vector<StorageNode*>* online);
    Status repair_block(const std::string& key, int32_t block_size, std::vector<Bytes> shards,
                        const std::vector<int>& indexes);
    Status fetch_for_repair(const std::string& key, int repair_index, std::vector<Bytes>* shards);
    static Bytes encode_meta(int32_t size);
    // server.go:70's checksum of the entry (meta, S-byte shard) from the shard's R(shard)
    static uint16_t entry_checksum(const Bytes& meta, size_t S, uint32_t raw);
    // the mutcask value checksum (cask.go:73-79) of the entry holding a shard with entry
    // checksum crc16 and CRC-32 R32(shard) = raw32
    static uint32_t value_checksum(const Bytes& meta, size_t S, uint16_t crc16, uint32_t raw32);

    DagNodeConfig config_;
    std::vector<StorageNode> nodes_;
    std::vector<uint8_t> slots_;
    int num_slots_ = 0;
    // the members' devices and, for a device that repeats, which of its contexts (erasure.hpp)
    std::vector<int> devices_{0}, replicas_{0};
    rsmi_ctx* member_ctx(int member, int* rc) const;  // the member's shared context for (k, m)
    Status member_erasure(int member, int64_t block_size, Erasure* out) const;
    // A chunk of nb blocks reordered so each member's blocks are contiguous: stable, member
    // ascending; perm[j] is the chunk position staged at slot j, and ranges[i] = (first slot,
    // count) of member i.  One member: the identity.
    struct MemberOrder {
        std::vector<size_t> perm;
        std::vector<std::pair<size_t, size_t>> ranges;
    };
    MemberOrder member_order(size_t nb, const std::function<int(size_t)>& member_of_pos) const;
    // code(ctx, first slot, count) for every member range with blocks, concurrently on the
    // member pool (one member: on this thread); the first nonzero status in member order
    int code_members(const MemberOrder& order, const std::function<int(rsmi_ctx*, size_t, size_t)>& code);
    std::unique_ptr<FanOut> member_fan_;
    bool gpu_checksums_ = true;
    bool gpu_value_checksums_ = false;
    bool gpu_verified_reads_ = false;
    // GPU check of the unverified shards of one fetch wave; failures become errors in got[]
    void verify_wave(int member, const std::vector<int>& wave, const std::vector<Bytes>& metas, const std::vector<Bytes>& data,
                     const std::vector<DataNodeClient::Stored>& stored, std::vector<Status>& got);
    bool parallel_ = true;
    bool lone_paths_ = true;
    size_t fanout_min_ = size_t(128) << 10;
    std::atomic<int> active_{0};          // caller threads inside the public calls
    std::atomic<size_t> last_shard_{0};   // shard size of the latest Put / Get (for GetMeta)
    std::unique_ptr<FanOut> fan_;
    void fan(int count, const std::function<void(int)>& f, size_t shard_bytes);
    // memcpy, spread over the fan-out pool for a lone caller's large copies
    void copy_bytes(uint8_t* dst, const uint8_t* src, size_t n);
    // whole-key tasks (GetMany): on the pool for a lone caller, whatever the shard size
    void fan_keys(int count, const std::function<void(int)>& f);
    struct Active {  // counts a caller for the fan-out policy
        std::atomic<int>& a;
        explicit Active(std::atomic<int>& x) : a(x) { a++; }
        ~Active() { a--; }
    };

    std::mutex q_mu_;
    std::condition_variable q_cv_;
    std::deque<std::function<void()>> repair_queue_;
    std::thread worker_;
    bool stop_ = false;
};

// Slot-migration data move (dag/pool/poolservice/cluster.go:244-270, per key: from.Get ->
// to.Put -> from.DeleteBlock) with both coding steps batched on the GPU: GetMany on the
// source erasure set, PutMany on the destination (the two sets may use different (k, m)).
// statuses[i]: ok when key i now lives on `to`; a key absent on `from` counts as migrated
// (format.IsNotFound); delete failures on `from` only warn in the reference and are ignored.
void MigrateBlocks(DagNode& from, DagNode& to, const std::vector<std::string>& keys, std::vector<Status>* statuses,
                   size_t batch = 256);

// reduceQuorumErrs (error.go:73-82): most frequent error (ignoring errNodeNotFound /
// errNodeAccessDenied; an empty string is nil and wins ties) if it reaches quorum.
Status reduce_quorum_errs(const std::vector<Status>& errs, int quorum, const char* quorum_err);
// findMetaInQuorum (node.go:491-533)
Status find_meta_in_quorum(const std::vector<Meta>& metas, int quorum, Meta* out);

}  // namespace host
}  // namespace rsmi
