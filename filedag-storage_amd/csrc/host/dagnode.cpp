// dagnode.cpp -- see dagnode.hpp.  Line references are to the reference's
// dag/node/dagnode/node.go, data_recovery.go and error.go.
#include "dagnode.hpp"

#include <algorithm>
#include <cstring>
#include <exception>
#include <future>
#include <map>
#include <stdexcept>

// 1: PutMany and GetMany without their overlap (one chunk at a time: writes joined at once, no
// fetch ahead) -- round 4's loops, for same-box A/B library builds (tools/dagnode_ab.sh)
#ifndef RSMI_BATCH_SERIAL
#define RSMI_BATCH_SERIAL 0
#endif
// Where PutMany and RepairDataNodeBatched run a chunk's codec call: on the calling thread before
// the chunk's writes go to the helper task, or as the task's first step, overlapping the next
// chunk's staging copy.  The calling thread's critical path per chunk is max(stage + codec,
// writes) in the first form and max(stage, codec + writes) in the second, so the codec call goes
// with the shorter of the two: 0 = chosen per chunk from the previous chunk's measured staging and
// write times (default), 1 = always on the calling thread (round 5), 2 = always in the task (A/B
// library builds, profiles/r06/b/).
// 1 (default): a Put writes its block-only data shards while the GPU encodes the parity; 0: every
// write after the codec call (round 5's order), for same-box A/B library builds
#ifndef RSMI_PUT_OVERLAP
#define RSMI_PUT_OVERLAP 1
#endif
// blocks up to this size: the calling thread writes those shards inside its codec call's wait
// (rsmi_set_wait_hook); larger blocks hand them to the fan-out pool, which writes them in parallel
#ifndef RSMI_PUT_HOOK_MAX_BLOCK
#define RSMI_PUT_HOOK_MAX_BLOCK 1048576
#endif
#ifndef RSMI_BATCH_CODEC_PLACE
#define RSMI_BATCH_CODEC_PLACE 0
#endif
// 0: no writes inside the codec call's wait (the blocks RSMI_PUT_HOOK_MAX_BLOCK covers write every
// shard after the call, round 5's order), for A/B library builds
#ifndef RSMI_PUT_WAIT_HOOK
#define RSMI_PUT_WAIT_HOOK 1
#endif
// 1 (default): a lone degraded Get copies the block's present data rows inside its decode call's
// wait (rsmi_set_wait_hook); 0: the whole block from the staging after the call (A/B builds)
#ifndef RSMI_GET_WAIT_HOOK
#define RSMI_GET_WAIT_HOOK 1
#endif
// 1: GetMany assembles its decoded blocks' present data rows from the fetched shards while the GPU
// rebuilds the missing ones (measured level, profiles/r06/ac; A/B builds); 0 (default): every block
// from the staging after the decode
#ifndef RSMI_GETMANY_PRESENT_OVERLAP
#define RSMI_GETMANY_PRESENT_OVERLAP 0
#endif

namespace rsmi {
namespace host {

const char* const kErrReadQuorum = "Read failed. Insufficient number of nodes online";  // error.go:12
const char* const kErrNodeNotFound = "node not found";                                   // error.go:9
static const char* const kErrNodeAccessDenied = "node access denied";                     // error.go:18
static const char* const kErrCanceled = "context canceled";

// ------------------------------------------------------------------ quorum helpers
namespace {

// paralleltask.Wait (parallel_task.go:59-84) applied to results in arrival order.
class QuorumWait {
public:
    QuorumWait(int success_quorum, int failure_quorum) : sq_(success_quorum), fq_(failure_quorum) {}
    // returns true once the outcome is decided
    bool add(const Status& s) {
        if (decided_) return true;
        if (s.ok()) {
            if (++succ_ >= sq_) decided_ = true;
        } else if (++fail_ >= fq_) {
            result_ = s;  // "return last error"
            decided_ = true;
        }
        return decided_;
    }
    bool decided() const { return decided_; }
    // if every task finished without reaching either quorum, Wait would block forever in Go
    // (all goroutines done); report it as the read/write quorum failure instead
    Status result(const char* undecided) const { return decided_ ? result_ : Status::Error(undecided); }

private:
    int sq_, fq_, succ_ = 0, fail_ = 0;
    bool decided_ = false;
    Status result_;
};

// task() on this thread inside the next codec call's wait (rsmi_set_wait_hook), or right after the
// call when the call did not take it, so it runs exactly once; an exception from task() is rethrown
// once the call has returned (none may cross the C-ABI), and one from call() leaves no hook behind
template <class Call>
int with_wait_task(const std::function<void()>& task, Call&& call) {
    struct Task {
        const std::function<void()>* fn;
        std::exception_ptr err;
        static void run(void* p) {
            auto* t = static_cast<Task*>(p);
            try {
                (*t->fn)();
            } catch (...) {
                t->err = std::current_exception();
            }
        }
    } t{&task, nullptr};
    struct Clear {
        ~Clear() { rsmi_set_wait_hook(nullptr, nullptr); }
    } clear;
    rsmi_set_wait_hook(&Task::run, &t);
    const int rc = call();
    rsmi_run_wait_hook();
    if (t.err) std::rethrow_exception(t.err);
    return rc;
}

}  // namespace

Status reduce_quorum_errs(const std::vector<Status>& errs, int quorum, const char* quorum_err) {
    std::vector<std::pair<std::string, int>> counts;  // first-occurrence order (Go: map order)
    for (const auto& e : errs) {
        if (e.err == kErrNodeNotFound || e.err == kErrNodeAccessDenied) continue;
        auto it = std::find_if(counts.begin(), counts.end(), [&](auto& p) { return p.first == e.err; });
        if (it == counts.end())
            counts.push_back({e.err, 1});
        else
            it->second++;
    }
    int max = 0;
    std::string max_err;
    for (auto& p : counts) {
        if (max < p.second) {
            max = p.second;
            max_err = p.first;
        } else if (max == p.second && p.first.empty()) {
            max_err.clear();  // prefer nil on ties (error.go:51-54)
        }
    }
    if (max >= quorum) return Status{max_err};
    return Status::Error(quorum_err);
}

Status find_meta_in_quorum(const std::vector<Meta>& metas, int quorum, Meta* out) {
    if (quorum < 2) return Status::Error(kErrReadQuorum);  // node.go:493-495
    // the reference hashes fmt.Sprint(BlockSize) with sha256; equal hashes <=> equal sizes
    std::vector<std::pair<int32_t, int>> counts;
    for (const auto& m : metas) {
        auto it = std::find_if(counts.begin(), counts.end(), [&](auto& p) { return p.first == m.block_size; });
        if (it == counts.end())
            counts.push_back({m.block_size, 1});
        else
            it->second++;
    }
    int max = 0;
    int32_t best = 0;
    for (auto& p : counts)
        if (p.second > max) {
            max = p.second;
            best = p.first;
        }
    if (max < quorum) return Status::Error(kErrReadQuorum);
    out->block_size = best;
    return Status::Ok();
}

// ------------------------------------------------------------------ construction
Status DagNode::New(const DagNodeConfig& cfg, std::vector<std::shared_ptr<DataNodeClient>> clients,
                    std::unique_ptr<DagNode>* out, int device) {
    return New(cfg, std::move(clients), out, std::vector<int>{device});
}

Status DagNode::New(const DagNodeConfig& cfg, std::vector<std::shared_ptr<DataNodeClient>> clients,
                    std::unique_ptr<DagNode>* out, const std::vector<int>& devices) {
    const size_t n = cfg.nodes.size();
    if (n != size_t(cfg.data_blocks + cfg.parity_blocks) || n == 0 || clients.size() != n)
        return Status::Error("dag node config is incorrect");  // node.go:55-57
    if (devices.empty() || devices.size() > size_t(kClusterSlots)) return Status::Error("dag node device list is empty");
    std::unique_ptr<DagNode> d(new DagNode());
    d->config_ = cfg;
    d->devices_ = devices;
    d->replicas_.assign(devices.size(), 0);
    for (size_t i = 0; i < devices.size(); i++)
        for (size_t j = 0; j < i; j++) d->replicas_[i] += devices[j] == devices[i];
    d->slots_.assign(kClusterSlots / 8, 0);
    for (auto& c : clients) d->nodes_.push_back(StorageNode{c, false});
    d->fan_.reset(new FanOut(int(n) - 1));  // the calling thread runs one share itself
    if (devices.size() > 1) d->member_fan_.reset(new FanOut(int(devices.size()) - 1));
    for (size_t i = 0; i < devices.size(); i++)  // the codec contexts, before the first call
        warm_contexts(cfg.data_blocks, cfg.parity_blocks, devices[i], d->replicas_[i]);
    *out = std::move(d);
    return Status::Ok();
}

int DagNode::MemberOfKey(const std::string& key) const {
    if (devices_.size() <= 1) return 0;
    const int slot = rsmi_key_slot(reinterpret_cast<const uint8_t*>(key.data()), key.size());
    if (slot < 0) return 0;
    return int(size_t(slot) * devices_.size() / size_t(kClusterSlots));  // as rsmi_group_member_of_key
}

rsmi_ctx* DagNode::member_ctx(int member, int* rc) const {
    return shared_context(config_.data_blocks, config_.parity_blocks, devices_[size_t(member)], rc,
                          replicas_[size_t(member)]);
}

Status DagNode::member_erasure(int member, int64_t block_size, Erasure* out) const {
    return Erasure::New(config_.data_blocks, config_.parity_blocks, block_size, out, devices_[size_t(member)],
                        replicas_[size_t(member)]);
}

DagNode::MemberOrder DagNode::member_order(size_t nb, const std::function<int(size_t)>& member_of_pos) const {
    MemberOrder o;
    const size_t M = devices_.size();
    o.perm.resize(nb);
    o.ranges.assign(M, {0, 0});
    if (M == 1) {
        for (size_t j = 0; j < nb; j++) o.perm[j] = j;
        o.ranges[0] = {0, nb};
        return o;
    }
    std::vector<int> mem(nb);
    for (size_t j = 0; j < nb; j++) {
        mem[j] = member_of_pos(j);
        o.ranges[size_t(mem[j])].second++;
    }
    for (size_t i = 1; i < M; i++) o.ranges[i].first = o.ranges[i - 1].first + o.ranges[i - 1].second;
    std::vector<size_t> next(M);
    for (size_t i = 0; i < M; i++) next[i] = o.ranges[i].first;
    for (size_t j = 0; j < nb; j++) o.perm[next[size_t(mem[j])]++] = j;
    return o;
}

int DagNode::code_members(const MemberOrder& order, const std::function<int(rsmi_ctx*, size_t, size_t)>& code) {
    std::vector<int> live;
    for (size_t i = 0; i < order.ranges.size(); i++)
        if (order.ranges[i].second) live.push_back(int(i));
    std::vector<int> rc(live.size(), RSMI_OK);
    auto one = [&](int t) {
        const int i = live[size_t(t)];
        rsmi_ctx* ctx = member_ctx(i, &rc[size_t(t)]);
        if (ctx) rc[size_t(t)] = code(ctx, order.ranges[size_t(i)].first, order.ranges[size_t(i)].second);
    };
    if (live.size() > 1 && member_fan_)
        member_fan_->run(int(live.size()), one);  // each member's call on its own thread
    else
        for (size_t t = 0; t < live.size(); t++) one(int(t));
    for (int r : rc)
        if (r != RSMI_OK) return r;
    return RSMI_OK;
}

void DagNode::fan(int count, const std::function<void(int)>& f, size_t shard_bytes) {
    if (parallel_ && fan_ && shard_bytes >= fanout_min_ && active_.load() <= 1)
        fan_->run(count, f);
    else
        for (int i = 0; i < count; i++) f(i);
}

void DagNode::fan_keys(int count, const std::function<void(int)>& f) {
    if (parallel_ && fan_ && active_.load() <= 1)
        fan_->run(count, f);
    else
        for (int i = 0; i < count; i++) f(i);
}


void DagNode::copy_bytes(uint8_t* dst, const uint8_t* src, size_t n) {
    // a lone caller's bulk copies into page-locked staging run on the idle fan-out pool (one core
    // copies ~10-20 GB/s, a few together saturate far more of the socket's bandwidth)
    // only for copies large enough to repay waking pool threads (a 256 KiB block copies in
    // ~15 us on one core, about what the hand-off costs); streaming stores from 1 MiB
    // (copy_to_staging), also in each part
    constexpr size_t kPart = size_t(256) << 10, kMin = size_t(1) << 20;
    const int parts = n < kMin ? 1 : int(std::min<size_t>(8, n / kPart));
    if (parts < 2 || !parallel_ || !fan_ || active_.load() > 1) {
        copy_to_staging(dst, src, n);
        return;
    }
    fan_->run(parts, [&](int t) {
        const size_t a = n * size_t(t) / size_t(parts), b = n * size_t(t + 1) / size_t(parts);
        if (b - a >= kMin / 8) copy_streaming(dst + a, src + a, b - a);
        else std::memcpy(dst + a, src + a, b - a);
    });
}

DagNode::~DagNode() { Close(); }

void DagNode::Close() {
    {
        std::lock_guard<std::mutex> g(q_mu_);
        stop_ = true;
    }
    q_cv_.notify_all();
    if (worker_.joinable()) worker_.join();
}

std::pair<int, int> DagNode::EntryQuorum() const {  // node.go:439-446
    int write_quorum = config_.data_blocks;
    if (config_.data_blocks == config_.parity_blocks) write_quorum++;
    return {config_.data_blocks, write_quorum};
}

bool DagNode::GetDataNodeState(int i) const {
    if (i < 0 || i >= int(nodes_.size())) throw std::out_of_range("input setIndex is illegal");  // log.Fatalf
    return nodes_[i].state;
}

bool DagNode::AddSlot(uint64_t slot) {
    if (slot >= uint64_t(kClusterSlots)) throw std::out_of_range("slot out of range");
    const bool old = slots_[slot / 8] >> (slot % 8) & 1;
    slots_[slot / 8] |= uint8_t(1u << (slot % 8));
    if (!old) num_slots_++;
    return old;
}

bool DagNode::ClearSlot(uint64_t slot) {
    if (slot >= uint64_t(kClusterSlots)) throw std::out_of_range("slot out of range");
    const bool old = slots_[slot / 8] >> (slot % 8) & 1;
    slots_[slot / 8] &= uint8_t(~(1u << (slot % 8)));
    if (old) num_slots_--;
    return old;
}

bool DagNode::GetSlot(uint64_t slot) const {
    if (slot >= uint64_t(kClusterSlots)) throw std::out_of_range("slot out of range");
    return slots_[slot / 8] >> (slot % 8) & 1;
}

void DagNode::HealthCheckAll() {
    for (auto& sn : nodes_) sn.state = sn.client->Healthy();
}

// ------------------------------------------------------------------ meta
Bytes DagNode::encode_meta(int32_t size) {
    Bytes b(4);
    for (int i = 0; i < 4; i++) b[i] = uint8_t(uint32_t(size) >> (8 * i));  // binary.LittleEndian
    return b;
}

uint16_t DagNode::entry_checksum(const Bytes& meta, size_t S, uint32_t raw) {
    // |meta size (4 LE)|data size (4 LE)|meta| precede the shard in the checksummed bytes
    Bytes head(8 + meta.size());
    for (int i = 0; i < 4; i++) {
        head[i] = uint8_t(uint32_t(meta.size()) >> (8 * i));
        head[4 + i] = uint8_t(uint32_t(S) >> (8 * i));
    }
    std::copy(meta.begin(), meta.end(), head.begin() + 8);
    return rsmi_crc16_entry(head.data(), head.size(), raw, S);
}

uint32_t DagNode::value_checksum(const Bytes& meta, size_t S, uint16_t crc16, uint32_t raw32) {
    // the whole entry |crc16 (4 LE)|meta size|data size|meta| precedes the shard in the value
    Bytes head(12 + meta.size());
    for (int i = 0; i < 4; i++) {
        head[i] = uint8_t(uint32_t(crc16) >> (8 * i));
        head[4 + i] = uint8_t(uint32_t(meta.size()) >> (8 * i));
        head[8 + i] = uint8_t(uint32_t(S) >> (8 * i));
    }
    std::copy(meta.begin(), meta.end(), head.begin() + 12);
    return rsmi_crc32_entry(head.data(), head.size(), raw32, S);
}

Status DagNode::get_meta_info(const std::string& key, Meta* meta, std::vector<StorageNode*>* online) {
    const size_t n = nodes_.size();
    std::vector<Meta> metas(n);
    std::vector<Status> errs(n);
    fan(int(n), [&](int i) {  // readAllMeta (node.go:450-489): one goroutine per datanode
        Bytes mb;
        Status s = nodes_[i].client->GetMeta(key, &mb);
        if (!s.ok()) {
            errs[i] = s;
            return;
        }
        if (mb.size() < 4) {
            errs[i] = Status::Error("unexpected EOF");
            return;
        }
        metas[i].block_size = int32_t(uint32_t(mb[0]) | uint32_t(mb[1]) << 8 | uint32_t(mb[2]) << 16 |
                                      uint32_t(mb[3]) << 24);
    }, last_shard_.load());  // GetMeta checks the whole entry's CRC: cost follows the shard size
    const int read_quorum = EntryQuorum().first;
    Status r = reduce_quorum_errs(errs, read_quorum, kErrReadQuorum);
    if (!r.ok()) return r;
    Status f = find_meta_in_quorum(metas, read_quorum, meta);
    if (!f.ok()) return f;
    if (online) {
        online->assign(n, nullptr);
        for (size_t i = 0; i < n; i++)
            if (metas[i].block_size == meta->block_size) (*online)[i] = &nodes_[i];
    }
    return Status::Ok();
}

Status DagNode::GetSize(const std::string& key, int* size) {
    Active act(active_);
    Meta meta;
    Status s = get_meta_info(key, &meta, nullptr);
    *size = meta.block_size;
    return s;
}

Status DagNode::Has(const std::string& key, bool* has) {
    int size;
    Status s = GetSize(key, &size);
    *has = s.ok();
    return s;
}

// ------------------------------------------------------------------ write path
Status DagNode::Put(const std::string& key, const Bytes& block) {  // node.go:358-408
    Active act(active_);
    const Bytes meta = encode_meta(int32_t(block.size()));
    const int member = MemberOfKey(key);
    Erasure enc;
    Status s = member_erasure(member, int64_t(block.size()), &enc);
    if (!s.ok()) return s;
    const int n = int(nodes_.size()), k = config_.data_blocks;
    const size_t S = size_t(enc.ShardSize());
    const int wq = EntryQuorum().second;
    std::vector<Status> res(nodes_.size());
    last_shard_ = S;
    auto quorum = [&] {
        QuorumWait w(wq, n - wq + 1);
        for (const Status& r : res) w.add(r);
        return w.result("Write failed. Insufficient number of nodes online");
    };
    if (block.empty()) {  // erasure.go:52-54: nil shards, no codec call
        fan(n, [&](int i) { res[i] = nodes_[i].client->Put(key, meta, ByteView(nullptr, 0)); }, 0);
        return quorum();
    }
    bool want32 = false;  // mutcask-backed datanodes keep a CRC-32 of every value as well
    for (auto& sn : nodes_) want32 |= gpu_checksums_ && gpu_value_checksums_ && sn.client->WantsValueChecksum();
    // Split into one page-locked buffer (coded there in place on the GPU), and each datanode gets
    // its shard as a view of it, as the Go slices alias Split's buffer
    uint8_t* flat = block_scratch(size_t(n) * S);
    if (!flat) return Status::Error("out of host memory");
    std::vector<uint32_t> raw(gpu_checksums_ ? size_t(n) : 0), raw32(want32 ? size_t(n) : 0);
    // a lone caller (nothing to coalesce with) spreads the copy over the idle fan-out pool and
    // codes the block with one zero-copy kernel; concurrent callers Split on their own thread and
    // meet in the engine's group commit
    const bool lone = lone_paths_ && active_.load() <= 1;
    if (lone) copy_bytes(flat, block.data(), block.size());
    else copy_to_staging(flat, block.data(), block.size());
    std::memset(flat + block.size(), 0, size_t(k) * S - block.size());  // Split zero-padding
    int rc = RSMI_OK;
    auto codec = [&] {
        const auto tc = PhaseClock::now();
        if (lone) {
            rsmi_ctx* ctx = member_ctx(member, &rc);
            if (ctx)
                rc = raw.empty() ? rsmi_encode_batch_host(ctx, flat, size_t(n) * S, flat + size_t(k) * S, size_t(n) * S, S, 1)
                                 : rsmi_encode_batch_host_crcs(ctx, flat, size_t(n) * S, flat + size_t(k) * S,
                                                               size_t(n) * S, S, 1, raw.data(),
                                                               raw32.empty() ? nullptr : raw32.data());
        } else {
            const Status e = enc.EncodeSplitFlat(block.size(), flat, raw.empty() ? nullptr : raw.data(),
                                                 raw32.empty() ? nullptr : raw32.data());
            rc = e.ok() ? RSMI_OK : RSMI_ERR_DEVICE;
            if (!e.ok()) s = e;
        }
        phase_add(Phase::Codec, tc);
    };
    // shard i to datanode i; with its entry checksum (and value checksum) from the GPU pass, or
    // the datanode computes them (sum = false)
    auto put_shard = [&](int i, bool sum) {
        DataNodeClient& cl = *nodes_[i].client;
        const ByteView shard(flat + size_t(i) * S, S);
        if (!sum || raw.empty()) {
            res[i] = cl.Put(key, meta, shard);
            return;
        }
        const uint16_t c16 = entry_checksum(meta, S, raw[i]);
        res[i] = !raw32.empty() && cl.WantsValueChecksum()
                     ? cl.PutWithChecksums(key, meta, shard, c16, value_checksum(meta, S, c16, raw32[i]))
                     : cl.PutWithChecksum(key, meta, shard, c16);
    };
    // The data rows that hold only block bytes are final once Split, so their datanode writes run
    // while the GPU encodes the parity (the datanodes checksum them).  The rest -- the row holding
    // the zero padding, which the engine's group commit rewrites, and the parity rows -- follow the
    // codec call, with the GPU's checksums.  Blocks up to RSMI_PUT_HOOK_MAX_BLOCK: the calling
    // thread writes those rows itself inside its codec call's wait -- the engine runs them between
    // the launch and the wait, or while another caller's batch codes the block
    // (rsmi_set_wait_hook) -- with no hand-off.  Larger blocks: the fan-out pool writes them in
    // parallel beside the codec call (one thread's sequential writes would outlast the encode).
    // Stored entries are the same either way; every outcome is replayed in node order
    // (DESIGN.md §5.3).
    const bool pool = RSMI_PUT_OVERLAP && block.size() > size_t(RSMI_PUT_HOOK_MAX_BLOCK);
    const int full = int(std::min<size_t>(size_t(k), block.size() / S));  // rows of block bytes only
    const int early = pool ? full : 0;
    const int hooked = RSMI_PUT_OVERLAP && RSMI_PUT_WAIT_HOOK && !pool ? full : 0;
    if (early > 0 && fan_) {
        fan_->run(2, [&](int t) {
            if (t == 0) {
                codec();
                return;
            }
            const auto tp = PhaseClock::now();
            fan(early, [&](int i) { put_shard(i, false); }, S);
            phase_add(Phase::Put, tp);
        });
    } else if (hooked > 0) {
        with_wait_task(
            [&] {
                // one after another (through the node fan-out instead: level)
                const auto tp = PhaseClock::now();
                for (int i = 0; i < hooked; i++) put_shard(i, false);
                phase_add(Phase::Put, tp);
            },
            [&] {
                codec();
                return rc;
            });
    } else {
        codec();
    }
    if (rc) {
        // the codec failed: the error is returned (node.go:382-386) and the data shards already
        // written stay, as the reference leaves the shards of a Put whose write quorum fails
        // (node.go:389-407).  They hold exactly the bytes a successful Put stores.  Deleting them
        // instead would destroy the shards of a block stored earlier under the same key (keys are
        // content ids, so a repeated Put rewrites identical shards).
        return s.ok() ? rsmi_status(rc) : s;
    }
    const auto t1 = PhaseClock::now();
    const int first = early + hooked;  // the rows still to write
    fan(n - first, [&](int t) { put_shard(first + t, true); }, S);  // one goroutine per datanode, no cancel
    phase_add(Phase::Put, t1);
    return quorum();
}

Status DagNode::PutMany(const std::vector<std::string>& keys, const std::vector<Bytes>& blocks) {
    Active act(active_);
    if (keys.size() != blocks.size()) return Status::Error("keys and blocks differ in length");
    const int k = config_.data_blocks, m = config_.parity_blocks, n = k + m;
    std::vector<Status> results(blocks.size());
    // group equal-size blocks: one GPU batch encode per size, then the per-block fan-out
    std::map<size_t, std::vector<size_t>> groups;
    for (size_t i = 0; i < blocks.size(); i++) groups[blocks[i].size()].push_back(i);
    for (auto& g : groups) {
        const size_t B = g.first;
        if (B == 0 || g.second.size() == 1) {
            for (size_t i : g.second) results[i] = Put(keys[i], blocks[i]);
            continue;
        }
        const size_t S = rsmi_shard_size(B, k);
        // Two halves of the thread's staging: a chunk is staged into one half, then a helper task
        // runs its codec call and its datanode writes while the next chunk is staged into the other
        // half (the codec call overlaps the next staging copy, the writes the next codec call).  A
        // chunk joins the previous chunk's task before it hands over its own, and the group joins
        // the last before the next group (or the return), so every block's outcome is the
        // sequential loop's.
        const size_t chunk = std::max<size_t>(1, staging_blocks(size_t(n) * S) / (RSMI_BATCH_SERIAL ? 1 : 2));
        const size_t half = std::min(chunk, g.second.size()) * size_t(n) * S;
        const Bytes meta = encode_meta(int32_t(B));
        const int wq = EntryQuorum().second;
        // datanodes over mutcask keep a CRC-32 of every value: the GPU pass supplies it too when
        // asked (SetGpuValueChecksums), else each datanode folds its own
        bool want32 = false;
        for (auto& sn : nodes_) want32 |= gpu_value_checksums_ && sn.client->WantsValueChecksum();
        uint8_t* base = thread_staging().reserve(2 * half);
        if (!base) {
            for (size_t i : g.second) results[i] = Status::Error("out of host memory");
            continue;
        }
        std::future<void> writing;
        auto join_writes = [&] {
            if (writing.valid()) writing.get();
        };
        int cur = 0;
        // the previous chunk's staging and write times, for the codec call's placement
        int64_t last_stage = 0;
        auto last_writes = std::make_shared<std::atomic<int64_t>>(0);
        for (size_t c0 = 0; c0 < g.second.size(); c0 += chunk) {
            const size_t nb = std::min(chunk, g.second.size() - c0);
            // the chunk's blocks ordered by member (a device list): each member codes one range
            MemberOrder ord = member_order(nb, [&](size_t j) { return MemberOfKey(keys[g.second[c0 + j]]); });
            {
                std::vector<size_t> tmp(nb);
                for (size_t j = 0; j < nb; j++) tmp[j] = g.second[c0 + ord.perm[j]];
                std::copy(tmp.begin(), tmp.end(), g.second.begin() + long(c0));
            }
            const size_t* idx = g.second.data() + c0;
            // per block: k data rows (Split, zero-padded) + m parity rows
            const auto t0 = PhaseClock::now();
            uint8_t* flat = base + (cur ? half : 0);
            fan_keys(int(std::min<size_t>(nb, 16)), [&](int t) {
                for (size_t j = size_t(t); j < nb; j += std::min<size_t>(nb, 16)) {
                    std::memcpy(flat + j * n * S, blocks[idx[j]].data(), B);
                    std::memset(flat + j * n * S + B, 0, size_t(k) * S - B);
                }
            });
            phase_add(Phase::Stage, t0);
            last_stage = std::chrono::duration_cast<std::chrono::nanoseconds>(PhaseClock::now() - t0).count();
            // the chunk's codec call: here or as the task's first step (RSMI_BATCH_CODEC_PLACE)
            auto raw = std::make_shared<std::vector<uint32_t>>(gpu_checksums_ ? nb * size_t(n) : 0);
            auto raw32 = std::make_shared<std::vector<uint32_t>>(want32 ? nb * size_t(n) : 0);
            auto code = [this, flat, S, k, n, want32, raw, raw32, ord = std::make_shared<MemberOrder>(std::move(ord))] {
                const auto t1 = PhaseClock::now();
                const int rc = code_members(*ord, [&](rsmi_ctx* ctx, size_t j0, size_t cnt) {
                    uint8_t* f = flat + j0 * size_t(n) * S;
                    if (!gpu_checksums_)
                        return rsmi_encode_batch_host(ctx, f, size_t(n) * S, f + size_t(k) * S, size_t(n) * S, S, cnt);
                    return rsmi_encode_batch_host_crcs(ctx, f, size_t(n) * S, f + size_t(k) * S, size_t(n) * S, S, cnt,
                                                       raw->data() + j0 * size_t(n),
                                                       want32 ? raw32->data() + j0 * size_t(n) : nullptr);
                });
                phase_add(Phase::Codec, t1);
                return rc;
            };
            const bool inline_codec = RSMI_BATCH_CODEC_PLACE == 1 ||
                                      (RSMI_BATCH_CODEC_PLACE == 0 && last_writes->load() > last_stage);
            const int pre = inline_codec ? code() : RSMI_OK;
            join_writes();  // the previous chunk's task ends before this one starts
            // the codec call, then the blocks' datanode writes (the reference's concurrent Puts),
            // each with its own node fan-out, each shard a view of the staging
            writing = std::async(std::launch::async, [this, &keys, &results, &meta, idx, nb, flat, S, n, wq, want32,
                                                      code, pre, inline_codec, raw, raw32, last_writes] {
                const int rc = inline_codec ? pre : code();
                if (rc) {
                    for (size_t j = 0; j < nb; j++) results[idx[j]] = rsmi_status(rc);
                    return;
                }
                const auto t2 = PhaseClock::now();
                fan_keys(int(nb), [&](int j) {
                    const uint8_t* bb = flat + size_t(j) * n * S;
                    std::vector<Status> res(static_cast<size_t>(n));
                    fan(n, [&](int i) {
                        const ByteView shard(bb + size_t(i) * S, S);
                        DataNodeClient& cl = *nodes_[i].client;
                        if (!gpu_checksums_) {
                            res[i] = cl.Put(keys[idx[j]], meta, shard);
                            return;
                        }
                        const uint16_t c16 = entry_checksum(meta, S, (*raw)[j * n + i]);
                        res[i] = want32 && cl.WantsValueChecksum()
                                     ? cl.PutWithChecksums(keys[idx[j]], meta, shard, c16,
                                                           value_checksum(meta, S, c16, (*raw32)[j * n + i]))
                                     : cl.PutWithChecksum(keys[idx[j]], meta, shard, c16);
                    }, S);
                    QuorumWait w(wq, n - wq + 1);
                    for (const Status& r : res) w.add(r);
                    results[idx[j]] = w.result("Write failed. Insufficient number of nodes online");
                });
                phase_add(Phase::Put, t2);
                last_writes->store(std::chrono::duration_cast<std::chrono::nanoseconds>(PhaseClock::now() - t2).count());
            });
            cur ^= 1;
            if (RSMI_BATCH_SERIAL) join_writes();
        }
        join_writes();
    }
    // node.go:411-416 returns the error of the last Put
    return results.empty() ? Status::Ok() : results.back();
}

Status DagNode::DeleteBlock(const std::string& key) {  // node.go:191-208
    Active act(active_);
    const int wq = EntryQuorum().second;
    std::vector<Status> res(nodes_.size());
    fan(int(nodes_.size()), [&](int i) { res[i] = nodes_[i].client->Delete(key); }, 0);  // cheap: stays serial
    QuorumWait w(wq, int(nodes_.size()) - wq + 1);
    for (const Status& r : res) w.add(r);
    return w.result("Write failed. Insufficient number of nodes online");
}

// ------------------------------------------------------------------ read path
Status DagNode::fetch_for_get(const std::string& key, Fetched* f, bool defer_verify) {  // node.go:220-275
    std::vector<StorageNode*> online;
    f->member = MemberOfKey(key);
    Status s = get_meta_info(key, &f->meta, &online);
    if (!s.ok()) return s;
    const int n = int(nodes_.size()), rq = EntryQuorum().first;
    f->shards.assign(static_cast<size_t>(n), Bytes());
    f->repair.clear();
    QuorumWait w(rq, n - rq + 1);
    // Node i's fetch result, replayed in node order exactly as the sequential loop would use
    // it.  Fetches run concurrently in waves: when node i is reached unfetched, the next
    // (successes still needed) online nodes are fetched at once.  A fetch the replay never
    // reaches (the quorum was decided first) is a cancelled goroutine: dropped, no repair.
    std::vector<Bytes> data(static_cast<size_t>(n)), metas(static_cast<size_t>(n));
    std::vector<Status> got(static_cast<size_t>(n));
    std::vector<DataNodeClient::Stored> stored(static_cast<size_t>(n));
    std::vector<char> fetched(static_cast<size_t>(n), 0);
    int succ = 0;
    for (int i = 0; i < n; i++) {
        if (!online[i]) {
            // runs even after the quorum is met: the goroutine returns before its first RPC
            if (nodes_[i].state) f->repair.push_back(i);
            w.add(Status::Error("offline node"));
            continue;
        }
        if (w.decided()) continue;  // cancelOther: later fetches are cancelled, no repair
        if (!fetched[i]) {
            std::vector<int> wave;
            for (int j = i; j < n && int(wave.size()) < std::max(1, rq - succ); j++)
                if (online[j] && !fetched[j]) wave.push_back(j);
            fan(int(wave.size()), [&](int t) {
                const int j = wave[t];
                got[j] = gpu_verified_reads_ ? online[j]->client->GetForVerify(key, &metas[j], &data[j], &stored[j])
                                             : online[j]->client->Get(key, &metas[j], &data[j]);
            }, size_t(ceil_frac(f->meta.block_size, config_.data_blocks)));
            if (gpu_verified_reads_ && !defer_verify) verify_wave(f->member, wave, metas, data, stored, got);
            for (int j : wave) fetched[j] = 1;
        }
        if (!got[i].ok()) {
            f->repair.push_back(i);  // any non-cancel error (node.go:254-258)
        } else {
            f->shards[i] = std::move(data[i]);
            succ++;
        }
        w.add(got[i]);
    }
    std::sort(f->repair.begin(), f->repair.end());
    if (gpu_verified_reads_ && defer_verify) {
        f->metas = std::move(metas);
        f->stored = std::move(stored);
    }
    return w.result(kErrReadQuorum);
}

void DagNode::verify_fetched(std::vector<Fetched>& fs, const std::vector<Status>& st, const std::vector<char>& skip,
                             std::vector<char>* bad) {
    bad->assign(fs.size(), 0);
    // (key, node) of every accepted shard with a stored checksum to check, by (shard size, the
    // key's member)
    std::map<std::pair<size_t, int>, std::vector<std::pair<size_t, int>>> by_size;
    for (size_t q = 0; q < fs.size(); q++) {
        if (!st[q].ok() || fs[q].stored.empty() || skip[q]) continue;
        for (size_t i = 0; i < fs[q].shards.size(); i++)
            if (!fs[q].shards[i].empty() && !fs[q].stored[i].verified)
                by_size[{fs[q].shards[i].size(), fs[q].member}].push_back({q, int(i)});
    }
    for (auto& g : by_size) {
        const size_t S = g.first.first, w = g.second.size();
        bool want32 = false;
        for (auto& e : g.second) want32 |= fs[e.first].stored[size_t(e.second)].has_value_crc;
        std::vector<uint32_t> r16(w, 0), r32(w, 0);
        int rc = RSMI_OK;
        rsmi_ctx* ctx = member_ctx(g.first.second, &rc);
        // rows gathered into page-locked staging by the key pool, then read in place by one GPU
        // pass (staging_blocks bounds the buffer; a huge GetMany takes several passes)
        const size_t per = std::max<size_t>(1, kStagingBytes / S);
        for (size_t r0 = 0; ctx && r0 < w && rc == RSMI_OK; r0 += per) {
            const size_t nr = std::min(per, w - r0);
            uint8_t* flat = thread_staging().reserve(nr * S);
            if (!flat) {
                rc = RSMI_ERR_DEVICE;
                break;
            }
            const int parts = int(std::min<size_t>(nr, 64));
            fan_keys(parts, [&](int t) {
                for (size_t i = size_t(t); i < nr; i += size_t(parts)) {
                    const auto& e = g.second[r0 + i];
                    std::memcpy(flat + i * S, fs[e.first].shards[size_t(e.second)].data(), S);
                }
            });
            rc = rsmi_crc_rows_host(ctx, flat, S, nr, S, r16.data() + r0, want32 ? r32.data() + r0 : nullptr);
        }
        for (size_t i = 0; i < w; i++) {
            const size_t q = g.second[i].first, j = size_t(g.second[i].second);
            const Bytes& meta = fs[q].metas[j];
            const DataNodeClient::Stored& sd = fs[q].stored[j];
            // no device: the read fails loudly, through the per-key path (there is no CPU path)
            if (rc || (sd.has_value_crc && value_checksum(meta, S, sd.crc, r32[i]) != sd.value_crc) ||
                entry_checksum(meta, S, r16[i]) != sd.crc)
                (*bad)[q] = 1;
        }
    }
}

void DagNode::verify_wave(int member, const std::vector<int>& wave, const std::vector<Bytes>& metas,
                          const std::vector<Bytes>& data, const std::vector<DataNodeClient::Stored>& stored,
                          std::vector<Status>& got) {
    // shards to check, grouped by size (one GPU call per size; a block's shards share one)
    std::map<size_t, std::vector<int>> by_size;
    for (int j : wave)
        if (got[j].ok() && !stored[j].verified) by_size[data[j].size()].push_back(j);
    for (auto& g : by_size) {
        const size_t S = g.first, w = g.second.size();
        bool want32 = false;
        for (int j : g.second) want32 |= stored[j].has_value_crc;
        std::vector<uint32_t> r16(w, 0), r32(w, 0);
        int rc = RSMI_OK;
        if (S > 0) {
            rsmi_ctx* ctx = member_ctx(member, &rc);
            uint8_t* flat = ctx ? thread_staging().reserve(w * S) : nullptr;
            if (ctx && !flat) rc = RSMI_ERR_DEVICE;
            if (flat) {
                for (size_t i = 0; i < w; i++) std::memcpy(flat + i * S, data[g.second[i]].data(), S);
                rc = rsmi_crc_rows_host(ctx, flat, S, w, S, r16.data(), want32 ? r32.data() : nullptr);
            }
        }
        for (size_t i = 0; i < w; i++) {
            const int j = g.second[i];
            if (rc) {  // no device: the read fails loudly (there is no CPU path)
                got[j] = rsmi_status(rc);
                continue;
            }
            // the mutcask engine checks its value first (cask.go:250), then the datanode its entry
            if (stored[j].has_value_crc && value_checksum(metas[j], S, stored[j].crc, r32[i]) != stored[j].value_crc)
                got[j] = Status::Error("mutcask: data may be rotted");
            else if (entry_checksum(metas[j], S, r16[i]) != stored[j].crc)
                got[j] = Status::Error("checking crc failed");
        }
    }
}

// A lone caller's degraded read: DecodeDataBlocks (erasure.go:70-83) with the survivors copied
// into the page-locked block scratch over the fan-out pool, the missing data rows rebuilt there
// in place by one zero-copy kernel, and the block (the first BlockSize bytes of the k data rows,
// node.go:311-319) taken straight from it.  *done = false leaves the call to the per-shard path:
// nothing to decode, or shard lengths that are not the block's shard size; every error the
// per-shard path would return (rsmi_check_shards, the decode) is returned the same way.
Status DagNode::decode_into_block(const std::string& key, Fetched& f, size_t S, Bytes* block, bool* done) {
    *done = false;
    const int k = config_.data_blocks, n = int(f.shards.size());
    if (n != int(nodes_.size())) return Status::Ok();
    bool any_empty = false, all_empty = true, data_missing = false;
    for (int i = 0; i < n; i++) {
        any_empty |= f.shards[i].empty();
        all_empty &= f.shards[i].empty();
        data_missing |= i < k && f.shards[i].empty();
    }
    if (!any_empty || all_empty || !data_missing) return Status::Ok();  // no decode runs
    std::vector<size_t> lens(static_cast<size_t>(n));
    std::vector<uint8_t> present(static_cast<size_t>(n));
    for (int i = 0; i < n; i++) {
        lens[i] = f.shards[i].size();
        present[i] = f.shards[i].empty() ? 0 : 1;
    }
    size_t S2 = 0;
    int rc = rsmi_check_shards(n, lens.data(), 1, &S2);
    if (rc) return rsmi_status(rc);
    if (S2 != S || S == 0) return Status::Ok();
    int np = 0;
    for (int i = 0; i < n; i++) np += present[i];
    if (np < k) return rsmi_status(RSMI_ERR_TOO_FEW_SHARDS);
    rsmi_ctx* ctx = member_ctx(MemberOfKey(key), &rc);
    if (!ctx) return rsmi_status(rc);
    uint8_t* flat = block_scratch(size_t(n) * S);
    if (!flat) return Status::Error("out of host memory");
    // the survivors the decode reads (the first k present) are the only rows it needs
    const bool stream = size_t(k) * S >= (size_t(1) << 20);  // as Erasure's staging of the survivors
    for (int i = 0, used = 0; i < n && used < k; i++)
        if (present[i]) {
            if (stream && S < (size_t(1) << 20)) copy_streaming(flat + size_t(i) * S, f.shards[i].data(), S);
            else copy_bytes(flat + size_t(i) * S, f.shards[i].data(), S);
            used++;
        }
    // the block (the first BlockSize bytes of the k data rows): the present data rows straight from
    // the fetched shards while the GPU rebuilds the missing ones (rsmi_set_wait_hook; not from the
    // staging, whose lines the kernel is reading over PCIe), then the rebuilt rows
    const size_t bs = size_t(f.meta.block_size);
    if (RSMI_GET_WAIT_HOOK) {
        rc = with_wait_task(
            [&] {
                // row by row, so only the missing rows' places are zero-filled before they arrive
                block->clear();
                block->reserve(bs);
                for (int i = 0; i < k && block->size() < bs; i++) {
                    const size_t take = std::min(S, bs - block->size());
                    if (present[i])
                        block->insert(block->end(), f.shards[i].begin(), f.shards[i].begin() + long(take));
                    else
                        block->resize(block->size() + take);
                }
            },
            [&] { return rsmi_reconstruct_batch_host(ctx, flat, size_t(n) * S, S, 1, present.data(), 1); });
        if (rc) return rsmi_status(rc);
        for (int i = 0; i < k && size_t(i) * S < bs; i++)  // the rebuilt rows into their places
            if (!present[i]) std::memcpy(block->data() + size_t(i) * S, flat + size_t(i) * S, std::min(S, bs - size_t(i) * S));
    } else {
        rc = rsmi_reconstruct_batch_host(ctx, flat, size_t(n) * S, S, 1, present.data(), 1);
        if (rc) return rsmi_status(rc);
        block->assign(flat, flat + std::min(bs, size_t(k) * S));
        block->resize(bs);
    }
    *done = true;
    return Status::Ok();
}

Status DagNode::finish_get(const std::string& key, Fetched& f, Bytes* block) {  // node.go:277-326
    Erasure enc;
    Status s = member_erasure(MemberOfKey(key), f.meta.block_size, &enc);
    if (!s.ok()) return s;
    const size_t S = size_t(enc.ShardSize());
    bool done = f.assembled;  // GetMany's batch decode already wrote the block
    if (!done && lone_paths_ && active_.load() <= 1 && (s = decode_into_block(key, f, S, block, &done), !s.ok()))
        return s;
    if (!done) {
        s = enc.DecodeDataBlocks(f.shards);
        if (!s.ok()) return s;
        // the first k shards concatenated and truncated to BlockSize (node.go:311-319), copied
        // once (no zero fill of the whole block first)
        const size_t bs = size_t(f.meta.block_size);
        block->clear();
        block->reserve(bs);
        for (int i = 0; i < config_.data_blocks && block->size() < bs; i++) {
            const size_t take = std::min(bs - block->size(), std::min(S, f.shards[i].size()));
            block->insert(block->end(), f.shards[i].begin(), f.shards[i].begin() + long(take));
            if (take < S && block->size() < bs) block->resize(std::min(bs, block->size() + (S - take)), 0);
        }
        block->resize(bs);
    }
    if (!f.repair.empty()) {  // the shards move into the task: `f` is spent after this
        const int32_t bs = f.meta.block_size;
        std::lock_guard<std::mutex> g(q_mu_);
        if (repair_queue_.size() < kRepairQueueCap) {  // else: "repair queue is full, discard this task"
            auto shards = std::make_shared<std::vector<Bytes>>(std::move(f.shards));
            repair_queue_.push_back([this, key, bs, shards, idx = std::move(f.repair)]() {
                (void)repair_block(key, bs, std::move(*shards), idx);
            });
        }
        q_cv_.notify_one();
    }
    return Status::Ok();
}

Status DagNode::Get(const std::string& key, Bytes* block) {
    if (gpu_verified_reads_) {
        // one key through GetMany's path (which holds the Active guard, so a lone caller keeps
        // its node fan-out): the shards are fetched unchecked, and a degraded read's survivors
        // are checked by the decode kernel itself (one GPU call, not one per fetch wave plus the
        // decode); quorum, repair list and errors are Get's (see GetMany)
        std::vector<Bytes> blocks;
        std::vector<Status> st;
        GetMany({key}, &blocks, &st, 1);
        if (st[0].ok()) *block = std::move(blocks[0]);
        return st[0];
    }
    Active act(active_);
    const auto t0 = PhaseClock::now();
    Fetched f;
    Status s = fetch_for_get(key, &f);
    phase_add(Phase::Fetch, t0);
    if (!s.ok()) return s;
    const auto t1 = PhaseClock::now();
    s = finish_get(key, f, block);  // the decode (survivors staged, codec call) and the block
    phase_add(Phase::Codec, t1);
    return s;
}

void DagNode::GetMany(const std::vector<std::string>& keys, std::vector<Bytes>* blocks, std::vector<Status>* statuses,
                      size_t batch) {
    Active act(active_);
    const int k = config_.data_blocks, m = config_.parity_blocks, n = k + m;
    if (batch == 0) batch = 1;
    blocks->assign(keys.size(), Bytes());
    statuses->assign(keys.size(), Status());
    // `batch` keys at a time: fetched shards are held for the current chunk and the next.  The
    // keys' fetches run concurrently, like the reference's concurrent Gets (one goroutine per dag
    // pool request), each with its own node fan-out, and the next chunk's fetch runs on a helper
    // thread while this one is checked, decoded and assembled (the GPU decode leaves the cores to
    // it); fetches only read, so fetching one chunk ahead changes no key's outcome.
    // With GPU-verified reads, the first waves of all keys are checked together: one GPU
    // pass per shard size instead of one per key and wave.  A key with a bad shard runs the
    // per-key fetch again (checked wave by wave), so quorum, repair list and errors are
    // exactly Get's; its first attempt only read.
    struct Chunk {
        std::vector<Fetched> fs;
        std::vector<Status> st;
    };
    auto fetch_chunk = [this, &keys](size_t c0, size_t cn) {
        const auto t0 = PhaseClock::now();
        Chunk c;
        c.fs.resize(cn);
        c.st.resize(cn);
        fan_keys(int(cn), [&](int q) { c.st[size_t(q)] = fetch_for_get(keys[c0 + size_t(q)], &c.fs[size_t(q)], true); });
        phase_add(Phase::Fetch, t0);
        return c;
    };
    // the first chunk on this thread (a one-key GetMany is Get: no helper thread), later ones
    // fetched ahead
    std::future<Chunk> ahead;
    for (size_t k0 = 0; k0 < keys.size(); k0 += batch) {
        const size_t nk = std::min(batch, keys.size() - k0);
        Chunk cur = k0 == 0 || RSMI_BATCH_SERIAL ? fetch_chunk(k0, nk) : ahead.get();
        if (k0 + batch < keys.size() && !RSMI_BATCH_SERIAL)
            ahead = std::async(std::launch::async, fetch_chunk, k0 + batch, std::min(batch, keys.size() - k0 - batch));
        std::vector<Fetched>& fs = cur.fs;
        for (size_t q = 0; q < nk; q++) (*statuses)[k0 + q] = std::move(cur.st[q]);
        // does key q's data need the batched decode below (else the per-key path decides)
        auto needs_decode = [&](size_t q) {
            if (!(*statuses)[k0 + q].ok() || fs[q].meta.block_size <= 0) return false;
            bool data_missing = false, any = false;
            for (int c = 0; c < k; c++) data_missing |= fs[q].shards[c].empty();
            for (auto& sh : fs[q].shards) any |= !sh.empty();
            return data_missing && any;
        };
        // keys whose check rides on the batched decode: exactly k survivors (the decode reads
        // them all) and entry checksums only (the decode kernel yields R, not R32)
        std::vector<char> fused(nk, 0), redo_after(nk, 0);
        auto refetch = [&](const std::vector<char>& mask) {
            std::vector<int> redo;
            for (size_t q = 0; q < nk; q++)
                if (mask[q]) redo.push_back(int(q));
            fan_keys(int(redo.size()), [&](int t) {
                const size_t q = size_t(redo[size_t(t)]);
                fs[q] = Fetched();
                (*statuses)[k0 + q] = fetch_for_get(keys[k0 + q], &fs[q]);
            });
        };
        if (gpu_verified_reads_) {
            for (size_t q = 0; q < nk; q++) {
                if (!needs_decode(q) || fs[q].stored.empty()) continue;
                int np = 0;
                bool r32 = false;
                for (int c = 0; c < n; c++)
                    if (!fs[q].shards[c].empty()) {
                        np++;
                        r32 |= fs[q].stored[c].has_value_crc;
                    }
                fused[q] = np == k && !r32;
            }
            std::vector<Status> st(statuses->begin() + long(k0), statuses->begin() + long(k0 + nk));
            std::vector<char> bad;
            verify_fetched(fs, st, fused, &bad);
            refetch(bad);
        }
        // (block size, survivor pattern) -> chunk positions of keys whose data shards need decoding
        std::map<std::pair<int32_t, std::string>, std::vector<size_t>> groups;
        for (size_t q = 0; q < nk; q++) {
            if (!needs_decode(q)) {
                if (fused[q]) redo_after[q] = 1;  // cannot happen; checked the per-key way regardless
                continue;
            }
            std::string pat(static_cast<size_t>(n), '0');
            for (int c = 0; c < n; c++) pat[c] = fs[q].shards[c].empty() ? '0' : '1';
            groups[{fs[q].meta.block_size, pat}].push_back(q);
        }
        // a fused key whose decode did not run is checked by a per-key fetch again
        auto unchecked = [&](const std::vector<size_t>& qs, size_t b0, size_t nb) {
            for (size_t j = b0; j < b0 + nb; j++) redo_after[qs[j]] |= fused[qs[j]];
        };
        for (auto& g : groups) {
            const size_t S = rsmi_shard_size(size_t(g.first.first), k);
            std::vector<uint8_t> present(static_cast<size_t>(n));
            for (int c = 0; c < n; c++) present[c] = uint8_t(g.first.second[c] == '1');
            bool sizes_ok = true;  // every present shard must have the common size (else per-key errors)
            for (size_t q : g.second)
                for (int c = 0; c < n; c++) sizes_ok &= !present[c] || fs[q].shards[c].size() == S;
            if (!sizes_ok) {  // finish_get reports the size error per key
                unchecked(g.second, 0, g.second.size());
                continue;
            }
            bool verify = false;
            for (size_t q : g.second) verify |= fused[q] != 0;
            std::vector<int> used;  // the survivors the decode reads, as rsmi_reconstruct_batch_host_verify
            for (int c = 0; c < n && int(used.size()) < k; c++)
                if (present[c]) used.push_back(c);
            const size_t chunk = staging_blocks(size_t(n) * S);
            std::vector<uint32_t> r16(verify ? chunk * size_t(k) : 0);
            for (size_t b0 = 0; b0 < g.second.size(); b0 += chunk) {
                const size_t nb = std::min(chunk, g.second.size() - b0);
                // the chunk's keys ordered by member (a device list): each member decodes one range
                const MemberOrder ord = member_order(nb, [&](size_t j) { return fs[g.second[b0 + j]].member; });
                {
                    std::vector<size_t> tmp(nb);
                    for (size_t j = 0; j < nb; j++) tmp[j] = g.second[b0 + ord.perm[j]];
                    std::copy(tmp.begin(), tmp.end(), g.second.begin() + long(b0));
                }
                const auto ts = PhaseClock::now();
                uint8_t* flat = thread_staging().reserve(nb * size_t(n) * S);  // missing rows: don't-care bytes
                if (!flat) {
                    unchecked(g.second, b0, nb);
                    continue;
                }
                fan_keys(int(nb), [&](int j) {
                    for (int c = 0; c < n; c++)
                        if (present[c]) std::memcpy(flat + (j * n + c) * S, fs[g.second[b0 + j]].shards[c].data(), S);
                });
                phase_add(Phase::Stage, ts);
                // without verified reads (no key can be refetched), the blocks' present data rows go
                // in straight from the fetched shards on the key pool while the GPU rebuilds the
                // missing ones, row by row as in a lone Get (not from the staging, whose lines the
                // decode is reading over PCIe); the rebuilt rows follow the decode
                const bool rows_ahead = RSMI_GETMANY_PRESENT_OVERLAP && !verify;
                std::future<void> pre;
                if (rows_ahead)
                    pre = std::async(std::launch::async, [&, b0, nb] {
                        const auto tp = PhaseClock::now();
                        fan_keys(int(nb), [&](int j) {
                            const size_t q = g.second[b0 + size_t(j)];
                            Bytes& blk = (*blocks)[k0 + q];
                            const size_t bs = size_t(fs[q].meta.block_size);
                            blk.clear();
                            blk.reserve(bs);
                            for (int c = 0; c < k && blk.size() < bs; c++) {
                                const size_t take = std::min(S, bs - blk.size());
                                if (present[c])
                                    blk.insert(blk.end(), fs[q].shards[c].begin(), fs[q].shards[c].begin() + long(take));
                                else
                                    blk.resize(blk.size() + take);
                            }
                        });
                        phase_add(Phase::Stage, tp);
                    });
                const auto tc = PhaseClock::now();
                // with verified reads the same kernel returns R of every survivor it read
                const int drc = code_members(ord, [&](rsmi_ctx* ctx, size_t j0, size_t cnt) {
                    uint8_t* f = flat + j0 * size_t(n) * S;
                    return verify ? rsmi_reconstruct_batch_host_verify(ctx, f, size_t(n) * S, S, cnt, present.data(), 1,
                                                                       r16.data() + j0 * size_t(k))
                                  : rsmi_reconstruct_batch_host(ctx, f, size_t(n) * S, S, cnt, present.data(), 1);
                });
                phase_add(Phase::Codec, tc);
                if (pre.valid()) pre.get();
                if (drc != RSMI_OK) {  // finish_get reports a device error per key (and rewrites the block)
                    unchecked(g.second, b0, nb);
                    continue;  // leave these keys to the per-key path
                }
                for (size_t j = 0; verify && j < nb; j++) {
                    const size_t q = g.second[b0 + j];
                    if (!fused[q]) continue;
                    for (int c = 0; c < k; c++) {
                        const size_t i = size_t(used[size_t(c)]);
                        const DataNodeClient::Stored& sd = fs[q].stored[i];
                        if (!sd.verified && entry_checksum(fs[q].metas[i], S, r16[j * size_t(k) + size_t(c)]) != sd.crc)
                            redo_after[q] = 1;
                    }
                }
                // each block straight from the staging (its k data rows are the Split buffer: the
                // first BlockSize bytes, node.go:311-319), without copying the rebuilt rows into
                // the key's shards first; a key to be fetched again keeps nothing from here
                const auto ta = PhaseClock::now();
                fan_keys(int(nb), [&](int j) {
                    const size_t q = g.second[b0 + j];
                    if (redo_after[q]) return;
                    const uint8_t* base = flat + size_t(j) * n * S;
                    const size_t bs = size_t(fs[q].meta.block_size);
                    if (rows_ahead) {  // the rebuilt rows only
                        for (int c = 0; c < k && size_t(c) * S < bs; c++)
                            if (!present[c])
                                std::memcpy((*blocks)[k0 + q].data() + size_t(c) * S, base + size_t(c) * S,
                                            std::min(S, bs - size_t(c) * S));
                    } else {
                        (*blocks)[k0 + q].assign(base, base + bs);
                    }
                    fs[q].assembled = true;
                });
                phase_add(Phase::Stage, ta);  // the assembly copies count as staging
            }
        }
        // a bad survivor: that key's fetch again, checked wave by wave (quorum, repair list and
        // errors exactly Get's, as above)
        refetch(redo_after);
        fan_keys(int(nk), [&](int q) {
            if ((*statuses)[k0 + q].ok()) (*statuses)[k0 + q] = finish_get(keys[k0 + q], fs[q], &(*blocks)[k0 + q]);
        });
    }
}

void MigrateBlocks(DagNode& from, DagNode& to, const std::vector<std::string>& keys, std::vector<Status>* statuses,
                   size_t batch) {
    statuses->assign(keys.size(), Status());
    for (size_t b0 = 0; b0 < keys.size(); b0 += std::max<size_t>(batch, 1)) {
        const size_t nb = std::min(std::max<size_t>(batch, 1), keys.size() - b0);
        std::vector<std::string> ks(keys.begin() + b0, keys.begin() + b0 + nb);
        std::vector<Bytes> blocks;
        std::vector<Status> st;
        from.GetMany(ks, &blocks, &st, batch);
        std::vector<std::string> put_keys;
        std::vector<Bytes> put_blocks;
        std::vector<size_t> put_idx;
        for (size_t j = 0; j < nb; j++) {
            if (!st[j].ok()) {
                // cluster.go:252-255: a block missing on `from` counts as migrated
                (*statuses)[b0 + j] = st[j].err == "Key not found" ? Status::Ok() : st[j];
                continue;
            }
            put_keys.push_back(ks[j]);
            put_blocks.push_back(std::move(blocks[j]));
            put_idx.push_back(b0 + j);
        }
        // PutMany reports only the last error, so verify each key landed with a meta read
        to.PutMany(put_keys, put_blocks);
        for (size_t j = 0; j < put_keys.size(); j++) {
            int size = -1;
            Status s = to.GetSize(put_keys[j], &size);
            if (s.ok() && size != int(put_blocks[j].size())) s = Status::Error("migrated block size mismatch");
            (*statuses)[put_idx[j]] = s;
            if (s.ok()) (void)from.DeleteBlock(put_keys[j]);  // cluster.go:265-267: warn only
        }
    }
}

// ------------------------------------------------------------------ repair
Status DagNode::repair_block(const std::string& key, int32_t block_size, std::vector<Bytes> shards,
                             const std::vector<int>& indexes) {  // data_recovery.go:115-167
    for (int i : indexes)
        if (i >= int(nodes_.size())) return Status::Error("repair index greater than max index of nodes");
    int available = 0;
    for (auto& sh : shards) available += !sh.empty();
    if (available < EntryQuorum().first) return Status::Error("repair index greater than max index of nodes");
    Erasure enc;
    Status s = member_erasure(MemberOfKey(key), block_size, &enc);
    if (!s.ok()) return s;
    s = enc.DecodeDataAndParityBlocks(shards);
    if (!s.ok()) return s;
    const Bytes meta = encode_meta(block_size);
    for (int i : indexes) {
        s = nodes_[i].client->Put(key, meta, shards[i]);
        if (!s.ok()) return s;
    }
    return Status::Ok();
}

size_t DagNode::RepairQueueLen() {
    std::lock_guard<std::mutex> g(q_mu_);
    return repair_queue_.size();
}

size_t DagNode::RunRepairTasks() {
    size_t ran = 0;
    for (;;) {
        std::function<void()> task;
        {
            std::lock_guard<std::mutex> g(q_mu_);
            if (repair_queue_.empty()) return ran;
            task = std::move(repair_queue_.front());
            repair_queue_.pop_front();
        }
        task();
        ran++;
    }
}

void DagNode::StartRepairWorker() {
    if (worker_.joinable()) return;
    worker_ = std::thread([this] {
        for (;;) {
            std::function<void()> task;
            {
                std::unique_lock<std::mutex> g(q_mu_);
                q_cv_.wait(g, [this] { return stop_ || !repair_queue_.empty(); });
                if (stop_) return;
                task = std::move(repair_queue_.front());
                repair_queue_.pop_front();
            }
            task();
        }
    });
}

// data_recovery.go:57-81: k shards from every node but the one under repair
Status DagNode::fetch_for_repair(const std::string& key, int repair_index, std::vector<Bytes>* shards) {
    const int n = int(nodes_.size()), rq = EntryQuorum().first;
    shards->assign(size_t(n), Bytes());
    QuorumWait w(rq, n - rq + 1);
    // waves of concurrent fetches replayed in node order, as in fetch_for_get
    std::vector<Bytes> data(static_cast<size_t>(n)), metas(static_cast<size_t>(n));
    std::vector<Status> got(static_cast<size_t>(n));
    std::vector<DataNodeClient::Stored> stored(static_cast<size_t>(n));
    std::vector<char> fetched(static_cast<size_t>(n), 0);
    int succ = 0;
    for (int i = 0; i < n && !w.decided(); i++) {
        if (i == repair_index) {
            w.add(Status::Error("there is no data in this node"));
            continue;
        }
        if (!fetched[i]) {
            std::vector<int> wave;
            for (int j = i; j < n && int(wave.size()) < std::max(1, rq - succ); j++)
                if (j != repair_index && !fetched[j]) wave.push_back(j);
            fan(int(wave.size()), [&](int t) {
                Bytes m;
                got[wave[t]] = nodes_[wave[t]].client->Get(key, &m, &data[wave[t]]);
            }, last_shard_.load());
            for (int j : wave) fetched[j] = 1;
        }
        Status g = got[i];
        if (g.ok() && data[i].empty()) g = Status::Error("there is no data in this node");
        if (g.ok()) {
            (*shards)[i] = std::move(data[i]);
            succ++;
        }
        w.add(g);
    }
    return w.result(kErrReadQuorum);
}

// data_recovery.go:16-112 through the batched form: the same index checks, keys present on the
// target skipped (:41-43), keys whose size or k-of-n fetch fails skipped (:48-51, :78-81), and a
// decode or target write error returned (:83-92, :101-106).  Rows of one flush are written
// concurrently, so when a write fails, later keys of the same flush may have been repaired as
// well; the error returned is the first in key order.
Status DagNode::RepairDataNode(int from, int to) { return RepairDataNodeBatched(from, to, kRepairBatch); }

Status DagNode::RepairDataNodePerKey(int from, int to) {  // data_recovery.go:16-112, key by key
    if (from >= int(nodes_.size())) return Status::Error("index greater than max index of nodes");
    if (to >= int(nodes_.size())) return Status::Error("repair index greater than max index of nodes");
    std::vector<std::string> keys;
    Status s = nodes_[from].client->AllKeys(&keys);
    if (!s.ok()) return s;
    for (const auto& key : keys) {
        Bytes mb;
        if (nodes_[to].client->GetMeta(key, &mb).ok()) continue;
        int size;
        if (!GetSize(key, &size).ok()) continue;
        std::vector<Bytes> shards;
        if (!fetch_for_repair(key, to, &shards).ok()) continue;
        bool done = false;
        if (lone_paths_ && active_.load() == 0 && (s = repair_row_in_place(key, size, shards, to, &done), !s.ok()))
            return s;
        if (done) continue;
        Erasure enc;
        s = member_erasure(MemberOfKey(key), size, &enc);
        if (!s.ok()) return s;
        s = enc.DecodeDataAndParityBlocks(shards);
        if (!s.ok()) return s;
        s = nodes_[to].client->Put(key, encode_meta(size), shards[to]);
        if (!s.ok()) return s;
    }
    return Status::Ok();
}

// RepairDataNode's per-key rebuild and write (data_recovery.go:95-106) for a lone caller: the k
// survivors the decode reads are copied into the page-locked block scratch, only the repaired
// node's row is rebuilt there in place, and the datanode gets a view of it with a plain Put (the
// datanode's own carry-less CRC of one row costs less than a GPU checksum pass and its read-back).
// *done = false leaves the key to the per-shard path (an empty block, shard lengths that are not
// the block's shard size); the decode's errors are returned as the per-shard path returns them.
Status DagNode::repair_row_in_place(const std::string& key, int size, const std::vector<Bytes>& shards, int to,
                                    bool* done) {
    *done = false;
    const int k = config_.data_blocks, n = int(nodes_.size());
    if (size <= 0 || int(shards.size()) != n) return Status::Ok();
    const size_t S = rsmi_shard_size(size_t(size), k);
    std::vector<size_t> lens(static_cast<size_t>(n));
    std::vector<uint8_t> present(static_cast<size_t>(n)), required(static_cast<size_t>(n), 0);
    for (int i = 0; i < n; i++) {
        lens[i] = shards[i].size();
        present[i] = shards[i].empty() ? 0 : 1;
    }
    size_t S2 = 0;
    int rc = rsmi_check_shards(n, lens.data(), 1, &S2);
    if (rc) return rsmi_status(rc);
    if (S2 != S || present[to]) return Status::Ok();
    int np = 0;
    for (int i = 0; i < n; i++) np += present[i];
    if (np < k) return rsmi_status(RSMI_ERR_TOO_FEW_SHARDS);
    required[to] = 1;
    rsmi_ctx* ctx = member_ctx(MemberOfKey(key), &rc);
    if (!ctx) return rsmi_status(rc);
    uint8_t* flat = block_scratch(size_t(n) * S);
    if (!flat) return Status::Error("out of host memory");
    for (int i = 0, used = 0; i < n && used < k; i++)
        if (present[i]) {
            copy_bytes(flat + size_t(i) * S, shards[i].data(), S);
            used++;
        }
    rc = rsmi_reconstruct_rows_batch_host(ctx, flat, size_t(n) * S, S, 1, present.data(), required.data());
    if (rc) return rsmi_status(rc);
    Status s = nodes_[to].client->Put(key, encode_meta(size), ByteView(flat + size_t(to) * S, S));
    if (!s.ok()) return s;
    *done = true;
    return Status::Ok();
}

Status DagNode::RepairDataNodeBatched(int from, int to, size_t batch, size_t* repaired) {
    Active act(active_);
    if (from >= int(nodes_.size())) return Status::Error("index greater than max index of nodes");
    if (to >= int(nodes_.size())) return Status::Error("repair index greater than max index of nodes");
    if (batch == 0) batch = 1;
    const int k = config_.data_blocks, m = config_.parity_blocks, n = k + m;
    std::vector<std::string> keys;
    Status s = nodes_[from].client->AllKeys(&keys);
    if (!s.ok()) return s;
    size_t done = 0;
    struct Pending {
        std::string key;
        std::vector<Bytes> shards;
    };
    // (block size, survivor pattern) -> pending keys
    std::map<std::pair<int, std::string>, std::vector<Pending>> groups;
    DataNodeClient& target = *nodes_[to].client;
    // A flush stages its keys' survivors into one of two page-locked buffers (the halves of the
    // thread's staging), then hands the buffer to a helper task that runs the codec call and writes
    // the rebuilt rows to the target; the next flush stages into the other half meanwhile, so the
    // codec call overlaps the next staging copy as well as the next window's fetch.  A flush joins
    // the previous task before it launches its own (at most one in flight; the staging only grows
    // after it is joined), and every return joins it first, so the rows written, the count and the
    // first error returned (in key order; a codec error counts for every key of its flush, none
    // written) are those of the sequential loop.
    std::future<std::vector<Status>> writing;
    auto join_writes = [&]() -> Status {
        if (!writing.valid()) return Status::Ok();
        const auto tw = PhaseClock::now();
        const std::vector<Status> ps = writing.get();
        trace_add(kTraceWaitWrites, tw, PhaseClock::now());
        for (const Status& st : ps) {
            if (!st.ok()) return st;
            done++;
        }
        return Status::Ok();
    };
    int cur = 0;
    // the previous flush's staging and write times, for the codec call's placement
    int64_t last_stage = 0;
    auto last_writes = std::make_shared<std::atomic<int64_t>>(0);
    auto flush = [&](const std::pair<int, std::string>& gk, std::vector<Pending>& pend) -> Status {
        if (pend.empty()) return Status::Ok();
        const int size = gk.first;
        const size_t S = rsmi_shard_size(size_t(size), k), nb = pend.size();
        std::vector<uint8_t> present(static_cast<size_t>(n)), required(static_cast<size_t>(n), 0);
        for (int i = 0; i < n; i++) present[i] = uint8_t(gk.second[i] == '1');
        required[to] = 1;
        // the keys ordered by member (a device list): each member rebuilds one range; the
        // writes' outcomes are taken back in key order
        MemberOrder ord = member_order(nb, [&](size_t j) { return MemberOfKey(pend[j].key); });
        // the fetch returns exactly the k survivors the plan reads (fetch_for_repair stops at
        // the read quorum k), and only those are staged; the rows being rebuilt are not
        const auto t0 = PhaseClock::now();
        PinnedBuf& st = thread_staging();
        const size_t bytes = nb * size_t(n) * S;
        if (st.capacity() < 2 * bytes) {  // growing frees the buffer the task may be reading
            const Status w = join_writes();
            if (!w.ok()) return w;
        }
        uint8_t* base = st.reserve(2 * bytes);
        if (!base) {
            const Status w = join_writes();
            return w.ok() ? Status::Error("out of host memory") : w;
        }
        uint8_t* flat = base + (cur ? st.capacity() / 2 : 0);
        fan_keys(int(nb), [&](int j) {
            const Pending& p = pend[ord.perm[size_t(j)]];
            for (int i = 0; i < n; i++)
                if (present[i]) std::memcpy(flat + (size_t(j) * n + i) * S, p.shards[i].data(), S);
        });
        phase_add(Phase::Stage, t0);
        last_stage = std::chrono::duration_cast<std::chrono::nanoseconds>(PhaseClock::now() - t0).count();
        std::vector<std::string> wkeys(nb);
        for (size_t j = 0; j < nb; j++) wkeys[j] = std::move(pend[ord.perm[j]].key);
        pend.clear();
        // the rebuilt rows' checksums come from the GPU pass too (sender checksums, as in Put)
        const bool want32 = gpu_checksums_ && gpu_value_checksums_ && target.WantsValueChecksum();
        // the flush's codec call: here or as the task's first step (RSMI_BATCH_CODEC_PLACE)
        auto r16 = std::make_shared<std::vector<uint32_t>>(gpu_checksums_ ? nb * size_t(n) : 0);
        auto r32 = std::make_shared<std::vector<uint32_t>>(want32 ? nb * size_t(n) : 0);
        auto po = std::make_shared<MemberOrder>(std::move(ord));
        auto code = [this, flat, S, n, want32, r16, r32, po, present = std::move(present),
                     required = std::move(required)] {
            const auto t1 = PhaseClock::now();
            const int rc = code_members(*po, [&](rsmi_ctx* ctx, size_t j0, size_t cnt) {
                uint8_t* f = flat + j0 * size_t(n) * S;
                if (!gpu_checksums_)
                    return rsmi_reconstruct_rows_batch_host(ctx, f, size_t(n) * S, S, cnt, present.data(),
                                                            required.data());
                return rsmi_reconstruct_rows_batch_host_crcs(ctx, f, size_t(n) * S, S, cnt, present.data(),
                                                             required.data(), r16->data() + j0 * size_t(n),
                                                             want32 ? r32->data() + j0 * size_t(n) : nullptr);
            });
            phase_add(Phase::Codec, t1);
            return rc;
        };
        const bool inline_codec = RSMI_BATCH_CODEC_PLACE == 1 ||
                                  (RSMI_BATCH_CODEC_PLACE == 0 && last_writes->load() > last_stage);
        const int pre = inline_codec ? code() : RSMI_OK;
        // the previous flush's task (its codec call and writes) ends before this one starts
        const Status w = join_writes();
        if (!w.ok()) return w;
        writing = std::async(std::launch::async, [this, &target, flat, S, n, to, want32, meta = encode_meta(size), po,
                                                  code, pre, inline_codec, r16, r32, last_writes,
                                                  wkeys = std::move(wkeys)] {
            const size_t nw = wkeys.size();
            const int rc = inline_codec ? pre : code();
            const MemberOrder& ord = *po;
            std::vector<Status> ps(nw);  // by key order (perm[j]: slot j's key)
            if (rc) {
                for (auto& x : ps) x = rsmi_status(rc);
                return ps;
            }
            // the rebuilt rows go to the target concurrently, each as a view of the staging buffer
            const auto t2 = PhaseClock::now();
            fan_keys(int(nw), [&](int j) {
                const ByteView shard(flat + (size_t(j) * n + size_t(to)) * S, S);
                Status& out = ps[ord.perm[size_t(j)]];
                if (!gpu_checksums_) {
                    out = target.Put(wkeys[j], meta, shard);
                    return;
                }
                const uint16_t c16 = entry_checksum(meta, S, (*r16)[size_t(j) * n + size_t(to)]);
                out = want32 ? target.PutWithChecksums(wkeys[j], meta, shard, c16,
                                                       value_checksum(meta, S, c16, (*r32)[size_t(j) * n + size_t(to)]))
                             : target.PutWithChecksum(wkeys[j], meta, shard, c16);
            });
            phase_add(Phase::Put, t2);
            last_writes->store(std::chrono::duration_cast<std::chrono::nanoseconds>(PhaseClock::now() - t2).count());
            return ps;
        });
        cur ^= 1;
        return Status::Ok();
    };
    // Each key's checks and fetch (the target's GetMeta, the meta quorum, the k-of-n fetch) run
    // concurrently over a window of keys; the results are then taken in key order, so the
    // grouping, the flushes and the errors returned are those of the sequential loop.  The next
    // window is fetched on a helper thread while this thread stages, codes and writes the
    // current one (the GPU call no longer leaves the host idle); fetches only read, so running
    // one ahead changes no outcome, and a failing flush still returns before any later write.
    struct Fetch {
        bool use = false;
        int size = 0;
        std::vector<Bytes> shards;
    };
    auto fetch_window = [this, &keys, to](size_t c0, size_t nk) {
        const auto t0 = PhaseClock::now();
        std::vector<Fetch> fr(nk);
        fan_keys(int(nk), [&](int q) {
            const std::string& key = keys[c0 + size_t(q)];
            Bytes mb;
            if (nodes_[to].client->GetMeta(key, &mb).ok()) return;
            int size;
            if (!GetSize(key, &size).ok()) return;
            if (!fetch_for_repair(key, to, &fr[size_t(q)].shards).ok()) return;
            fr[size_t(q)].size = size;
            fr[size_t(q)].use = true;
        });
        phase_add(Phase::Fetch, t0);
        return fr;
    };
    // windows as large as one flush (half the staging, for the double buffer, by the shard size
    // seen last), at most batch
    size_t window = std::min<size_t>(batch, 16);
    auto next_window = [&](const std::vector<Fetch>& fr) {
        for (auto& f : fr)
            if (f.use && f.size > 0)
                window = std::max<size_t>(
                    1, std::min(batch, staging_blocks(2 * size_t(n) * rsmi_shard_size(size_t(f.size), k))));
    };
    std::future<std::vector<Fetch>> ahead;
    size_t c0 = 0, nk = std::min(window, keys.size());
    std::vector<Fetch> fr = fetch_window(c0, nk);
    while (c0 < keys.size()) {
        next_window(fr);
        const size_t c1 = c0 + nk, nk1 = std::min(window, keys.size() - std::min(c1, keys.size()));
        if (nk1) ahead = std::async(std::launch::async, fetch_window, c1, nk1);
        for (size_t q = 0; q < nk; q++) {
            if (!fr[q].use) continue;
            const std::string& key = keys[c0 + q];
            const int size = fr[q].size;
            std::vector<Bytes>& shards = fr[q].shards;
            if (size <= 0) {  // empty block: the per-key path's error behaviour (ErrShardNoData)
                s = join_writes();
                if (!s.ok()) return s;
                Erasure enc;
                s = member_erasure(MemberOfKey(key), size, &enc);
                if (s.ok()) s = enc.DecodeDataAndParityBlocks(shards);
                if (!s.ok()) return s;  // `ahead` (reads only) is joined by its destructor
                continue;
            }
            std::string pat(size_t(n), '0');
            for (int i = 0; i < n; i++) pat[i] = shards[i].empty() ? '0' : '1';
            auto gk = std::make_pair(size, pat);
            auto& pend = groups[gk];
            pend.push_back(Pending{key, std::move(shards)});
            if (pend.size() >= std::min(batch, staging_blocks(2 * size_t(n) * rsmi_shard_size(size_t(size), k)))) {
                s = flush(gk, pend);
                if (!s.ok()) return s;
            }
        }
        c0 = c1;
        nk = nk1;
        const auto tw = PhaseClock::now();
        if (nk1) fr = ahead.get();
        trace_add(kTraceWaitFetch, tw, PhaseClock::now());
    }
    for (auto& g : groups) {
        s = flush(g.first, g.second);
        if (!s.ok()) return s;
    }
    s = join_writes();
    if (!s.ok()) return s;
    if (repaired) *repaired = done;
    return Status::Ok();
}

void DagNode::phase_add(Phase p, PhaseClock::time_point t0) {
    if (!phase_on_.load(std::memory_order_relaxed)) return;
    const auto t1 = PhaseClock::now();
    phase_ns_[int(p)] += uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count());
    trace_add(int(p), t0, t1);
}

void DagNode::trace_add(int id, PhaseClock::time_point t0, PhaseClock::time_point t1) {
    if (!phase_on_.load(std::memory_order_relaxed) || !trace_on_.load(std::memory_order_relaxed)) return;
    std::lock_guard<std::mutex> g(trace_mu_);
    const auto sec = [&](PhaseClock::time_point t) { return std::chrono::duration<double>(t - trace_epoch_).count(); };
    trace_.push_back(PhaseEvent{id, uint64_t(std::hash<std::thread::id>()(std::this_thread::get_id())), sec(t0), sec(t1)});
}

std::vector<DagNode::PhaseEvent> DagNode::PhaseEvents() {
    std::lock_guard<std::mutex> g(trace_mu_);
    return trace_;
}

std::array<double, 4> DagNode::PhaseSeconds() const {
    std::array<double, 4> r{};
    for (int i = 0; i < 4; i++) r[size_t(i)] = double(phase_ns_[i].load()) * 1e-9;
    return r;
}

void DagNode::ResetPhases() {
    for (auto& x : phase_ns_) x = 0;
    std::lock_guard<std::mutex> g(trace_mu_);
    trace_.clear();
    trace_epoch_ = PhaseClock::now();
}

}  // namespace host
}  // namespace rsmi
