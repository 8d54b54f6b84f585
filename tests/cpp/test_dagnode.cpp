// test_dagnode.cpp -- the Dag Node / datanode host mirror, in the shape of the reference's
// own Go tests (dag/node/dagnode/node_test.go, dag/node/datanode/server_test.go).
//
//   test_dagnode cpu   datanode framing/CRC, quorum helpers, slots, config checks (no GPU)
//   test_dagnode gpu   TestDagNode "123456" round trip, RS(10,4) failure/quorum matrix,
//                      read-repair, RepairDataNode (per key and batched), PutMany batch,
//                      GetMany (batched degraded reads), RS(10,4) -> RS(4,2) migration,
//                      GPU entry (CRC-16) and mutcask value (CRC-32) checksums;
//                      every stored shard is compared with the CPU oracle (test-only).
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../filedag-storage_amd/csrc/group_commit.hpp"
#include "../../filedag-storage_amd/csrc/host/dagnode.hpp"
#include "../../oracle/rs_oracle.h"

using namespace rsmi::host;

static int g_fail = 0, g_checks = 0;
#define CHECK(cond)                                                                  \
    do {                                                                             \
        g_checks++;                                                                  \
        if (!(cond)) {                                                               \
            g_fail++;                                                                \
            std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
        }                                                                            \
    } while (0)
#define CHECK_OK(st)                                                                              \
    do {                                                                                          \
        Status _s = (st);                                                                         \
        g_checks++;                                                                               \
        if (!_s.ok()) {                                                                           \
            g_fail++;                                                                             \
            std::fprintf(stderr, "%s:%d: unexpected error: %s\n", __FILE__, __LINE__, _s.err.c_str()); \
        }                                                                                         \
    } while (0)

static Bytes str(const char* s) { return Bytes(s, s + std::strlen(s)); }

// Block sizes of the Dag Node tests: the bench shape (256 KiB) and a dag-pb 1 MiB leaf.  The
// sanitizer builds (mode "sanitize": fake_rsmi.cpp codes with the scalar oracle, under
// ThreadSanitizer / AddressSanitizer) run the same tests at a scale of 1/32.
static size_t g_big = 262144, g_leaf = 1048590, g_huge = 4194304;
static size_t g_fanout_min = size_t(128) << 10;  // sanitize: 0, so the fan-out pool runs at the small sizes
static size_t big(long d = 0) { return size_t(long(g_big) + d); }
// The Dag Nodes' device list (DagNode::New): {0}, or, for the suite's member pass, two members
// naming device 0 (the GPU box has one GPU), so every per-key call and batch range is routed by
// hash slot over two contexts.
static std::vector<int> g_devices{0};

static Bytes rand_bytes(std::mt19937_64& r, size_t n) {
    Bytes b(n);
    for (auto& x : b) x = uint8_t(r());
    return b;
}

struct Cluster {
    std::vector<std::shared_ptr<InProcDataNode>> dn;
    std::unique_ptr<DagNode> node;
    explicit Cluster(int k, int m, KvEngine engine = KvEngine::Badger) {
        DagNodeConfig cfg;
        cfg.name = "dag_node1";
        cfg.data_blocks = k;
        cfg.parity_blocks = m;
        std::vector<std::shared_ptr<DataNodeClient>> clients;
        for (int i = 0; i < k + m; i++) {
            cfg.nodes.push_back("127.0.0.1:" + std::to_string(9011 + i));
            dn.push_back(std::make_shared<InProcDataNode>(cfg.nodes.back(), engine));
            clients.push_back(dn.back());
        }
        Status s = DagNode::New(cfg, clients, &node, g_devices);
        if (!s.ok()) {
            std::fprintf(stderr, "NewDagNode: %s\n", s.err.c_str());
            std::exit(2);
        }
        node->SetFanoutMinBytes(g_fanout_min);
        node->HealthCheckAll();
    }
};

// oracle shards of a block: (k+m) rows of S bytes
static std::vector<Bytes> oracle_shards(int k, int m, const Bytes& block) {
    const size_t S = rs_oracle_shard_size(block.size(), k);
    Bytes flat(size_t(k + m) * S);
    rs_oracle_split(k, m, block.data(), block.size(), flat.data());
    rs_oracle_encode(k, m, flat.data(), S);
    std::vector<Bytes> out;
    for (int i = 0; i < k + m; i++) out.emplace_back(flat.begin() + i * S, flat.begin() + (i + 1) * S);
    return out;
}

static Bytes stored_shard(InProcDataNode& d, const std::string& key) {
    Bytes meta, data;
    if (!d.server().Get(key, &meta, &data).ok()) return Bytes();
    return data;
}

// ------------------------------------------------------------------ CPU-only tests
static void test_datanode_server() {
    DataNodeServer s;
    // server_test.go:14-22 (badger): empty key rejected
    CHECK(!s.Put("", Bytes(), str("123")).ok());
    CHECK_OK(s.Put("1234567", Bytes(), str("\b\x02\x12\a1234567\x18\a")));
    CHECK_OK(s.Put("@#", Bytes(), str("@#$$&*^@*")));
    Bytes meta = {6, 0, 0, 0}, data = str("123456"), m2, d2;
    CHECK_OK(s.Put("key", meta, data));
    CHECK_OK(s.Get("key", &m2, &d2));
    CHECK(m2 == meta && d2 == data);
    int64_t sz = 0;
    CHECK_OK(s.Size("key", &sz));
    CHECK(sz == kHeaderSize + 4 + 6);  // HeaderSize + len(meta) + len(data) (server_test.go:147-152)
    Bytes e;
    CHECK(s.RawEntry("key", &e));
    // | crc | metaSize | dataSize | meta | data |, crc over bytes [4:], little endian
    CHECK(e.size() == 22 && e[4] == 4 && e[8] == 6);
    const uint16_t crc = crc16_ibm(e.data() + 4, e.size() - 4);
    CHECK(e[0] == (crc & 0xFF) && e[1] == (crc >> 8) && e[2] == 0 && e[3] == 0);
    // corruption is caught by the crc check on Get and GetMeta (server.go:93-97)
    s.CorruptByte("key", 15);
    Status g = s.Get("key", &m2, &d2);
    CHECK(!g.ok() && g.err == "checking crc failed");
    CHECK(!s.GetMeta("key", &m2).ok());
    CHECK_OK(s.Delete("key"));
    CHECK(!s.Get("key", &m2, &d2).ok());
    CHECK(!s.Size("key", &sz).ok());
    std::vector<std::string> keys;
    CHECK_OK(s.AllKeys(&keys));
    CHECK(keys.size() == 2);
    // CRC-16/USB check value of the restated IBM-table variant
    const char* cv = "123456789";
    CHECK(crc16_ibm(reinterpret_cast<const uint8_t*>(cv), 9) == 0xB4C8);
}

static void test_datanode_sender_checksum() {
    DataNodeServer s;
    const Bytes meta{4, 0, 0, 0}, data = str("shard-bytes");
    CHECK_OK(s.Put("a", meta, data));
    Bytes ea;
    CHECK(s.RawEntry("a", &ea));
    const uint16_t good = uint16_t(ea[0] | ea[1] << 8);
    CHECK_OK(s.PutWithChecksum("b", meta, data, good));
    Bytes eb;
    CHECK(s.RawEntry("b", &eb));
    CHECK(ea == eb);
    CHECK_OK(s.PutWithChecksum("c", meta, data, uint16_t(good ^ 1)));
    Bytes m2, d2;
    Status st = s.Get("c", &m2, &d2);
    CHECK(!st.ok() && st.err == "checking crc failed");
    CHECK(rs_oracle_datanode_entry_crc(meta.data(), meta.size(), data.data(), data.size()) == good);
}

static uint32_t le32(const Bytes& b, size_t off) {
    return uint32_t(b[off]) | uint32_t(b[off + 1]) << 8 | uint32_t(b[off + 2]) << 16 | uint32_t(b[off + 3]) << 24;
}

// kv/mutcask/cask.go:73-97 under the datanode (server.go:207): the stored value is
// |crc32 (4 LE)|entry|, re-checked on every read; Size stays the entry size (cask.go:235)
static void test_datanode_mutcask() {
    const char* cv = "mutation of bitcask";  // cask_test.go TestValueEncodeDecode's value
    CHECK(crc32_ieee(reinterpret_cast<const uint8_t*>(cv), std::strlen(cv)) ==
          rs_oracle_crc32_ieee(reinterpret_cast<const uint8_t*>(cv), std::strlen(cv)));
    CHECK(crc32_ieee(reinterpret_cast<const uint8_t*>("123456789"), 9) == 0xCBF43926u);
    DataNodeServer s(KvEngine::Mutcask);
    const Bytes meta = {6, 0, 0, 0}, data = str("123456");
    CHECK_OK(s.Put("key", meta, data));
    Bytes v, e, m2, d2;
    CHECK(s.RawValue("key", &v) && s.RawEntry("key", &e));
    CHECK(v.size() == e.size() + 4 && Bytes(v.begin() + 4, v.end()) == e);
    CHECK(le32(v, 0) == rs_oracle_crc32_ieee(e.data(), e.size()));
    CHECK(le32(v, 0) == rs_oracle_mutcask_entry_crc(le32(e, 0), meta.data(), 4, data.data(), data.size()));
    CHECK(le32(e, 0) == rs_oracle_datanode_entry_crc(meta.data(), 4, data.data(), data.size()));
    CHECK_OK(s.Get("key", &m2, &d2));
    CHECK(m2 == meta && d2 == data);
    int64_t sz = 0;
    CHECK_OK(s.Size("key", &sz));
    CHECK(sz == kHeaderSize + 4 + 6);
    // the sender's pair of checksums gives the same stored value; a wrong value checksum is
    // caught by the engine before the datanode's own check
    CHECK_OK(s.PutWithChecksums("k2", meta, data, uint16_t(le32(e, 0)), le32(v, 0)));
    Bytes v2;
    CHECK(s.RawValue("k2", &v2) && v2 == v);
    CHECK_OK(s.PutWithChecksums("k3", meta, data, uint16_t(le32(e, 0)), le32(v, 0) ^ 1));
    Status g = s.Get("k3", &m2, &d2);
    CHECK(!g.ok() && g.err == "mutcask: data may be rotted");
    CHECK(!s.GetMeta("k3", &m2).ok());
    s.CorruptByte("key", kHeaderSize + 4 + 2);  // a data byte of the entry
    g = s.Get("key", &m2, &d2);
    CHECK(!g.ok() && g.err == "mutcask: data may be rotted");
    // a client over badger drops the value checksum and keeps the entry byte-identical
    InProcDataNode b("b");
    CHECK(!b.WantsValueChecksum() && InProcDataNode("m", KvEngine::Mutcask).WantsValueChecksum());
    CHECK_OK(b.PutWithChecksums("key", meta, data, uint16_t(le32(e, 0)), 12345));
    Bytes eb;
    CHECK(b.server().RawEntry("key", &eb) && b.server().RawValue("key", &v2) && eb == e && v2 == e);
}

static void test_quorum_helpers() {
    // reduceQuorumErrs
    std::vector<Status> errs = {Status(), Status(), Status::Error("x"), Status::Error(kErrNodeNotFound)};
    CHECK(reduce_quorum_errs(errs, 2, kErrReadQuorum).ok());
    CHECK(reduce_quorum_errs(errs, 3, kErrReadQuorum).err == kErrReadQuorum);
    errs = {Status::Error("Key not found"), Status::Error("Key not found"), Status::Error("Key not found")};
    CHECK(reduce_quorum_errs(errs, 2, kErrReadQuorum).err == "Key not found");
    errs = {Status::Error("a"), Status(), Status::Error("a"), Status()};
    CHECK(reduce_quorum_errs(errs, 2, kErrReadQuorum).ok());  // nil wins ties
    // findMetaInQuorum
    Meta out;
    CHECK(find_meta_in_quorum({{6}, {6}, {6}}, 1, &out).err == kErrReadQuorum);  // quorum < 2 fails
    CHECK(find_meta_in_quorum({{6}, {6}, {0}}, 2, &out).ok() && out.block_size == 6);
    CHECK(!find_meta_in_quorum({{6}, {7}, {0}}, 2, &out).ok());
}

static void test_config_and_slots() {
    DagNodeConfig cfg;
    cfg.data_blocks = 2;
    cfg.parity_blocks = 1;
    cfg.nodes = {"a", "b"};
    std::unique_ptr<DagNode> d;
    std::vector<std::shared_ptr<DataNodeClient>> c = {std::make_shared<InProcDataNode>("a"),
                                                      std::make_shared<InProcDataNode>("b")};
    CHECK(DagNode::New(cfg, c, &d).err == "dag node config is incorrect");  // node.go:55-57
    cfg.nodes.push_back("c");
    c.push_back(std::make_shared<InProcDataNode>("c"));
    CHECK_OK(DagNode::New(cfg, c, &d));
    CHECK(d->EntryQuorum() == std::make_pair(2, 2));
    CHECK(d->AddSlot(5) == false && d->AddSlot(5) == true && d->GetNumSlots() == 1);
    CHECK(d->GetSlot(5) && !d->GetSlot(6));
    CHECK(d->ClearSlot(5) == true && d->GetNumSlots() == 0);
    CHECK(!d->GetDataNodeState(0));
    d->HealthCheckAll();
    CHECK(d->GetDataNodeState(0));
    cfg.data_blocks = cfg.parity_blocks = 2;
    cfg.nodes.push_back("d");
    c.push_back(std::make_shared<InProcDataNode>("d"));
    CHECK_OK(DagNode::New(cfg, c, &d));
    CHECK(d->EntryQuorum() == std::make_pair(2, 3));  // k == m -> write quorum k+1
    // Get of an absent key on a healthy cluster surfaces the KV's error
    Bytes b;
    Status s = d->Get("nope", &b);
    CHECK(!s.ok() && s.err == "Key not found");
}

// ------------------------------------------------------------------ GPU tests
static void test_dagnode_123456() {  // node_test.go:18-65, RS(2,1) over 3 datanodes
    Cluster c(2, 1);
    const Bytes block = str("123456");
    CHECK_OK(c.node->Put("QmTestBlock", block));
    Bytes got;
    CHECK_OK(c.node->Get("QmTestBlock", &got));
    CHECK(got == block);
    int size = 0;
    CHECK_OK(c.node->GetSize("QmTestBlock", &size));
    CHECK(size == 6);
    // the shards on the datanodes: "123", "456", parity 3b 3c 39
    CHECK(stored_shard(*c.dn[0], "QmTestBlock") == str("123"));
    CHECK(stored_shard(*c.dn[1], "QmTestBlock") == str("456"));
    CHECK((stored_shard(*c.dn[2], "QmTestBlock") == Bytes{0x3b, 0x3c, 0x39}));
    int64_t sz;
    CHECK_OK(c.dn[0]->Size("QmTestBlock", &sz));
    CHECK(sz == kHeaderSize + 4 + 3);
    // any single datanode down: still readable (read quorum 2), reconstruct on the GPU
    for (int down = 0; down < 3; down++) {
        c.dn[down]->SetOffline(true);
        got.clear();
        CHECK_OK(c.node->Get("QmTestBlock", &got));
        CHECK(got == block);
        c.dn[down]->SetOffline(false);
    }
    CHECK_OK(c.node->DeleteBlock("QmTestBlock"));
    bool has = true;
    c.node->Has("QmTestBlock", &has);
    CHECK(!has);
}

static void test_rs10_4_failures() {
    const int k = 10, m = 4, n = k + m;
    Cluster c(k, m);
    std::mt19937_64 r(0xF11EDA6);
    const size_t sizes[] = {1, 6, 9, 10, 11, 4099, 65536, big(-1), big(), big(1), g_leaf};
    std::vector<std::string> keys;
    std::vector<Bytes> blocks;
    for (size_t i = 0; i < sizeof(sizes) / sizeof(sizes[0]); i++) {
        keys.push_back("bafy-" + std::to_string(i));
        blocks.push_back(rand_bytes(r, sizes[i]));
        CHECK_OK(c.node->Put(keys.back(), blocks.back()));
        // every stored shard equals the oracle's
        auto want = oracle_shards(k, m, blocks.back());
        for (int j = 0; j < n; j++) CHECK(stored_shard(*c.dn[j], keys.back()) == want[j]);
    }
    // up to m datanodes down: every block still reads back
    const int downs[][4] = {{0, -1, -1, -1}, {0, 1, 2, 3}, {10, 11, 12, 13}, {0, 5, 11, 13}, {9, 3, 12, -1}};
    for (auto& d : downs) {
        for (int x : d)
            if (x >= 0) c.dn[x]->SetOffline(true);
        for (size_t i = 0; i < keys.size(); i++) {
            Bytes got;
            CHECK_OK(c.node->Get(keys[i], &got));
            CHECK(got == blocks[i]);
        }
        for (int x : d)
            if (x >= 0) c.dn[x]->SetOffline(false);
    }
    // m+1 down: read quorum lost
    for (int x = 0; x < m + 1; x++) c.dn[x]->SetOffline(true);
    Bytes got;
    CHECK(!c.node->Get(keys[0], &got).ok());
    // write quorum is k: with m+1 down a Put fails, with m down it succeeds
    CHECK(!c.node->Put("w1", blocks[3]).ok());
    c.dn[m]->SetOffline(false);
    CHECK_OK(c.node->Put("w2", blocks[3]));
    for (int x = 0; x < m; x++) c.dn[x]->SetOffline(false);
    CHECK_OK(c.node->Get("w2", &got));
    CHECK(got == blocks[3]);
}

static void test_read_repair() {
    const int k = 10, m = 4;
    Cluster c(k, m);
    std::mt19937_64 r(7);
    const Bytes block = rand_bytes(r, big());
    CHECK_OK(c.node->Put("blk", block));
    auto want = oracle_shards(k, m, block);
    // a datanode loses two shards of the block (data 3 and parity 12)
    c.dn[3]->server().Delete("blk");
    c.dn[12]->server().Delete("blk");
    Bytes got;
    CHECK_OK(c.node->Get("blk", &got));
    CHECK(got == block);
    CHECK(c.node->RepairQueueLen() == 1);  // node.go:289-308
    CHECK(c.node->RunRepairTasks() == 1);
    CHECK(stored_shard(*c.dn[3], "blk") == want[3]);
    CHECK(stored_shard(*c.dn[12], "blk") == want[12]);
    // a corrupted shard fails its CRC, is treated as a failed read and repaired
    c.dn[5]->server().CorruptByte("blk", 100);
    CHECK_OK(c.node->Get("blk", &got));
    CHECK(got == block);
    CHECK(c.node->RunRepairTasks() == 1);
    CHECK(stored_shard(*c.dn[5], "blk") == want[5]);
    // background worker variant
    c.dn[0]->server().Delete("blk");
    c.node->StartRepairWorker();
    CHECK_OK(c.node->Get("blk", &got));
    for (int i = 0; i < 200 && stored_shard(*c.dn[0], "blk").empty(); i++) {
        struct timespec ts = {0, 10 * 1000 * 1000};
        nanosleep(&ts, nullptr);
    }
    CHECK(stored_shard(*c.dn[0], "blk") == want[0]);
    c.node->Close();
}

static void test_repair_datanode(bool batched) {
    const int k = 10, m = 4, n = k + m;
    Cluster c(k, m);
    std::mt19937_64 r(batched ? 11 : 13);
    std::vector<std::string> keys;
    std::vector<Bytes> blocks;
    for (int i = 0; i < 40; i++) {
        keys.push_back("key-" + std::to_string(i));
        blocks.push_back(rand_bytes(r, i % 3 == 0 ? big() : (i % 3 == 1 ? 1000 + i : 65536)));
        CHECK_OK(c.node->Put(keys.back(), blocks.back()));
    }
    // datanode 6 is replaced by an empty one; one more node is down during the repair
    c.dn[6]->server().Wipe();
    c.dn[2]->SetOffline(true);
    size_t repaired = 0;
    if (batched)
        CHECK_OK(c.node->RepairDataNodeBatched(0, 6, 16, &repaired));
    else
        CHECK_OK(c.node->RepairDataNodePerKey(0, 6));
    if (batched) CHECK(repaired == keys.size());
    c.dn[2]->SetOffline(false);
    for (size_t i = 0; i < keys.size(); i++) {
        auto want = oracle_shards(k, m, blocks[i]);
        CHECK(stored_shard(*c.dn[6], keys[i]) == want[6]);
    }
    // RepairDataNode itself (the batched form), onto the node wiped again: the same rows
    if (!batched) {
        c.dn[6]->server().Wipe();
        c.dn[2]->SetOffline(true);
        CHECK_OK(c.node->RepairDataNode(0, 6));
        c.dn[2]->SetOffline(false);
        for (size_t i = 0; i < keys.size(); i++) CHECK(stored_shard(*c.dn[6], keys[i]) == oracle_shards(k, m, blocks[i])[6]);
    }
    // a target that fails its writes: the first failing flush's error comes back (the next
    // window's fetch, running ahead on a helper thread, only read), and nothing counts as repaired
    if (batched) {
        c.dn[6]->server().Wipe();
        c.dn[6]->SetOffline(true);
        size_t rep2 = 99;
        Status s = c.node->RepairDataNodeBatched(0, 6, 4, &rep2);
        CHECK(!s.ok() && s.err.find("rpc error") == 0);
        CHECK(rep2 == 99);  // not written on failure
        c.dn[6]->SetOffline(false);
    }
    // bad indexes (data_recovery.go:17-22)
    CHECK(c.node->RepairDataNode(n, 0).err == "index greater than max index of nodes");
    CHECK(c.node->RepairDataNode(0, n).err == "repair index greater than max index of nodes");
}

static void test_putmany_batch() {
    const int k = 4, m = 2;
    Cluster c(k, m);
    std::mt19937_64 r(5);
    std::vector<std::string> keys;
    std::vector<Bytes> blocks;
    for (int i = 0; i < 64; i++) {
        keys.push_back("pm-" + std::to_string(i));
        blocks.push_back(rand_bytes(r, i % 2 ? big() : 4097));
    }
    blocks[7].clear();  // an empty block travels the per-block path
    CHECK_OK(c.node->PutMany(keys, blocks));
    for (size_t i = 0; i < keys.size(); i++) {
        if (blocks[i].empty()) continue;
        auto want = oracle_shards(k, m, blocks[i]);
        for (int j = 0; j < k + m; j++) CHECK(stored_shard(*c.dn[j], keys[i]) == want[j]);
        Bytes got;
        CHECK_OK(c.node->Get(keys[i], &got));
        CHECK(got == blocks[i]);
    }
    // empty block: Put succeeds, Get fails with ErrShardNoData
    Bytes got;
    Status s = c.node->Get(keys[7], &got);
    CHECK(!s.ok() && s.err == "no shard data");
    int size = -1;
    CHECK_OK(c.node->GetSize(keys[7], &size));
    CHECK(size == 0);
}

static void test_getmany() {
    const int k = 10, m = 4;
    Cluster c(k, m);
    std::mt19937_64 r(21);
    std::vector<std::string> keys;
    std::vector<Bytes> blocks;
    for (int i = 0; i < 60; i++) {
        keys.push_back("gm-" + std::to_string(i));
        blocks.push_back(rand_bytes(r, i % 4 == 0 ? big() : (i % 4 == 1 ? 6 : (i % 4 == 2 ? 65537 : g_leaf))));
        CHECK_OK(c.node->Put(keys.back(), blocks.back()));
    }
    // shards lost in different patterns: node 1 down, some keys missing a data shard on
    // node 4, one key missing more than m shards (unreadable), one absent key
    c.dn[1]->SetOffline(true);
    for (int i = 0; i < 60; i += 3) c.dn[4]->server().Delete(keys[i]);
    for (int j = 5; j <= 9; j++) c.dn[j]->server().Delete(keys[7]);
    keys.push_back("absent");
    std::vector<Bytes> got;
    std::vector<Status> st;
    c.node->GetMany(keys, &got, &st, 8);
    for (size_t i = 0; i < 60; i++) {
        if (i == 7) {
            CHECK(!st[i].ok());
            continue;
        }
        CHECK_OK(st[i]);
        CHECK(got[i] == blocks[i]);
        Bytes one;  // same answer as the per-key Get
        CHECK_OK(c.node->Get(keys[i], &one));
        CHECK(one == blocks[i]);
    }
    CHECK(!st[60].ok() && st[60].err == "Key not found");
    CHECK(c.node->RepairQueueLen() > 0);  // read-repairs queued exactly as Get does
}

// Batches larger than one staging chunk (64 MiB: 12 blocks of RS(16,4) x 4 MiB): PutMany
// encodes in 3 chunks, GetMany works 25 keys at a time and decodes each group in chunks.
static void test_batches_span_staging_chunks() {
    const int k = 16, m = 4;
    Cluster c(k, m);
    std::mt19937_64 r(77);
    std::vector<std::string> keys;
    std::vector<Bytes> blocks;
    for (int i = 0; i < 30; i++) {
        keys.push_back("big-" + std::to_string(i));
        blocks.push_back(rand_bytes(r, g_huge));
    }
    CHECK_OK(c.node->PutMany(keys, blocks));
    for (int i : {0, 11, 12, 23, 24, 29}) {  // chunk edges
        auto want = oracle_shards(k, m, blocks[i]);
        for (int j = 0; j < k + m; j++) CHECK(stored_shard(*c.dn[j], keys[i]) == want[j]);
    }
    c.dn[0]->SetOffline(true);
    c.dn[9]->SetOffline(true);
    std::vector<Bytes> got;
    std::vector<Status> st;
    c.node->GetMany(keys, &got, &st, 25);
    for (size_t i = 0; i < keys.size(); i++) {
        CHECK_OK(st[i]);
        CHECK(got[i] == blocks[i]);
    }
}

static void test_migrate() {
    Cluster from(10, 4), to(4, 2);
    std::mt19937_64 r(99);
    std::vector<std::string> keys;
    std::vector<Bytes> blocks;
    for (int i = 0; i < 24; i++) {
        keys.push_back("mig-" + std::to_string(i));
        blocks.push_back(rand_bytes(r, i % 2 ? big() : 777));
        CHECK_OK(from.node->Put(keys.back(), blocks.back()));
    }
    from.dn[0]->SetOffline(true);  // the source set is degraded during the move
    keys.push_back("never-stored");
    std::vector<Status> st;
    MigrateBlocks(*from.node, *to.node, keys, &st, 5);
    from.dn[0]->SetOffline(false);
    for (size_t i = 0; i < keys.size(); i++) CHECK_OK(st[i]);
    for (size_t i = 0; i < blocks.size(); i++) {
        Bytes got;
        CHECK_OK(to.node->Get(keys[i], &got));
        CHECK(got == blocks[i]);
        auto want = oracle_shards(4, 2, blocks[i]);
        for (int j = 0; j < 6; j++) CHECK(stored_shard(*to.dn[j], keys[i]) == want[j]);
        bool has = true;
        from.node->Has(keys[i], &has);
        CHECK(!has);  // deleted from the source after the move
    }
}

// GPU entry checksums: entries stored through Put / PutMany with the
// checksum computed on the GPU are byte-identical to the datanode's own server.go:70 pass,
// and their checksum equals the oracle's for every shard, block size and batch shape.
static void test_gpu_entry_checksums() {
    for (auto km : {std::make_pair(2, 1), std::make_pair(10, 4), std::make_pair(16, 4)}) {
        const int k = km.first, m = km.second, n = k + m;
        Cluster gpu(k, m), host(k, m);
        host.node->SetGpuChecksums(false);
        std::mt19937_64 r(77 + k);
        std::vector<std::string> keys;
        std::vector<Bytes> blocks;
        const size_t sizes[] = {1, 6, 17, 4099, big(), big(1), g_leaf};
        for (size_t sz : sizes) {
            keys.push_back("single-" + std::to_string(sz));
            blocks.push_back(rand_bytes(r, sz));
            CHECK_OK(gpu.node->Put(keys.back(), blocks.back()));
            CHECK_OK(host.node->Put(keys.back(), blocks.back()));
        }
        std::vector<std::string> bk;
        std::vector<Bytes> bb;
        for (int i = 0; i < 37; i++) {
            bk.push_back("batch-" + std::to_string(i));
            bb.push_back(rand_bytes(r, big()));
        }
        CHECK_OK(gpu.node->PutMany(bk, bb));
        CHECK_OK(host.node->PutMany(bk, bb));
        keys.insert(keys.end(), bk.begin(), bk.end());
        blocks.insert(blocks.end(), bb.begin(), bb.end());
        for (size_t j = 0; j < keys.size(); j++) {
            auto want = oracle_shards(k, m, blocks[j]);
            Bytes meta(4);
            for (int b = 0; b < 4; b++) meta[b] = uint8_t(uint32_t(blocks[j].size()) >> (8 * b));
            for (int i = 0; i < n; i++) {
                Bytes eg, eh;
                CHECK(gpu.dn[i]->server().RawEntry(keys[j], &eg));
                CHECK(host.dn[i]->server().RawEntry(keys[j], &eh));
                CHECK(eg == eh);
                const uint32_t crc = uint32_t(eg[0]) | uint32_t(eg[1]) << 8 | uint32_t(eg[2]) << 16 | uint32_t(eg[3]) << 24;
                CHECK(crc == rs_oracle_datanode_entry_crc(meta.data(), 4, want[i].data(), want[i].size()));
            }
            Bytes got;
            CHECK_OK(gpu.node->Get(keys[j], &got));
            CHECK(got == blocks[j]);
        }
    }
}

// Mutcask-backed datanodes: PutMany hands every datanode both checksums from the GPU pass
// (R(shard) CRC-16 and R32(shard) CRC-32, rsmi_encode_batch_host_crcs); the stored values --
// |crc32|crc16|sizes|meta|shard| -- are byte-identical to the ones the datanodes compute
// themselves, and both checksums equal the oracle's.  Single Puts get both from the
// coalesced encode (rsmi_encode_block_coalesced_crcs).  Reads verify both.
static void test_gpu_value_checksums() {
    // the value CRC-32 from the GPU pass (SetGpuValueChecksums) and from each datanode's own
    // fold (the default): stored values byte-identical to the host-checksummed cluster's
    for (bool gpu32 : {true, false})
    for (auto km : {std::make_pair(2, 1), std::make_pair(10, 4), std::make_pair(16, 4)}) {
        const int k = km.first, m = km.second, n = k + m;
        Cluster gpu(k, m, KvEngine::Mutcask), host(k, m, KvEngine::Mutcask);
        gpu.node->SetGpuValueChecksums(gpu32);
        host.node->SetGpuChecksums(false);
        std::mt19937_64 r(91 + k);
        std::vector<std::string> keys;
        std::vector<Bytes> blocks;
        for (size_t sz : {size_t(6), size_t(4099), big()}) {
            keys.push_back("single-" + std::to_string(sz));
            blocks.push_back(rand_bytes(r, sz));
            CHECK_OK(gpu.node->Put(keys.back(), blocks.back()));
            CHECK_OK(host.node->Put(keys.back(), blocks.back()));
        }
        for (size_t sz : {size_t(17), big(), g_leaf}) {
            std::vector<std::string> bk;
            std::vector<Bytes> bb;
            for (int i = 0; i < 9; i++) {
                bk.push_back("batch-" + std::to_string(sz) + "-" + std::to_string(i));
                bb.push_back(rand_bytes(r, sz));
            }
            CHECK_OK(gpu.node->PutMany(bk, bb));
            CHECK_OK(host.node->PutMany(bk, bb));
            keys.insert(keys.end(), bk.begin(), bk.end());
            blocks.insert(blocks.end(), bb.begin(), bb.end());
        }
        for (size_t j = 0; j < keys.size(); j++) {
            auto want = oracle_shards(k, m, blocks[j]);
            Bytes meta(4);
            for (int b = 0; b < 4; b++) meta[b] = uint8_t(uint32_t(blocks[j].size()) >> (8 * b));
            for (int i = 0; i < n; i++) {
                Bytes vg, vh;
                CHECK(gpu.dn[i]->server().RawValue(keys[j], &vg));
                CHECK(host.dn[i]->server().RawValue(keys[j], &vh));
                CHECK(vg == vh);
                const uint32_t c16 = rs_oracle_datanode_entry_crc(meta.data(), 4, want[i].data(), want[i].size());
                CHECK(le32(vg, 4) == c16);
                CHECK(le32(vg, 0) == rs_oracle_mutcask_entry_crc(c16, meta.data(), 4, want[i].data(), want[i].size()));
            }
            Bytes got;
            CHECK_OK(gpu.node->Get(keys[j], &got));
            CHECK(got == blocks[j]);
        }
        // RepairDataNodeBatched onto a wiped mutcask node: the rebuilt rows carry both
        // checksums from the GPU (rsmi_reconstruct_rows_batch_host_crcs); every stored value
        // is byte-identical to the one written by the original Put
        std::vector<Bytes> before(keys.size());
        for (size_t j = 0; j < keys.size(); j++) CHECK(gpu.dn[1]->server().RawValue(keys[j], &before[j]));
        gpu.dn[1]->server().Wipe();
        size_t repaired = 0;
        CHECK_OK(gpu.node->RepairDataNodeBatched(0, 1, 8, &repaired));
        CHECK(repaired == keys.size());
        for (size_t j = 0; j < keys.size(); j++) {
            Bytes v;
            CHECK(gpu.dn[1]->server().RawValue(keys[j], &v) && v == before[j]);
        }
        // a rotted value on one datanode: the read treats that shard as missing and
        // reconstructs from the others (node.go:254-258), then read-repair rewrites it
        gpu.dn[0]->server().CorruptByte(keys.back(), kHeaderSize + 4 + 1);
        Bytes got;
        CHECK_OK(gpu.node->Get(keys.back(), &got));
        CHECK(got == blocks.back());
    }
}

// GPU-verified reads (SetGpuVerifiedReads): datanodes return shards with their stored
// checksums unchecked and the DagNode checks every fetch wave on the GPU.  A node that delivers
// a flipped byte (corrupted in transit: its GetMeta still passes) is caught there, treated as a
// failed fetch, and the block still comes back intact from the other shards, with the node on
// the read-repair list -- over badger and mutcask datanodes, for Get and GetMany.
struct FlippingNode : InProcDataNode {
    using InProcDataNode::InProcDataNode;
    bool flip = false;
    Status GetForVerify(const std::string& key, Bytes* meta, Bytes* data, Stored* st) override {
        Status s = InProcDataNode::GetForVerify(key, meta, data, st);
        if (s.ok() && flip && !data->empty()) (*data)[data->size() / 2] ^= 0x01;
        return s;
    }
};

static void test_gpu_verified_reads() {
    for (KvEngine engine : {KvEngine::Badger, KvEngine::Mutcask}) {
        const int k = 10, m = 4;
        DagNodeConfig cfg;
        cfg.name = "verify";
        cfg.data_blocks = k;
        cfg.parity_blocks = m;
        std::vector<std::shared_ptr<FlippingNode>> dn;
        std::vector<std::shared_ptr<DataNodeClient>> clients;
        for (int i = 0; i < k + m; i++) {
            cfg.nodes.push_back("127.0.0.1:" + std::to_string(9111 + i));
            dn.push_back(std::make_shared<FlippingNode>(cfg.nodes.back(), engine));
            clients.push_back(dn.back());
        }
        std::unique_ptr<DagNode> node;
        CHECK_OK(DagNode::New(cfg, clients, &node, g_devices));
        node->HealthCheckAll();
        node->SetGpuVerifiedReads(true);
        std::mt19937_64 r(21);
        std::vector<std::string> keys;
        std::vector<Bytes> blocks;
        for (size_t sz : {size_t(6), size_t(4099), big(), g_leaf}) {
            keys.push_back("v-" + std::to_string(sz));
            blocks.push_back(rand_bytes(r, sz));
            CHECK_OK(node->Put(keys.back(), blocks.back()));
        }
        for (size_t j = 0; j < keys.size(); j++) {
            Bytes got;
            CHECK_OK(node->Get(keys[j], &got));
            CHECK(got == blocks[j]);
        }
        CHECK(node->RepairQueueLen() == 0);
        dn[1]->flip = true;  // data shard 1 arrives corrupted
        for (size_t j = 0; j < keys.size(); j++) {
            Bytes got;
            CHECK_OK(node->Get(keys[j], &got));
            CHECK(got == blocks[j]);
        }
        CHECK(node->RepairQueueLen() == keys.size());
        std::vector<Bytes> gm;
        std::vector<Status> st;
        node->GetMany(keys, &gm, &st, 8);
        for (size_t j = 0; j < keys.size(); j++) {
            CHECK_OK(st[j]);
            CHECK(gm[j] == blocks[j]);
        }
        dn[1]->flip = false;
        // degraded GetMany: data node 0 down, so every key decodes from 10 survivors whose
        // checksums (badger) come out of the decode kernel itself; first all clean, then a
        // survivor corrupted in transit, which the decode's check catches
        dn[0]->SetOffline(true);
        for (int pass = 0; pass < 2; pass++) {
            dn[3]->flip = pass == 1;
            node->GetMany(keys, &gm, &st, 8);
            for (size_t j = 0; j < keys.size(); j++) {
                CHECK_OK(st[j]);
                CHECK(gm[j] == blocks[j]);
                Bytes one;
                CHECK_OK(node->Get(keys[j], &one));
                CHECK(one == blocks[j]);
            }
        }
        dn[3]->flip = false;
        dn[0]->SetOffline(false);
        node->Close();
    }
}

// Concurrent DagNode.Put from many threads (the reference's goroutine-per-request Dag Pool):
// the per-block encodes coalesce into GPU batches (rsmi_encode_block_coalesced), and every
// stored shard and entry checksum still equals the oracle's.
static void test_concurrent_puts() {
    const int k = 10, m = 4, n = k + m;
    Cluster c(k, m);
    const int T = 12, per = 10;
    std::vector<std::string> keys(size_t(T * per));
    std::vector<Bytes> blocks(size_t(T * per));
    std::mt19937_64 r(99);
    for (int i = 0; i < T * per; i++) {
        keys[i] = "conc-" + std::to_string(i);
        blocks[i] = rand_bytes(r, i % 7 == 0 ? 4099 : big());
    }
    int rc;
    rsmi_ctx* ctx = shared_context(k, m, 0, &rc);
    CHECK(ctx != nullptr);
    // the coalescing counters summed over the node's members
    auto lane_stat = [&](int kk, int mm, int, const char* key) {
        long v = 0;
        for (int i = 0; i < c.node->Members(); i++)
            v += rsmi::host::lane_stat(kk, mm, c.node->MemberDevice(i), key, c.node->MemberReplica(i));
        return v;
    };
    // every Put and degraded Get through the group commit (no lone-caller path), so the counters
    // are exact
    c.node->SetLoneCallerPaths(false);
    const long calls0 = lane_stat(k, m, 0, "coalesced_calls"), batches0 = lane_stat(k, m, 0, "coalesced_batches");
    std::vector<std::thread> th;
    std::vector<Status> st(size_t(T * per));
    for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {
            for (int j = 0; j < per; j++) st[size_t(t * per + j)] = c.node->Put(keys[t * per + j], blocks[t * per + j]);
        });
    for (auto& x : th) x.join();
    const long calls = lane_stat(k, m, 0, "coalesced_calls") - calls0;
    const long batches = lane_stat(k, m, 0, "coalesced_batches") - batches0;
    CHECK(calls == T * per);
    CHECK(batches >= 1 && batches <= calls);
    std::printf("concurrent puts: %ld encodes in %ld GPU batches\n", calls, batches);
    // degraded Gets from the same threads with data shard 2's node down: one erasure
    // pattern, so the per-key reconstructs coalesce; every block must come back intact
    c.dn[2]->SetOffline(true);
    const long rc0 = lane_stat(k, m, 0, "coalesced_calls"), rb0 = lane_stat(k, m, 0, "coalesced_batches");
    std::vector<Bytes> got(size_t(T * per));
    std::vector<Status> gst(size_t(T * per));
    th.clear();
    for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {
            for (int j = 0; j < per; j++) gst[size_t(t * per + j)] = c.node->Get(keys[t * per + j], &got[size_t(t * per + j)]);
        });
    for (auto& x : th) x.join();
    c.dn[2]->SetOffline(false);
    const long rcalls = lane_stat(k, m, 0, "coalesced_calls") - rc0, rbatches = lane_stat(k, m, 0, "coalesced_batches") - rb0;
    CHECK(rcalls == T * per);  // every Get misses data shard 2: one reconstruct each
    c.node->SetLoneCallerPaths(true);
    std::printf("concurrent degraded gets: %ld reconstructs in %ld GPU batches\n", rcalls, rbatches);
    for (int i = 0; i < T * per; i++) {
        CHECK_OK(gst[i]);
        CHECK(got[i] == blocks[i]);
    }
    for (int i = 0; i < T * per; i++) {
        CHECK_OK(st[i]);
        auto want = oracle_shards(k, m, blocks[i]);
        Bytes meta(4);
        for (int b = 0; b < 4; b++) meta[b] = uint8_t(uint32_t(blocks[i].size()) >> (8 * b));
        for (int s = 0; s < n; s++) {
            CHECK(stored_shard(*c.dn[s], keys[i]) == want[s]);
            Bytes e;
            CHECK(c.dn[s]->server().RawEntry(keys[i], &e));
            const uint32_t crc = uint32_t(e[0]) | uint32_t(e[1]) << 8 | uint32_t(e[2]) << 16 | uint32_t(e[3]) << 24;
            CHECK(crc == rs_oracle_datanode_entry_crc(meta.data(), 4, want[s].data(), want[s].size()));
        }
    }
}

// A Put whose codec call fails returns the error (node.go:382-386).  The block-only data shards
// were written while the GPU encoded (blocks above 1 MiB by the pool, smaller ones by the calling
// thread inside the codec call's wait, rsmi_set_wait_hook); they stay, holding
// exactly the bytes a successful Put stores (no parity, no padded row), as the reference leaves
// the shards of a Put whose write quorum fails.  A block stored earlier under the same key (keys
// are content ids) stays readable through a failed repeat Put.  The failure is the coalescer's
// host-fault test hook (RSMI_ERR_HOST); the next Put succeeds.
static void test_put_codec_failure() {
    const int k = 10, m = 4, n = k + m;
    Cluster c(k, m);
    int rc;
    std::mt19937_64 r(404);
    auto arm = [&](int v) {  // a member the key did not reach keeps its fault armed until disarmed
        for (int i = 0; i < c.node->Members(); i++) {
            rsmi_ctx* x = shared_context(k, m, c.node->MemberDevice(i), &rc, c.node->MemberReplica(i));
            if (v)
                CHECK(x && rsmi_set_option(x, "inject_host_fault", 1) == RSMI_OK);
            else if (x)
                (void)rsmi_set_option(x, "inject_host_fault", 0);
        }
    };
    // through the group commit (lone paths off, where the hook fails a batch) and as a lone caller
    // (the hook fails the direct call); modes 0 and 3 written inside the wait, 1 and 2 by the pool
    for (const int mode : {0, 1, 2, 3}) {
        const bool lone = mode >= 2;
        c.node->SetLoneCallerPaths(lone);
        const Bytes block = rand_bytes(r, mode == 1 || mode == 2 ? size_t(k) * 131072 + 17 : big());
        const std::string key = "codec-fails-" + std::to_string(mode);
        const auto want = oracle_shards(k, m, block);
        arm(1);
        Status s = c.node->Put(key, block);
        CHECK(!s.ok());
        for (int j = 0; j < n; j++) {
            const Bytes got = stored_shard(*c.dn[j], key);
            CHECK(got.empty() || (j < k - 1 && got == want[j]));  // never parity, never wrong bytes
        }
        arm(0);
        CHECK_OK(c.node->Put(key, block));
        for (int j = 0; j < n; j++) CHECK(stored_shard(*c.dn[j], key) == want[j]);
        // the same block Put again with the codec failing: the stored block survives it
        arm(1);
        CHECK(!c.node->Put(key, block).ok());
        arm(0);
        for (int j = 0; j < n; j++) CHECK(stored_shard(*c.dn[j], key) == want[j]);
        Bytes got;
        CHECK_OK(c.node->Get(key, &got));
        CHECK(got == block);
    }
    c.node->SetLoneCallerPaths(true);
}

// A Dag Node on a device list (DagNode::New): every per-key call codes on the member that owns the
// key's hash slot (hash_slot.go:20-22, crc16 IBM of the key & 0x3FFF, in contiguous ranges of
// 16384 / members slots), and each member's group-commit queue sees exactly its own keys.  The two
// members name the same device (one GPU per test box; the sanitizer build's fake device layer).
static void test_member_routing() {
    const int k = 10, m = 4, n = k + m;
    const std::vector<int> saved = g_devices;
    g_devices = {0, 0};
    Cluster c(k, m);
    g_devices = saved;
    CHECK(c.node->Members() == 2);
    CHECK(c.node->MemberReplica(0) == 0 && c.node->MemberReplica(1) == 1);
    c.node->SetLoneCallerPaths(false);  // per-block Put through the member's group commit
    long before[2], expect[2] = {0, 0};
    for (int r = 0; r < 2; r++) before[r] = lane_stat(k, m, 0, "coalesced_calls", r);
    std::mt19937_64 rng(31);
    for (int i = 0; i < 48; i++) {
        const std::string key = "bafkrei-route-" + std::to_string(i);
        const int slot = rs_oracle_crc16_ibm(reinterpret_cast<const uint8_t*>(key.data()), key.size()) & 0x3FFF;
        const int want = slot * 2 / 16384;
        CHECK(c.node->MemberOfKey(key) == want);
        expect[want]++;
        const Bytes b = rand_bytes(rng, size_t(1000 + 97 * i));
        CHECK_OK(c.node->Put(key, b));
        const auto sh = oracle_shards(k, m, b);
        for (int j = 0; j < n; j++) CHECK(stored_shard(*c.dn[j], key) == sh[j]);
    }
    for (int r = 0; r < 2; r++) CHECK(lane_stat(k, m, 0, "coalesced_calls", r) - before[r] == expect[r]);
    CHECK(expect[0] > 0 && expect[1] > 0);
    c.node->SetLoneCallerPaths(true);
    // four members: the slot's quarter
    g_devices = {0, 0, 0, 0};
    Cluster c4(2, 1);
    g_devices = saved;
    for (int i = 0; i < 64; i++) {
        const std::string key = "QmRoute" + std::to_string(i * 7919);
        const int slot = rs_oracle_crc16_ibm(reinterpret_cast<const uint8_t*>(key.data()), key.size()) & 0x3FFF;
        CHECK(c4.node->MemberOfKey(key) == slot * 4 / 16384);
    }
    // an empty device list is refused
    DagNodeConfig cfg;
    cfg.data_blocks = 2;
    cfg.parity_blocks = 1;
    std::vector<std::shared_ptr<DataNodeClient>> cl;
    for (int i = 0; i < 3; i++) {
        cfg.nodes.push_back("x" + std::to_string(i));
        cl.push_back(std::make_shared<InProcDataNode>(cfg.nodes.back()));
    }
    std::unique_ptr<DagNode> d;
    CHECK(!DagNode::New(cfg, cl, &d, std::vector<int>{}).ok());
}

// group_commit.hpp: an executor whose batch throws completes every request of that batch with
// the fail code and releases the executor role, so concurrent and later callers still finish
// (a throwing exec used to leave executing_ set and every caller waiting forever).
static void test_group_commit_exec_throws() {
    struct Req {
        int id = 0, rc = -1;
        bool done = false;
    };
    rsmi::GroupCommit<Req> gc(-7);
    std::atomic<int> throws{0};
    auto exec = [&](std::vector<Req*>& batch, int) {
        for (Req* r : batch)
            if (r->id % 3 == 0) {  // a batch holding any multiple of 3 fails as a whole
                throws++;
                throw std::bad_alloc();
            }
        for (Req* r : batch) r->rc = r->id;
    };
    std::vector<Req> reqs(48);
    std::vector<std::thread> th;
    for (int t = 0; t < 8; t++)
        th.emplace_back([&, t] {
            for (int i = t; i < 48; i += 8) {
                reqs[size_t(i)].id = i;
                gc.submit(reqs[size_t(i)], 4, 50, 1, exec);
            }
        });
    for (auto& x : th) x.join();
    int failed = 0;
    for (int i = 0; i < 48; i++) {
        const Req& r = reqs[size_t(i)];
        CHECK(r.done && (r.rc == i || r.rc == -7));
        if (i % 3 == 0) CHECK(r.rc == -7);  // its own batch threw
        failed += r.rc == -7;
    }
    CHECK(throws.load() >= 1 && failed >= 16 && gc.calls() == 48);
    Req last;
    last.id = 100;
    gc.submit(last, 4, 0, 1, exec);  // the queue still works after the failures
    CHECK(last.done && last.rc == 100);
}

// The grouping checks below need callers to pile up behind a running batch; on a loaded machine
// (a sanitizer build beside other jobs) the threads may otherwise run one after another, each
// call its own batch.  The first batch therefore waits (up to a second) until every thread has
// entered submit, then a little longer for them to queue.
static void hold_first_batch(std::atomic<bool>& first, const std::atomic<int>& entered, int T) {
    if (!first.exchange(false)) return;
    const auto until = std::chrono::steady_clock::now() + std::chrono::seconds(1);
    while (entered.load() < T && std::chrono::steady_clock::now() < until) std::this_thread::yield();
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
}

// group_commit.hpp with several lanes (and lanes that carry on to queued batches): at most
// `lanes` batches execute at once, the batches
// executing at once hold distinct lane ids, every request completes exactly once with its own
// result, and the calls group (fewer batches than calls when callers pile up behind busy lanes).
static void test_group_commit_lanes() {
    struct Req {
        int id = 0, rc = -1;
        bool done = false;
    };
    const int T = 12, per = 20;
    for (int lanes : {1, 2, 3})
    for (int carry : {0, 2}) {
        rsmi::GroupCommit<Req> gc(-7);
        std::atomic<int> running{0}, peak{0}, overlap{0};
        std::atomic<uint32_t> busy{0};
        std::atomic<int> executed{0}, entered{0};
        std::atomic<bool> first{true};
        auto exec = [&](std::vector<Req*>& batch, int lane) {
            hold_first_batch(first, entered, T);
            const uint32_t bit = 1u << lane;
            if (lane < 0 || lane >= lanes || (busy.fetch_or(bit) & bit)) overlap++;  // lane id in use twice
            const int now = ++running;
            for (int p = peak.load(); now > p && !peak.compare_exchange_weak(p, now);) {
            }
            std::this_thread::sleep_for(std::chrono::microseconds(200));
            for (Req* r : batch) {
                r->rc = r->id;
                executed++;
            }
            running--;
            busy.fetch_and(~bit);
        };
        std::vector<Req> reqs(size_t(T * per));
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] {
                for (int i = t; i < T * per; i += T) {
                    reqs[size_t(i)].id = i;
                    entered++;
                    gc.submit(reqs[size_t(i)], 256, 0, lanes, exec, carry);
                }
            });
        for (auto& x : th) x.join();
        for (int i = 0; i < T * per; i++) CHECK(reqs[size_t(i)].done && reqs[size_t(i)].rc == i);
        CHECK(overlap.load() == 0);
        CHECK(peak.load() >= 1 && peak.load() <= lanes);
        CHECK(executed.load() == T * per && gc.calls() == uint64_t(T * per));
        CHECK(gc.batches() < gc.calls());
        std::printf("group commit, %d lane(s), carry %d: %llu calls in %llu batches, at most %d at once\n", lanes,
                    carry, (unsigned long long)gc.calls(), (unsigned long long)gc.batches(), peak.load());
    }
}

// group_commit.hpp with pipelined batches: exec launches and returns a finisher, and the executor
// launches the next queued batch before it finishes the current one.  Per lane, finishers run
// once each in launch order, at most two batches of a lane are in flight, a request's caller
// returns only after its batch's finisher ran, and a finisher's error reaches its requests.
#ifndef __SANITIZE_THREAD__  // ThreadSanitizer does not follow C++ exception unwinding (see main)
constexpr bool kThrowingFinishers = true;
#else
constexpr bool kThrowingFinishers = false;
#endif
static void test_group_commit_pipelined() {
    struct Req {
        int id = 0, rc = -1;
        bool done = false;
        std::atomic<int> finished{0};
    };
    const int T = 12, per = 20;
    for (int lanes : {1, 2})
    for (int carry : {1, 3}) {
        rsmi::GroupCommit<Req> gc(-7);
        std::mutex mu;
        std::vector<std::vector<int>> launched(static_cast<size_t>(lanes)), finished(static_cast<size_t>(lanes));
        std::atomic<int> seq{0}, bad{0}, deep{0}, entered{0};
        std::atomic<bool> first{true};
        std::vector<std::atomic<int>> inflight(static_cast<size_t>(lanes));
        auto exec = [&](std::vector<Req*>& batch, int lane) -> std::function<void()> {
            hold_first_batch(first, entered, T);
            const int b = seq++;
            {
                std::lock_guard<std::mutex> g(mu);
                launched[size_t(lane)].push_back(b);
            }
            if (++inflight[size_t(lane)] > 2) deep++;
            for (Req* r : batch) r->rc = r->id;
            std::vector<Req*> mine = batch;
            return [&, b, lane, mine]() {
                std::this_thread::sleep_for(std::chrono::microseconds(150));
                {
                    std::lock_guard<std::mutex> g(mu);
                    finished[size_t(lane)].push_back(b);
                }
                bool boom = false;
                for (Req* r : mine) {
                    if (r->done) bad++;  // its caller may not have returned yet
                    r->finished++;
                    if (r->id % 37 == 5) r->rc = -3;  // an error found by the wait
                    boom |= kThrowingFinishers && r->id % 53 == 7;
                }
                inflight[size_t(lane)]--;
                if (boom) throw std::bad_alloc();  // the wait itself fails: the batch completes with the fail code
            };
        };
        std::vector<Req> reqs(size_t(T * per));
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] {
                for (int i = t; i < T * per; i += T) {
                    reqs[size_t(i)].id = i;
                    entered++;
                    gc.submit(reqs[size_t(i)], 6, 0, lanes, exec, carry);
                }
            });
        for (auto& x : th) x.join();
        // a request whose batch's finisher threw completes with the fail code (-7); which other
        // requests shared that batch depends on timing, so only the thrower's own rc is fixed
        for (int i = 0; i < T * per; i++) {
            const Req& r = reqs[size_t(i)];
            CHECK(r.done && r.finished.load() == 1);
            if (kThrowingFinishers && i % 53 == 7) CHECK(r.rc == -7);
            else CHECK(r.rc == -7 || r.rc == (i % 37 == 5 ? -3 : i));
        }
        CHECK(bad.load() == 0 && deep.load() == 0);
        for (int l = 0; l < lanes; l++) CHECK(launched[size_t(l)] == finished[size_t(l)]);
        CHECK(gc.calls() == uint64_t(T * per) && gc.batches() < gc.calls());
        std::printf("group commit pipelined, %d lane(s), carry %d: %llu calls in %llu batches\n", lanes, carry,
                    (unsigned long long)gc.calls(), (unsigned long long)gc.batches());
    }
}

// group_commit.hpp idle tasks (the engine side of rsmi_set_wait_hook): every caller's task runs
// exactly once, on the caller's own thread, before its submit returns; a lone caller's task runs
// while its batch is in flight (after exec launched it, before its finisher); every request still
// completes with its own result, over 1..3 lanes, with plain and pipelined execs.
static void test_group_commit_idle() {
    struct Req {
        int id = 0, rc = -1;
        bool done = false;
    };
    struct Task {
        std::atomic<int> runs{0};
        std::thread::id ran_on;
        int id = 0;
        const std::atomic<int>* launched = nullptr;  // per request: 1 once launched, 2 once finished
        std::atomic<int> saw = {0};                  // the state of the task's own batch when it ran
    };
    auto task = [](void* p) {
        auto* t = static_cast<Task*>(p);
        t->ran_on = std::this_thread::get_id();
        if (t->launched) t->saw = t->launched[t->id].load();
        std::this_thread::sleep_for(std::chrono::microseconds(30));
        t->runs++;
    };
    // one caller: every batch is its own request alone, so the task overlaps the batch
    {
        rsmi::GroupCommit<Req> gc(-7);
        std::vector<std::atomic<int>> state(40);
        auto exec = [&](std::vector<Req*>& batch, int) -> std::function<void()> {
            for (Req* r : batch) {
                r->rc = r->id;
                state[size_t(r->id)] = 1;
            }
            std::vector<Req*> mine = batch;
            return [&state, mine]() {
                for (Req* r : mine) state[size_t(r->id)] = 2;
            };
        };
        for (int i = 0; i < 40; i++) {
            Req r;
            r.id = i;
            Task t;
            t.id = i;
            t.launched = state.data();
            gc.submit(r, 8, 0, 2, exec, 1, +task, &t);
            CHECK(r.done && r.rc == i && t.runs.load() == 1 && t.saw.load() == 1);
            CHECK(t.ran_on == std::this_thread::get_id());
        }
    }
    const int T = 12, per = 15;
    for (int lanes : {1, 2, 3})
    for (int piped : {0, 1}) {
        rsmi::GroupCommit<Req> gc(-7);
        std::atomic<int> entered{0};
        std::atomic<bool> first{true};
        auto plain = [&](std::vector<Req*>& batch, int) {
            hold_first_batch(first, entered, T);
            std::this_thread::sleep_for(std::chrono::microseconds(100));
            for (Req* r : batch) r->rc = r->id;
        };
        auto pipe = [&](std::vector<Req*>& batch, int) -> std::function<void()> {
            hold_first_batch(first, entered, T);
            for (Req* r : batch) r->rc = r->id;
            return [] { std::this_thread::sleep_for(std::chrono::microseconds(100)); };
        };
        std::vector<Req> reqs(size_t(T * per));
        std::vector<Task> tasks(size_t(T * per));
        std::vector<std::thread> th;
        std::atomic<int> wrong_thread{0}, early{0};
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] {
                for (int i = t; i < T * per; i += T) {
                    reqs[size_t(i)].id = i;
                    entered++;
                    if (piped)
                        gc.submit(reqs[size_t(i)], 6, 0, lanes, pipe, 1, +task, &tasks[size_t(i)]);
                    else
                        gc.submit(reqs[size_t(i)], 6, 0, lanes, plain, 1, +task, &tasks[size_t(i)]);
                    if (tasks[size_t(i)].runs.load() != 1) early++;  // ran before submit returned
                    if (tasks[size_t(i)].ran_on != std::this_thread::get_id()) wrong_thread++;
                }
            });
        for (auto& x : th) x.join();
        for (int i = 0; i < T * per; i++) {
            CHECK(reqs[size_t(i)].done && reqs[size_t(i)].rc == i);
            CHECK(tasks[size_t(i)].runs.load() == 1);
        }
        CHECK(early.load() == 0 && wrong_thread.load() == 0);
        CHECK(gc.calls() == uint64_t(T * per) && gc.batches() < gc.calls());
        std::printf("group commit with idle tasks, %d lane(s), %s: %llu calls in %llu batches\n", lanes,
                    piped ? "pipelined" : "plain", (unsigned long long)gc.calls(), (unsigned long long)gc.batches());
    }
}

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "cpu";
    if (rs_oracle_selftest() != 0) {
        std::fprintf(stderr, "oracle selftest failed\n");
        return 2;
    }
    test_datanode_server();
    test_datanode_sender_checksum();
    test_datanode_mutcask();
    test_quorum_helpers();
    test_config_and_slots();
#ifndef __SANITIZE_THREAD__  // ThreadSanitizer does not follow C++ exception unwinding (it reports a
                             // double lock on the queue's mutex once a throw has crossed a frame)
    test_group_commit_exec_throws();
#endif
    test_group_commit_lanes();
    test_group_commit_pipelined();
    test_group_commit_idle();
    if (mode == "sanitize") {  // the Dag Node suite at 1/32 scale on the fake device layer
        g_big /= 32;
        g_leaf = g_leaf / 32 + 14;
        g_huge /= 32;
        g_fanout_min = 0;
    }
    if (mode == "gpu" || mode == "sanitize") {
        test_dagnode_123456();
        test_rs10_4_failures();
        test_read_repair();
        test_repair_datanode(false);
        test_repair_datanode(true);
        test_putmany_batch();
        test_getmany();
        test_batches_span_staging_chunks();
        test_migrate();
        test_gpu_entry_checksums();
        test_gpu_value_checksums();
        test_gpu_verified_reads();
        test_concurrent_puts();
        test_put_codec_failure();
        test_member_routing();
        // the member pass: the Dag Node tests again on a two-member device list, every shard
        // and block still the oracle's
        const int before = g_checks;
        g_devices = {0, 0};
        test_dagnode_123456();
        test_rs10_4_failures();
        test_read_repair();
        test_repair_datanode(false);
        test_repair_datanode(true);
        test_putmany_batch();
        test_getmany();
        test_batches_span_staging_chunks();
        test_migrate();
        test_gpu_entry_checksums();
        test_gpu_verified_reads();
        test_concurrent_puts();
        test_put_codec_failure();
        g_devices = {0};
        std::printf("member pass: %d checks\n", g_checks - before);
    }
    release_shared_contexts();
    std::printf("%s: %d checks, %d failed\n", mode.c_str(), g_checks, g_fail);
    return g_fail ? 1 : 0;
}
