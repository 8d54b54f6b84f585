// datanode.hpp -- the datanode shard store behind a DataNodeClient interface.
//
// Mirrors dag/node/datanode/server.go: a shard is stored as one entry
//   | crc (4 B LE) | meta size (4 B LE) | data size (4 B LE) | meta | data |     (server.go:40-41)
// whose crc is CRC-16 "IBM" over every byte after the crc field (server.go:70), checked on
// Get/GetMeta (server.go:93-97, :115-119).  The KV engine below it (badger / mutcask,
// server.go:183-238) is out of scope as storage; an in-memory map stands in, with badger's
// rule that keys must be non-empty.  Its checksum is not: with the mutcask engine
// (server.go:207) every value is stored as | crc32 (4 B LE) | entry | (kv/mutcask/cask.go:73-79,
// Go crc32.ChecksumIEEE) and re-checked on every read (cask.go:81-97, :250), a second
// byte-serial pass over each shard that a sender can precompute (PutWithChecksums).  DataNodeClient mirrors proto.DataNodeClient
// (dag/proto/datanode.proto:9-17) so the DagNode talks to any implementation, and an
// in-process client can be switched offline to exercise the quorum paths.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace rsmi {
namespace host {

using Bytes = std::vector<uint8_t>;

// A read-only view of bytes: what a Go []byte argument is (node.go:376-399 hands each datanode a
// sub-slice of the one buffer Split + Encode filled, with no copy).  Built from a Bytes or from
// a pointer and a length; the caller keeps the bytes alive for the call.
class ByteView {
public:
    ByteView(const Bytes& b) : p_(b.data()), n_(b.size()) {}  // NOLINT: implicit, like a slice
    ByteView(const uint8_t* p, size_t n) : p_(p), n_(n) {}
    const uint8_t* data() const { return p_; }
    size_t size() const { return n_; }
    bool empty() const { return n_ == 0; }
    Bytes bytes() const { return Bytes(p_, p_ + n_); }

private:
    const uint8_t* p_;
    size_t n_;
};

// A Go-style error value: ok() when empty.
struct Status {
    std::string err;
    bool ok() const { return err.empty(); }
    static Status Ok() { return {}; }
    static Status Error(std::string e) { return Status{std::move(e)}; }
};

// howeyc/crc16 Checksum(data, IBMTable) as restated in SURVEY.md 8(a) a10: reflected
// polynomial 0xA001, register complemented on entry and exit (CRC-16/USB; check value
// 0xB4C8).  The upstream source is absent, so this variant is parity-unpinned.
uint16_t crc16_ibm(const uint8_t* p, size_t n, uint16_t crc = 0);
// Go crc32.ChecksumIEEE (the zlib CRC-32), slice-by-8
uint32_t crc32_ieee(const uint8_t* p, size_t n);

// server.go:29-35 KVType: the engine under the datanode
enum class KvEngine { Badger, Mutcask };

constexpr int kHeaderSize = 12;  // server.go:37

class DataNodeClient {
public:
    virtual ~DataNodeClient() = default;
    virtual Status Put(const std::string& key, const Bytes& meta, ByteView data) = 0;
    // Put with the entry checksum computed by the sender (the DagNode gets R(shard) from the
    // GPU encode).  Over gRPC this is an optional AddRequest field; a
    // datanode without it recomputes, which is what this default does.
    virtual Status PutWithChecksum(const std::string& key, const Bytes& meta, ByteView data, uint16_t crc) {
        (void)crc;
        return Put(key, meta, data);
    }
    // ... and with the mutcask value checksum of that entry as well (cask.go:73-79), for a
    // datanode whose engine keeps one (WantsValueChecksum); others drop it
    virtual Status PutWithChecksums(const std::string& key, const Bytes& meta, ByteView data, uint16_t crc,
                                    uint32_t value_crc) {
        (void)value_crc;
        return PutWithChecksum(key, meta, data, crc);
    }
    virtual bool WantsValueChecksum() const { return false; }
    // A Get whose checksum check the caller makes (GPU-verified reads): the shard plus the
    // checksums stored with it, unchecked (*verified = false); value_crc is the mutcask value
    // checksum when *has_value_crc.  A datanode without this RPC runs its verified Get
    // (*verified = true), which is what this default does.
    struct Stored {
        uint16_t crc = 0;
        uint32_t value_crc = 0;
        bool has_value_crc = false;
        bool verified = true;
    };
    virtual Status GetForVerify(const std::string& key, Bytes* meta, Bytes* data, Stored* st) {
        *st = Stored{};
        return Get(key, meta, data);
    }
    virtual Status Get(const std::string& key, Bytes* meta, Bytes* data) = 0;
    virtual Status GetMeta(const std::string& key, Bytes* meta) = 0;
    virtual Status Delete(const std::string& key) = 0;
    virtual Status Size(const std::string& key, int64_t* size) = 0;
    virtual Status AllKeys(std::vector<std::string>* keys) = 0;  // AllKeysChan
    virtual bool Healthy() = 0;                                   // grpc.health Check
    virtual std::string Address() const = 0;
};

// server.go's `server` over an in-memory KV.
class DataNodeServer {
public:
    explicit DataNodeServer(KvEngine engine = KvEngine::Badger) : engine_(engine) {}
    KvEngine engine() const { return engine_; }
    Status Put(const std::string& key, const Bytes& meta, ByteView data);
    // the same entry, with the sender's checksum in place of the server.go:70 CRC pass; Get
    // and GetMeta still verify it, so a wrong sender checksum fails the read like corruption
    Status PutWithChecksum(const std::string& key, const Bytes& meta, ByteView data, uint16_t crc);
    // mutcask: the value checksum too (a wrong one fails later reads with "data may be rotted")
    Status PutWithChecksums(const std::string& key, const Bytes& meta, ByteView data, uint16_t crc,
                            uint32_t value_crc);
    Status Get(const std::string& key, Bytes* meta, Bytes* data);
    // the entry's parts and stored checksums without checking either (the reader verifies)
    Status GetUnverified(const std::string& key, Bytes* meta, Bytes* data, DataNodeClient::Stored* st);
    Status GetMeta(const std::string& key, Bytes* meta);
    Status Delete(const std::string& key);
    Status Size(const std::string& key, int64_t* size);
    Status AllKeys(std::vector<std::string>* keys);
    // test hooks: the datanode entry, the KV engine's stored value (mutcask: crc32 + entry),
    // and a flipped byte at an entry offset
    bool RawEntry(const std::string& key, Bytes* entry);
    bool RawValue(const std::string& key, Bytes* value);
    void CorruptByte(const std::string& key, size_t offset);
    void Wipe();

private:
    // a stored value: len bytes in a buffer of cap bytes
    struct Value {
        std::unique_ptr<uint8_t[]> p;
        size_t len = 0, cap = 0;
        const uint8_t* data() const { return p.get(); }
        size_t size() const { return len; }
    };
    Status store(const std::string& key, const Bytes& meta, ByteView data, const uint16_t* crc,
                 const uint32_t* value_crc);
    Status read_entry(const std::string& key, const Value** entry);  // caller holds mu_
    size_t prefix() const { return engine_ == KvEngine::Mutcask ? 4 : 0; }
    KvEngine engine_;
    std::mutex mu_;
    std::map<std::string, Value> kv_;
    // replaced values kept for reuse: an overwrite frames into a recycled buffer instead of a
    // fresh allocation (whose pages the kernel would fault in again on every Put of a key)
    std::vector<Value> spare_;
    static constexpr size_t kSpareValues = 64;
};

// An in-process client; Offline(true) makes every call fail like a dead gRPC peer.
class InProcDataNode : public DataNodeClient {
public:
    explicit InProcDataNode(std::string addr, KvEngine engine = KvEngine::Badger)
        : addr_(std::move(addr)), server_(engine) {}
    Status Put(const std::string& key, const Bytes& meta, ByteView data) override;
    Status PutWithChecksum(const std::string& key, const Bytes& meta, ByteView data, uint16_t crc) override;
    Status PutWithChecksums(const std::string& key, const Bytes& meta, ByteView data, uint16_t crc,
                            uint32_t value_crc) override;
    bool WantsValueChecksum() const override { return server_.engine() == KvEngine::Mutcask; }
    Status Get(const std::string& key, Bytes* meta, Bytes* data) override;
    Status GetForVerify(const std::string& key, Bytes* meta, Bytes* data, Stored* st) override;
    Status GetMeta(const std::string& key, Bytes* meta) override;
    Status Delete(const std::string& key) override;
    Status Size(const std::string& key, int64_t* size) override;
    Status AllKeys(std::vector<std::string>* keys) override;
    bool Healthy() override { return !offline_; }
    std::string Address() const override { return addr_; }
    void SetOffline(bool v) { offline_ = v; }
    DataNodeServer& server() { return server_; }

private:
    Status down() const;
    std::string addr_;
    bool offline_ = false;
    DataNodeServer server_;
};

}  // namespace host
}  // namespace rsmi
