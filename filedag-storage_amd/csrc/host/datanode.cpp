// datanode.cpp -- entry framing + CRC-16 shard store, with the mutcask engine's CRC-32 value
// framing (see datanode.hpp).
#include "datanode.hpp"

#include <array>
#include <cstring>

#include "crc_clmul.hpp"

namespace rsmi {
namespace host {

namespace {

// Slice-by-8 tables for the reflected polynomial 0xA001: t[0] is the byte-serial table of
// howeyc/crc16 makeTable(IBM); t[s][b] is byte b followed by s zero bytes, so eight input
// bytes fold in with eight independent lookups.  Identical results, ~6x the throughput.
struct IbmTables {
    uint16_t t[8][256];
    IbmTables() {
        for (int i = 0; i < 256; i++) {
            uint16_t c = uint16_t(i);
            for (int j = 0; j < 8; j++) c = (c & 1) ? uint16_t((c >> 1) ^ 0xA001) : uint16_t(c >> 1);
            t[0][i] = c;
        }
        for (int s = 1; s < 8; s++)
            for (int i = 0; i < 256; i++) t[s][i] = uint16_t(t[0][t[s - 1][i] & 0xFF] ^ (t[s - 1][i] >> 8));
    }
};

// Slice-by-8 tables for the reflected polynomial 0xEDB88320 (Go crc32 IEEE / zlib)
struct IeeeTables {
    uint32_t t[8][256];
    IeeeTables() {
        for (int i = 0; i < 256; i++) {
            uint32_t c = uint32_t(i);
            for (int j = 0; j < 8; j++) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
            t[0][i] = c;
        }
        for (int s = 1; s < 8; s++)
            for (int i = 0; i < 256; i++) t[s][i] = t[0][t[s - 1][i] & 0xFF] ^ (t[s - 1][i] >> 8);
    }
};

void put_le32(uint8_t* p, uint32_t v) {
    for (int i = 0; i < 4; i++) p[i] = uint8_t(v >> (8 * i));
}
uint32_t get_le32(const uint8_t* p) {
    return uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
}

Status not_found() { return Status::Error("Key not found"); }

// parse + crc check shared by Get and GetMeta (server.go:83-124), over an entry of n bytes
Status unpack(const uint8_t* e, size_t n, Bytes* meta, Bytes* data) {
    if (n < size_t(kHeaderSize)) return Status::Error("unexpected EOF");
    const uint32_t crc = get_le32(e);
    const uint32_t msz = get_le32(e + 4), dsz = get_le32(e + 8);
    if (crc != crc16_ibm(e + 4, n - 4)) return Status::Error("checking crc failed");
    if (size_t(kHeaderSize) + msz + dsz > n) return Status::Error("unexpected EOF");
    if (meta) meta->assign(e + kHeaderSize, e + kHeaderSize + msz);
    if (data) data->assign(e + kHeaderSize + msz, e + kHeaderSize + msz + dsz);
    return Status::Ok();
}

}  // namespace

uint16_t crc16_ibm(const uint8_t* p, size_t n, uint16_t crc) {
    bool done;  // 256 bytes and more: carry-less-multiply folding (crc_clmul.hpp), ~7x slice-by-8
    const uint32_t f = clmul_crc16(uint16_t(~crc), p, n, &done);
    if (done) return uint16_t(~f);
    static const IbmTables T;
    const auto& t = T.t;
    crc = uint16_t(~crc);
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        const uint8_t b0 = uint8_t(p[i] ^ crc), b1 = uint8_t(p[i + 1] ^ (crc >> 8));
        crc = uint16_t(t[7][b0] ^ t[6][b1] ^ t[5][p[i + 2]] ^ t[4][p[i + 3]] ^ t[3][p[i + 4]] ^ t[2][p[i + 5]] ^
                       t[1][p[i + 6]] ^ t[0][p[i + 7]]);
    }
    for (; i < n; i++) crc = uint16_t(t[0][uint8_t(crc ^ p[i])] ^ (crc >> 8));
    return uint16_t(~crc);
}

uint32_t crc32_ieee(const uint8_t* p, size_t n) {
    bool done;
    const uint32_t f = clmul_crc32(~0u, p, n, &done);
    if (done) return ~f;
    static const IeeeTables T;
    const auto& t = T.t;
    uint32_t crc = ~0u;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        const uint32_t lo = crc ^ get_le32(p + i);
        crc = t[7][lo & 0xFF] ^ t[6][(lo >> 8) & 0xFF] ^ t[5][(lo >> 16) & 0xFF] ^ t[4][lo >> 24] ^ t[3][p[i + 4]] ^
              t[2][p[i + 5]] ^ t[1][p[i + 6]] ^ t[0][p[i + 7]];
    }
    for (; i < n; i++) crc = t[0][(crc ^ p[i]) & 0xFF] ^ (crc >> 8);
    return ~crc;
}

Status DataNodeServer::store(const std::string& key, const Bytes& meta, ByteView data, const uint16_t* crc,
                             const uint32_t* value_crc) {
    if (key.empty()) return Status::Error("Key cannot be empty");  // badger, server_test.go:14-22
    const size_t pre = prefix();  // mutcask: | crc32 (4 LE) | entry |  (cask.go:73-79)
    const size_t len = pre + size_t(kHeaderSize) + meta.size() + data.size();
    // the entry is framed straight into the value the KV keeps (a recycled buffer when one is
    // large enough; every byte is written below), outside the lock, with no second copy
    // The smallest spare that fits, and none more than twice the entry's size: a few large
    // displaced values are not handed to small entries, where they would stay allocated for as
    // long as the key lives
    Value nv;
    {
        std::lock_guard<std::mutex> g(mu_);
        size_t best = spare_.size();
        for (size_t i = 0; i < spare_.size(); i++)
            if (spare_[i].cap >= len && spare_[i].cap <= 2 * len && (best == spare_.size() || spare_[i].cap < spare_[best].cap))
                best = i;
        if (best < spare_.size()) {
            nv = std::move(spare_[best]);
            spare_.erase(spare_.begin() + long(best));
        }
    }
    if (!nv.p) {
        nv.p.reset(new uint8_t[len]);
        nv.cap = len;
    }
    nv.len = len;
    uint8_t* e = nv.p.get() + pre;
    put_le32(e + 4, uint32_t(meta.size()));
    put_le32(e + 8, uint32_t(data.size()));
    if (!meta.empty()) std::memcpy(e + kHeaderSize, meta.data(), meta.size());
    if (!data.empty()) std::memcpy(e + kHeaderSize + meta.size(), data.data(), data.size());
    put_le32(e, crc ? *crc : crc16_ibm(e + 4, len - pre - 4));  // server.go:70-75
    if (pre) put_le32(nv.p.get(), value_crc ? *value_crc : crc32_ieee(e, len - pre));
    std::lock_guard<std::mutex> g(mu_);
    std::swap(kv_[key], nv);
    // a displaced value is kept for reuse while the pool has room; when it is full, the new one
    // replaces the largest spare if it is smaller (the pool drifts towards the sizes in use)
    if (nv.p) {
        if (spare_.size() < kSpareValues) {
            spare_.push_back(std::move(nv));
        } else {
            size_t big = 0;
            for (size_t i = 1; i < spare_.size(); i++)
                if (spare_[i].cap > spare_[big].cap) big = i;
            if (spare_[big].cap > nv.cap) spare_[big] = std::move(nv);
        }
    }
    return Status::Ok();
}

// the KV engine's read: mutcask re-checks its value checksum on every read (cask.go:250)
Status DataNodeServer::read_entry(const std::string& key, const Value** entry) {
    auto it = kv_.find(key);
    if (it == kv_.end()) return not_found();
    const Value& v = it->second;
    if (engine_ == KvEngine::Mutcask) {
        if (v.size() <= 4) return Status::Error("mutcask: invalid value format");
        if (get_le32(v.data()) != crc32_ieee(v.data() + 4, v.size() - 4))
            return Status::Error("mutcask: data may be rotted");
    }
    *entry = &v;
    return Status::Ok();
}

Status DataNodeServer::Put(const std::string& key, const Bytes& meta, ByteView data) {
    return store(key, meta, data, nullptr, nullptr);
}

Status DataNodeServer::PutWithChecksum(const std::string& key, const Bytes& meta, ByteView data, uint16_t crc) {
    return store(key, meta, data, &crc, nullptr);
}

Status DataNodeServer::PutWithChecksums(const std::string& key, const Bytes& meta, ByteView data, uint16_t crc,
                                        uint32_t value_crc) {
    return store(key, meta, data, &crc, &value_crc);
}

Status DataNodeServer::Get(const std::string& key, Bytes* meta, Bytes* data) {
    std::lock_guard<std::mutex> g(mu_);
    const Value* v = nullptr;
    Status s = read_entry(key, &v);
    if (!s.ok()) return s;
    return unpack(v->data() + prefix(), v->size() - prefix(), meta, data);
}

Status DataNodeServer::GetUnverified(const std::string& key, Bytes* meta, Bytes* data, DataNodeClient::Stored* st) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = kv_.find(key);
    if (it == kv_.end()) return not_found();
    const Value& v = it->second;
    const size_t pre = prefix();
    if (v.size() < pre + size_t(kHeaderSize)) return Status::Error("unexpected EOF");
    const uint8_t* e = v.data() + pre;
    const size_t n = v.size() - pre;
    const uint32_t msz = get_le32(e + 4), dsz = get_le32(e + 8);
    if (size_t(kHeaderSize) + msz + dsz > n) return Status::Error("unexpected EOF");
    *st = DataNodeClient::Stored{};
    st->crc = uint16_t(get_le32(e));
    st->has_value_crc = pre != 0;
    st->value_crc = pre ? get_le32(v.data()) : 0;
    st->verified = false;
    if (meta) meta->assign(e + kHeaderSize, e + kHeaderSize + msz);
    if (data) data->assign(e + kHeaderSize + msz, e + kHeaderSize + msz + dsz);
    return Status::Ok();
}

Status DataNodeServer::GetMeta(const std::string& key, Bytes* meta) {
    std::lock_guard<std::mutex> g(mu_);
    const Value* v = nullptr;
    Status s = read_entry(key, &v);
    if (!s.ok()) return s;
    return unpack(v->data() + prefix(), v->size() - prefix(), meta, nullptr);
}

Status DataNodeServer::Delete(const std::string& key) {
    std::lock_guard<std::mutex> g(mu_);
    kv_.erase(key);
    return Status::Ok();
}

Status DataNodeServer::Size(const std::string& key, int64_t* size) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = kv_.find(key);
    if (it == kv_.end()) return not_found();
    *size = int64_t(it->second.size() - prefix());  // HeaderSize + meta + data (server_test.go:147-152;
                                                      // mutcask Size = VSize - 4, cask.go:235)
    return Status::Ok();
}

Status DataNodeServer::AllKeys(std::vector<std::string>* keys) {
    std::lock_guard<std::mutex> g(mu_);
    keys->clear();
    for (auto& kv : kv_) keys->push_back(kv.first);
    return Status::Ok();
}

bool DataNodeServer::RawEntry(const std::string& key, Bytes* entry) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = kv_.find(key);
    if (it == kv_.end()) return false;
    entry->assign(it->second.data() + prefix(), it->second.data() + it->second.size());
    return true;
}

bool DataNodeServer::RawValue(const std::string& key, Bytes* value) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = kv_.find(key);
    if (it == kv_.end()) return false;
    value->assign(it->second.data(), it->second.data() + it->second.size());
    return true;
}

void DataNodeServer::CorruptByte(const std::string& key, size_t offset) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = kv_.find(key);
    if (it != kv_.end() && prefix() + offset < it->second.size()) it->second.p[prefix() + offset] ^= 0x5A;
}

void DataNodeServer::Wipe() {
    std::lock_guard<std::mutex> g(mu_);
    kv_.clear();
    spare_.clear();
}

Status InProcDataNode::down() const { return Status::Error("rpc error: code = Unavailable desc = " + addr_); }

Status InProcDataNode::Put(const std::string& key, const Bytes& meta, ByteView data) {
    return offline_ ? down() : server_.Put(key, meta, data);
}
Status InProcDataNode::PutWithChecksum(const std::string& key, const Bytes& meta, ByteView data, uint16_t crc) {
    return offline_ ? down() : server_.PutWithChecksum(key, meta, data, crc);
}
Status InProcDataNode::PutWithChecksums(const std::string& key, const Bytes& meta, ByteView data, uint16_t crc,
                                        uint32_t value_crc) {
    return offline_ ? down() : server_.PutWithChecksums(key, meta, data, crc, value_crc);
}
Status InProcDataNode::Get(const std::string& key, Bytes* meta, Bytes* data) {
    return offline_ ? down() : server_.Get(key, meta, data);
}
Status InProcDataNode::GetForVerify(const std::string& key, Bytes* meta, Bytes* data, Stored* st) {
    return offline_ ? down() : server_.GetUnverified(key, meta, data, st);
}
Status InProcDataNode::GetMeta(const std::string& key, Bytes* meta) {
    return offline_ ? down() : server_.GetMeta(key, meta);
}
Status InProcDataNode::Delete(const std::string& key) { return offline_ ? down() : server_.Delete(key); }
Status InProcDataNode::Size(const std::string& key, int64_t* size) {
    return offline_ ? down() : server_.Size(key, size);
}
Status InProcDataNode::AllKeys(std::vector<std::string>* keys) {
    return offline_ ? down() : server_.AllKeys(keys);
}

}  // namespace host
}  // namespace rsmi
