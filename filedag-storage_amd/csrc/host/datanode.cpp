// datanode.cpp -- entry framing + CRC-16 shard store (see datanode.hpp).
#include "datanode.hpp"

#include <array>
#include <cstring>

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

void put_le32(uint8_t* p, uint32_t v) {
    for (int i = 0; i < 4; i++) p[i] = uint8_t(v >> (8 * i));
}
uint32_t get_le32(const uint8_t* p) {
    return uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
}

Status not_found() { return Status::Error("Key not found"); }

// parse + crc check shared by Get and GetMeta (server.go:83-124)
Status unpack(const Bytes& e, Bytes* meta, Bytes* data) {
    if (e.size() < size_t(kHeaderSize)) return Status::Error("unexpected EOF");
    const uint32_t crc = get_le32(e.data());
    const uint32_t msz = get_le32(e.data() + 4), dsz = get_le32(e.data() + 8);
    if (crc != crc16_ibm(e.data() + 4, e.size() - 4)) return Status::Error("checking crc failed");
    if (size_t(kHeaderSize) + msz + dsz > e.size()) return Status::Error("unexpected EOF");
    if (meta) meta->assign(e.begin() + kHeaderSize, e.begin() + kHeaderSize + msz);
    if (data) data->assign(e.begin() + kHeaderSize + msz, e.begin() + kHeaderSize + msz + dsz);
    return Status::Ok();
}

}  // namespace

uint16_t crc16_ibm(const uint8_t* p, size_t n, uint16_t crc) {
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

Status DataNodeServer::store(const std::string& key, const Bytes& meta, const Bytes& data, const uint16_t* crc) {
    if (key.empty()) return Status::Error("Key cannot be empty");  // badger, server_test.go:14-22
    Bytes e(size_t(kHeaderSize) + meta.size() + data.size());
    put_le32(e.data() + 4, uint32_t(meta.size()));
    put_le32(e.data() + 8, uint32_t(data.size()));
    if (!meta.empty()) std::memcpy(e.data() + kHeaderSize, meta.data(), meta.size());
    if (!data.empty()) std::memcpy(e.data() + kHeaderSize + meta.size(), data.data(), data.size());
    put_le32(e.data(), crc ? *crc : crc16_ibm(e.data() + 4, e.size() - 4));  // server.go:70-75
    std::lock_guard<std::mutex> g(mu_);
    kv_[key] = std::move(e);
    return Status::Ok();
}

Status DataNodeServer::Put(const std::string& key, const Bytes& meta, const Bytes& data) {
    return store(key, meta, data, nullptr);
}

Status DataNodeServer::PutWithChecksum(const std::string& key, const Bytes& meta, const Bytes& data, uint16_t crc) {
    return store(key, meta, data, &crc);
}

Status DataNodeServer::Get(const std::string& key, Bytes* meta, Bytes* data) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = kv_.find(key);
    if (it == kv_.end()) return not_found();
    return unpack(it->second, meta, data);
}

Status DataNodeServer::GetMeta(const std::string& key, Bytes* meta) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = kv_.find(key);
    if (it == kv_.end()) return not_found();
    return unpack(it->second, meta, nullptr);
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
    *size = int64_t(it->second.size());  // HeaderSize + meta + data (server_test.go:147-152)
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
    *entry = it->second;
    return true;
}

void DataNodeServer::CorruptByte(const std::string& key, size_t offset) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = kv_.find(key);
    if (it != kv_.end() && offset < it->second.size()) it->second[offset] ^= 0x5A;
}

void DataNodeServer::Wipe() {
    std::lock_guard<std::mutex> g(mu_);
    kv_.clear();
}

Status InProcDataNode::down() const { return Status::Error("rpc error: code = Unavailable desc = " + addr_); }

Status InProcDataNode::Put(const std::string& key, const Bytes& meta, const Bytes& data) {
    return offline_ ? down() : server_.Put(key, meta, data);
}
Status InProcDataNode::PutWithChecksum(const std::string& key, const Bytes& meta, const Bytes& data, uint16_t crc) {
    return offline_ ? down() : server_.PutWithChecksum(key, meta, data, crc);
}
Status InProcDataNode::Get(const std::string& key, Bytes* meta, Bytes* data) {
    return offline_ ? down() : server_.Get(key, meta, data);
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
