// rsmi_group.cpp -- one process driving several GPUs (include/rsmi.h "device groups").
//
// The reference's Dag Pool hosts every DagNode of the cluster in one process
// (dag/pool/poolservice/cluster.go:28-41) and routes each key to a node by its hash slot
// (hash_slot.go:20-22: crc16(key) & 0x3FFF).  Blocks are coded independently
// (dag/node/dagnode/node.go:358-408), so a group of per-device contexts spreads a host batch over
// the node's GPUs as contiguous block ranges, each range on its own context (own HIP streams
// and page-locked staging); no data crosses devices and no collective runs.  The caller's
// buffers are written in place, so results need no reordering.
//
// Host memory placement.  An MI355X node has two sockets, and each GPU hangs off one of them.
// Every member runs its ranges on a persistent worker thread bound to its GPU's NUMA node (the
// node's CPUs, and a preferred-node memory policy), so the page-locked staging its context
// allocates (hipHostMallocNumaUser, rsmi_core.cpp pinned_alloc) lands in that socket's memory,
// and the CPU copies of pageable callers run on that socket.  rsmi_group_host_alloc gives a
// caller one buffer whose member ranges sit on the members' nodes, so on the zero-copy path
// (kernels read and write page-locked caller memory in place over PCIe) each member's DMA touches
// only its own socket's memory.  The device -> node map comes from the runtime
// (hipDeviceAttributeHostNumaId) or sysfs (bus/pci/devices/<bus id>/numa_node).
#include "rsmi_impl.hpp"

#include <linux/mempolicy.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cctype>
#include <fstream>
#include <functional>
#include <sstream>
#include <thread>

using namespace rsmi;
using namespace rsmi::impl;

namespace {

constexpr int kClusterSlots = 16384;  // dag/slotsmgr/slots_mgr.go:8

// A member's persistent worker: runs one job at a time, bound to a NUMA node.
class Worker {
public:
    explicit Worker(int node) : node_(node), th_([this] { loop(); }) {}
    ~Worker() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        th_.join();
    }
    void post(std::function<void()> job) {
        {
            std::lock_guard<std::mutex> g(mu_);
            job_ = std::move(job);
            busy_ = true;
        }
        cv_.notify_all();
    }
    void wait() {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !busy_; });
    }
    int bound() const { return bound_.load(); }

private:
    void loop() {
        bound_ = rsmi_bind_thread_to_numa_node(node_) == RSMI_OK ? 1 : 0;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || busy_; });
            if (busy_) {
                std::function<void()> job = std::move(job_);
                lk.unlock();
                job();  // run_parts' jobs catch everything and return status codes
                lk.lock();
                busy_ = false;
                cv_.notify_all();
                continue;
            }
            if (stop_) return;
        }
    }
    const int node_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::function<void()> job_;
    bool busy_ = false, stop_ = false;
    std::atomic<int> bound_{0};
    std::thread th_;  // last: started once the members above exist
};

std::string read_file(const std::string& path) {
    std::ifstream f(path);
    if (!f) return "";
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

}  // namespace

struct rsmi_group {
    int k = 0, m = 0;
    std::vector<rsmi_ctx*> ctx;  // one per entry of the device list (a device may repeat)
    std::vector<int> node;       // each member's NUMA node (-1: unknown, the worker is unbound)
    std::vector<std::unique_ptr<Worker>> workers;
    std::mutex call_mu;  // one batch call at a time: each member has one worker
    std::mutex alloc_mu;
    std::map<void*, size_t> allocs;  // rsmi_group_host_alloc ranges
};

namespace {

// Run f(i, start, count) for every non-empty part on member i's worker thread; the first failing
// part's status in part order, so results do not depend on timing.  nblocks == 0 runs part 0
// with an empty range on the caller's thread, so argument errors surface exactly as the
// single-context calls report them.
template <class F>
int run_parts(rsmi_group* s, size_t nblocks, F f) {
    if (nblocks == 0) return f(size_t(0), size_t(0), size_t(0));
    const size_t parts = s->ctx.size();
    std::vector<int> rc(parts, RSMI_OK);
    std::lock_guard<std::mutex> g(s->call_mu);
    // Every allocation happens before the first post: the jobs capture rc and f by reference, so
    // once one is posted this frame must not unwind (a std::bad_alloc from a later std::function
    // or push_back would leave a worker writing through dangling references).
    std::vector<std::pair<size_t, std::function<void()>>> jobs;
    jobs.reserve(parts);
    for (size_t i = 0; i < parts; i++) {
        size_t st, cnt;
        rsmi_partition(nblocks, int(parts), int(i), &st, &cnt);
        if (!cnt) continue;
        jobs.emplace_back(i, [&rc, &f, i, st, cnt] {
            // an exception must not leave the worker thread (std::terminate): the member's host
            // code allocates (std::bad_alloc), so it becomes the part's status
            try {
                rc[i] = f(i, st, cnt);
            } catch (...) {
                rc[i] = rsmi::impl::exception_status();
            }
        });
    }
    for (auto& j : jobs) s->workers[j.first]->post(std::move(j.second));  // moves only: no allocation
    for (auto& j : jobs) s->workers[j.first]->wait();
    for (int r : rc)
        if (r != RSMI_OK) return r;
    return RSMI_OK;
}

}  // namespace

extern "C" {

// ---------------------------------------------------------------- NUMA helpers (host only)

int rsmi_sysfs_numa_node(const char* sysfs_root, const char* pci_bus_id) try {
    if (!sysfs_root || !pci_bus_id) return -1;
    std::string id(pci_bus_id);
    for (auto& ch : id) ch = char(std::tolower(static_cast<unsigned char>(ch)));
    const std::string txt = read_file(std::string(sysfs_root) + "/bus/pci/devices/" + id + "/numa_node");
    if (txt.empty()) return -1;
    const int v = std::atoi(txt.c_str());
    return v >= 0 ? v : -1;
} catch (...) {
    return -1;  // host allocation failed
}

int rsmi_sysfs_node_cpus(const char* sysfs_root, int node, int* cpus, int max_cpus) try {
    if (!sysfs_root || node < 0 || (!cpus && max_cpus > 0)) return -1;
    const std::string txt =
        read_file(std::string(sysfs_root) + "/devices/system/node/node" + std::to_string(node) + "/cpulist");
    if (txt.empty()) return -1;
    int n = 0;
    std::stringstream ss(txt);
    std::string part;
    while (std::getline(ss, part, ',')) {  // "0-31,64-95"
        while (!part.empty() && std::isspace(static_cast<unsigned char>(part.back()))) part.pop_back();
        if (part.empty()) continue;
        const size_t dash = part.find('-');
        const int a = std::atoi(part.c_str());
        const int b = dash == std::string::npos ? a : std::atoi(part.c_str() + dash + 1);
        if (a < 0 || b < a) return -1;
        for (int c = a; c <= b; c++) {
            if (n < max_cpus) cpus[n] = c;
            n++;
        }
    }
    return n;
} catch (...) {
    return -1;  // host allocation failed
}

int rsmi_device_numa_node(int device) try {
    int v = -1;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeHostNumaId, device) == hipSuccess && v >= 0) return v;
    (void)hipGetLastError();
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    return rsmi_sysfs_numa_node("/sys", bus);
} catch (...) {
    return -1;  // host allocation failed
}

int rsmi_bind_thread_to_numa_node(int node) try {
    if (node < 0) return RSMI_ERR_INVALID_ARG;
    std::vector<int> cpus(4096);
    const int n = rsmi_sysfs_node_cpus("/sys", node, cpus.data(), int(cpus.size()));
    if (n <= 0) return RSMI_ERR_INVALID_ARG;
    // CPUs: only those the process may use (a container or job may own a subset of the node)
    cpu_set_t allowed, set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) CPU_ZERO(&allowed);
    int nset = 0;
    for (int i = 0; i < std::min(n, int(cpus.size())); i++)
        if (cpus[size_t(i)] < CPU_SETSIZE && CPU_ISSET(cpus[size_t(i)], &allowed)) {
            CPU_SET(cpus[size_t(i)], &set);
            nset++;
        }
    if (nset && sched_setaffinity(0, sizeof set, &set) != 0) return RSMI_ERR_INVALID_ARG;
    // memory: prefer the node (falls back to others when it is full, never fails an allocation)
    unsigned long mask[16] = {0};
    if (node >= int(sizeof mask * 8)) return RSMI_ERR_INVALID_ARG;
    mask[node / (8 * sizeof(unsigned long))] |= 1UL << (node % (8 * sizeof(unsigned long)));
    if (syscall(SYS_set_mempolicy, MPOL_PREFERRED, mask, sizeof mask * 8) != 0) return RSMI_ERR_INVALID_ARG;
    return RSMI_OK;
} catch (...) {
    return rsmi::impl::exception_status();
}

// ---------------------------------------------------------------- groups

int rsmi_group_open(int k, int m, const int* devices, int ndev, rsmi_group** out) try {
    if (!out) return RSMI_ERR_INVALID_ARG;
    *out = nullptr;
    if (k <= 0 || m <= 0) return RSMI_ERR_INV_SHARD_NUM;
    if (k + m > 256) return RSMI_ERR_MAX_SHARD_NUM;
    if (!devices || ndev <= 0 || ndev > 1024) return RSMI_ERR_INVALID_ARG;
    auto* s = new rsmi_group();
    s->k = k;
    s->m = m;
    const int have = rsmi_device_count();
    for (int i = 0; i < ndev; i++) {
        rsmi_ctx* c = nullptr;
        const int rc = rsmi_open(k, m, devices[i], &c);
        if (rc != RSMI_OK) {
            rsmi_group_close(s);
            return rc;
        }
        s->ctx.push_back(c);
        // no GPU (or an out-of-range device): the member stays unbound, its calls report the error
        s->node.push_back(devices[i] >= 0 && devices[i] < have ? rsmi_device_numa_node(devices[i]) : -1);
        try {
            s->workers.emplace_back(new Worker(s->node.back()));
        } catch (...) {  // std::system_error (no thread) or std::bad_alloc
            rsmi_group_close(s);
            return RSMI_ERR_DEVICE;
        }
    }
    *out = s;
    return RSMI_OK;
} catch (...) {
    return rsmi::impl::exception_status();
}

void rsmi_group_close(rsmi_group* s) {
    if (!s) return;
    s->workers.clear();  // joins them
    for (rsmi_ctx* c : s->ctx) rsmi_close(c);
    {
        std::lock_guard<std::mutex> g(s->alloc_mu);
        for (auto& a : s->allocs) {
            (void)hipHostUnregister(a.first);
            munmap(a.first, a.second);
        }
    }
    delete s;
}

int rsmi_group_size(const rsmi_group* s) { return s ? int(s->ctx.size()) : 0; }

rsmi_ctx* rsmi_group_context(rsmi_group* s, int i) {
    if (!s || i < 0 || size_t(i) >= s->ctx.size()) return nullptr;
    return s->ctx[size_t(i)];
}

int rsmi_group_member_numa_node(const rsmi_group* s, int i) {
    if (!s || i < 0 || size_t(i) >= s->node.size()) return -1;
    return s->node[size_t(i)];
}

int rsmi_group_member_of_key(const rsmi_group* s, const uint8_t* key, size_t len) {
    if (!s || s->ctx.empty()) return -1;
    const int slot = rsmi_key_slot(key, len);
    if (slot < 0) return -1;
    // contiguous slot ranges per member, like DagNodes owning SlotPairs (slotsmgr)
    return int(size_t(slot) * s->ctx.size() / kClusterSlots);
}

void* rsmi_group_host_alloc(rsmi_group* s, size_t block_bytes, size_t nblocks) try {
    if (!s || !block_bytes || !nblocks) return nullptr;
    const size_t page = size_t(sysconf(_SC_PAGESIZE));
    const size_t bytes = (block_bytes * nblocks + page - 1) / page * page;
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) return nullptr;
    // member i's block range on member i's node (pages straddling two ranges go to the first);
    // each worker touches its own pages first, so they are placed before they are pinned
    const size_t parts = s->ctx.size();
    {
        std::lock_guard<std::mutex> g(s->call_mu);
        for (size_t i = 0; i < parts; i++) {
            size_t st, cnt;
            rsmi_partition(nblocks, int(parts), int(i), &st, &cnt);
            const size_t a = (st * block_bytes + page - 1) / page * page;
            const size_t b = std::min(bytes, ((st + cnt) * block_bytes + page - 1) / page * page);
            if (!cnt || b <= a) continue;
            uint8_t* lo = static_cast<uint8_t*>(p) + a;
            const int node = s->node[i];
            if (node >= 0 && node < 1024) {
                unsigned long mask[16] = {0};
                mask[node / (8 * sizeof(unsigned long))] |= 1UL << (node % (8 * sizeof(unsigned long)));
                (void)syscall(SYS_mbind, lo, b - a, MPOL_PREFERRED, mask, sizeof mask * 8, 0);
            }
            s->workers[i]->post([lo, a, b] { std::memset(lo, 0, b - a); });
        }
        for (size_t i = 0; i < parts; i++) s->workers[i]->wait();
    }
    if (hipHostRegister(p, bytes, hipHostRegisterPortable | hipHostRegisterMapped) != hipSuccess) {
        (void)hipGetLastError();
        munmap(p, bytes);
        return nullptr;
    }
    std::lock_guard<std::mutex> g(s->alloc_mu);
    s->allocs[p] = bytes;
    return p;
} catch (...) {
    return nullptr;  // host allocation failed (a pinned range may stay mapped: never freed twice)
}

void rsmi_group_host_free(rsmi_group* s, void* p) {
    if (!s || !p) return;
    size_t bytes = 0;
    {
        std::lock_guard<std::mutex> g(s->alloc_mu);
        auto it = s->allocs.find(p);
        if (it == s->allocs.end()) return;
        bytes = it->second;
        s->allocs.erase(it);
    }
    (void)hipHostUnregister(p);
    munmap(p, bytes);
}

int rsmi_group_encode_batch_host(rsmi_group* s, const uint8_t* data, size_t data_block_stride, uint8_t* parity,
                               size_t parity_block_stride, size_t S, size_t nblocks) try {
    if (!s || !data || !parity) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    return run_parts(s, nblocks, [&](size_t i, size_t st, size_t cnt) {
        return rsmi_encode_batch_host(s->ctx[i], data + st * data_block_stride, data_block_stride,
                                      parity + st * parity_block_stride, parity_block_stride, S, cnt);
    });
} catch (...) {
    return rsmi::impl::exception_status();
}

int rsmi_group_encode_batch_host_crcs(rsmi_group* s, const uint8_t* data, size_t data_block_stride, uint8_t* parity,
                                    size_t parity_block_stride, size_t S, size_t nblocks, uint32_t* raw16_out,
                                    uint32_t* raw32_out) try {
    if (!s || !data || !parity) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    const size_t n = size_t(s->k + s->m);
    return run_parts(s, nblocks, [&](size_t i, size_t st, size_t cnt) {
        return rsmi_encode_batch_host_crcs(s->ctx[i], data + st * data_block_stride, data_block_stride,
                                           parity + st * parity_block_stride, parity_block_stride, S, cnt,
                                           raw16_out ? raw16_out + st * n : nullptr,
                                           raw32_out ? raw32_out + st * n : nullptr);
    });
} catch (...) {
    return rsmi::impl::exception_status();
}

int rsmi_group_reconstruct_batch_host(rsmi_group* s, uint8_t* shards, size_t block_stride, size_t S, size_t nblocks,
                                    const uint8_t* present, int data_only) try {
    if (!s || !shards || !present) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    return run_parts(s, nblocks, [&](size_t i, size_t st, size_t cnt) {
        return rsmi_reconstruct_batch_host(s->ctx[i], shards + st * block_stride, block_stride, S, cnt, present,
                                           data_only);
    });
} catch (...) {
    return rsmi::impl::exception_status();
}

int rsmi_group_reconstruct_rows_batch_host(rsmi_group* s, uint8_t* shards, size_t block_stride, size_t S,
                                         size_t nblocks, const uint8_t* present, const uint8_t* required) try {
    if (!s || !shards || !present || !required) return RSMI_ERR_INVALID_ARG;
    if (S == 0) return RSMI_ERR_SHARD_NO_DATA;
    return run_parts(s, nblocks, [&](size_t i, size_t st, size_t cnt) {
        return rsmi_reconstruct_rows_batch_host(s->ctx[i], shards + st * block_stride, block_stride, S, cnt, present,
                                                required);
    });
} catch (...) {
    return rsmi::impl::exception_status();
}

}  // extern "C"
