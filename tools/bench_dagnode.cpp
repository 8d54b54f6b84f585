// bench_dagnode.cpp -- end-to-end rates of the Dag Node mirror over in-process datanodes
// (host memory in, framed+CRC'd shard entries out): per-block vs GPU-batched Put (entry
// checksums from the GPU, and from the datanode's own CRC pass), Get with
// a lost data shard, RepairDataNode, and PutMany over mutcask-backed datanodes (CRC-32 value
// checksums from the GPU or the datanodes).  Diagnostic; numbers recorded in DESIGN.md.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <malloc.h>
#include <random>
#include <string>
#include <thread>

#include "../filedag-storage_amd/csrc/host/dagnode.hpp"
#ifdef FAKE_RSMI_FAST
#include "../oracle/rs_oracle.h"  // rs_cpu_isa: the CPU codec build (tools/Makefile bench_dagnode_cpu)
#endif

using namespace rsmi::host;
using clk = std::chrono::steady_clock;

static double secs(clk::time_point a) { return std::chrono::duration<double>(clk::now() - a).count(); }

int main(int argc, char** argv) {
    // The in-process data nodes copy every shard into a fresh heap block. glibc serves blocks
    // above its mmap threshold with mmap/munmap, and raises that threshold only after it frees
    // a large mapped block, so whether a Get leg's shard copies each fault in fresh pages under
    // the process-wide mmap lock depended on what the codec build happened to free before it
    // (the GPU build's page-locked scratch is not malloc'd; the CPU build's was, until the
    // scratch was pooled). Both builds fix the threshold so they start from the same heap.
    if (!std::getenv("BENCH_DAGNODE_DYNAMIC_MMAP")) {
        mallopt(M_MMAP_THRESHOLD, 32 << 20);
        mallopt(M_TRIM_THRESHOLD, 256 << 20);
    }
    const int k = argc > 1 ? atoi(argv[1]) : 10, m = argc > 2 ? atoi(argv[2]) : 4;
    const size_t B = argc > 3 ? size_t(atol(argv[3])) : 262144;
    const int N = argc > 4 ? atoi(argv[4]) : 512;
    DagNodeConfig cfg;
    cfg.data_blocks = k;
    cfg.parity_blocks = m;
    std::vector<std::shared_ptr<InProcDataNode>> dn;
    std::vector<std::shared_ptr<DataNodeClient>> cl;
    for (int i = 0; i < k + m; i++) {
        cfg.nodes.push_back("n" + std::to_string(i));
        dn.push_back(std::make_shared<InProcDataNode>(cfg.nodes.back()));
        cl.push_back(dn.back());
    }
    // BENCH_DAGNODE_DEVICES="0,0": the Dag Node on a device list (member routing, DagNode::New)
    std::vector<int> devices;
    if (const char* e = std::getenv("BENCH_DAGNODE_DEVICES"))
        for (const char* p = e; *p;) {
            devices.push_back(std::atoi(p));
            while (*p && *p != ',') p++;
            if (*p == ',') p++;
        }
    if (devices.empty()) devices.push_back(0);
    std::unique_ptr<DagNode> d;
    if (!DagNode::New(cfg, cl, &d, devices).ok()) return 2;
    d->HealthCheckAll();
    std::mt19937_64 r(1);
    std::vector<std::string> keys;
    std::vector<Bytes> blocks;
    for (int i = 0; i < N; i++) {
        keys.push_back("k" + std::to_string(i));
        Bytes b(B);
        for (auto& x : b) x = uint8_t(r());
        blocks.push_back(std::move(b));
    }
    const double gib = double(N) * B / (1 << 30);
    d->Put("warm", blocks[0]);
    // host CRC (datanode computes server.go:70) first, then GPU entry checksums (default)
    d->SetGpuChecksums(false);
    auto t0 = clk::now();
    for (int i = 0; i < N; i++) d->Put(keys[i], blocks[i]);
    const double put1h = secs(t0);
    t0 = clk::now();
    d->PutMany(keys, blocks);
    const double putbh = secs(t0);
    d->SetGpuChecksums(true);
    d->Put("warm", blocks[0]);
    // per-phase host time of the legs the GPU / CPU codec comparison is about (DagNode phases:
    // fetch, stage, codec, put; summed over threads)
    std::string phases;
    auto phase_json = [&](const char* leg, double wall) {
        const auto p = d->PhaseSeconds();
        char buf[256];
        std::snprintf(buf, sizeof buf, "%s\"%s\": {\"wall\": %.4f, \"fetch\": %.4f, \"stage\": %.4f, \"codec\": %.4f, \"put\": %.4f}",
                      phases.empty() ? "" : ", ", leg, wall, p[0], p[1], p[2], p[3]);
        phases += buf;
        d->ResetPhases();
    };
    // per-block Put, the lone-caller path on and off, alternated twice after an untimed pass
    // (the first pass after a PutMany runs slower for either setting); best of each
    for (int i = 0; i < N; i++) d->Put(keys[i], blocks[i]);
    double put1 = 1e30, put1n = 1e30;
    for (int rep = 0; rep < 2; rep++)
        for (bool lone : {true, false}) {
            d->SetLoneCallerPaths(lone);
            d->SetPhaseTiming(lone && rep == 0);
            d->ResetPhases();
            t0 = clk::now();
            for (int i = 0; i < N; i++) d->Put(keys[i], blocks[i]);
            const double t = secs(t0);
            if (lone && rep == 0) phase_json("put", t);
            (lone ? put1 : put1n) = std::min(lone ? put1 : put1n, t);
        }
    d->SetLoneCallerPaths(true);
    d->SetPhaseTiming(true);
    d->ResetPhases();
    t0 = clk::now();
    d->PutMany(keys, blocks);
    const double putb = secs(t0);
    phase_json("putmany", putb);
    d->SetPhaseTiming(false);
    // Put from 16 threads at once: the per-block encodes coalesce into GPU batches
    const int T = 16;
    long c0 = 0, b0 = 0;
    int rc;
    rsmi_ctx* ctx = shared_context(k, m, d->MemberDevice(0), &rc, d->MemberReplica(0));
    // the coalescing counters summed over the node's members
    auto node_stat = [&](const char* key) {
        long v = 0;
        for (int i = 0; i < d->Members(); i++) v += lane_stat(k, m, d->MemberDevice(i), key, d->MemberReplica(i));
        return v;
    };
    // an untimed pass first: the threads' page-locked scratch comes from the pool their
    // predecessors leave (erasure.hpp block_scratch), as in a server whose workers come and go
    auto put_threads = [&] {
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] {
                for (int i = t; i < N; i += T) d->Put(keys[i], blocks[i]);
            });
        for (auto& x : th) x.join();
    };
    if (!std::getenv("BENCH_DAGNODE_NO_WARM")) put_threads();  // diagnostic switch: no untimed pass
    long w0 = 0, wn0 = 0;
    if (ctx) {
        c0 = node_stat("coalesced_calls");
        b0 = node_stat("coalesced_batches");
        w0 = node_stat("coalesced_wakes");
        wn0 = node_stat("coalesced_wake_ns");
    }
    d->SetPhaseTiming(true);
    d->ResetPhases();
    t0 = clk::now();
    put_threads();
    const double putT = secs(t0);
    if (ctx) {  // the group commit's wake-ups during the timed pass (diagnostic)
        const long w = node_stat("coalesced_wakes") - w0, wn = node_stat("coalesced_wake_ns") - wn0;
        std::printf("WAKE put_threads: %ld wake-ups for %d calls, %.1f us from wake-up call to running (mean)\n", w, N,
                    w ? double(wn) / double(w) / 1e3 : 0.0);
    }
    phase_json("put_threads", putT);
    d->SetPhaseTiming(false);
    const long calls = ctx ? node_stat("coalesced_calls") - c0 : 0;
    const long batches = ctx ? node_stat("coalesced_batches") - b0 : 0;
    // CRC + framing alone (the datanode's byte-serial CPU loop), for context
    t0 = clk::now();
    volatile uint16_t sink = 0;
    for (int i = 0; i < N; i++) sink ^= crc16_ibm(blocks[i].data(), blocks[i].size());
    const double crc = secs(t0);
    dn[0]->SetOffline(true);  // a data shard is lost on every Get
    Bytes got;
    // per-block degraded Get, the lone-caller path on and off, alternated twice; best of each
    double get1 = 1e30, get1n = 1e30;
    for (int rep = 0; rep < 2; rep++)
        for (bool lone : {true, false}) {
            d->SetLoneCallerPaths(lone);
            d->SetPhaseTiming(lone && rep == 0);
            d->ResetPhases();
            t0 = clk::now();
            for (int i = 0; i < N; i++) d->Get(keys[i], &got);
            const double t = secs(t0);
            if (lone && rep == 0) phase_json("get", t);
            (lone ? get1 : get1n) = std::min(lone ? get1 : get1n, t);
        }
    d->SetPhaseTiming(false);
    d->SetLoneCallerPaths(true);
    std::vector<Bytes> gm;
    std::vector<Status> st;
    double getb = 0;
    size_t best_batch = 0;
    for (size_t gb : {size_t(16), size_t(64), size_t(256)}) {  // batch size: GPU batching vs cache locality
        t0 = clk::now();
        d->GetMany(keys, &gm, &st, gb);
        const double tb = secs(t0);
        std::printf("GetMany batch %3zu  %8.2f GiB/s\n", gb, gib / tb);
        if (getb == 0 || tb < getb) {
            getb = tb;
            best_batch = gb;
        }
    }
    // degraded Get from 16 threads: the reconstructs coalesce (one erasure pattern)
    const long gc0 = ctx ? node_stat("coalesced_calls") : 0, gb0 = ctx ? node_stat("coalesced_batches") : 0;
    d->SetPhaseTiming(true);
    d->ResetPhases();
    t0 = clk::now();
    {
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] {
                Bytes b;
                for (int i = t; i < N; i += T) d->Get(keys[i], &b);
            });
        for (auto& x : th) x.join();
    }
    const double getT = secs(t0);
    phase_json("get_threads", getT);
    d->SetPhaseTiming(false);
    const long gcalls = ctx ? node_stat("coalesced_calls") - gc0 : 0;
    const long gbatches = ctx ? node_stat("coalesced_batches") - gb0 : 0;
    // the same degraded reads with the checksums checked on the GPU instead of by each datanode
    d->SetGpuVerifiedReads(true);
    t0 = clk::now();
    for (int i = 0; i < N; i++) d->Get(keys[i], &got);
    const double get1v = secs(t0);
    // GetMany with and without GPU-verified reads, alternated three times (best of each)
    double getbv = 1e30;
    for (int rep = 0; rep < 3; rep++) {
        d->SetGpuVerifiedReads(false);
        d->SetPhaseTiming(rep == 0);
        d->ResetPhases();
        t0 = clk::now();
        d->GetMany(keys, &gm, &st, best_batch);
        if (rep == 0) phase_json("getmany", secs(t0));
        d->SetPhaseTiming(false);
        getb = std::min(getb, secs(t0));
        d->SetGpuVerifiedReads(true);
        t0 = clk::now();
        d->GetMany(keys, &gm, &st, best_batch);
        getbv = std::min(getbv, secs(t0));
        for (int i = 0; i < N; i++)
            if (!st[i].ok() || gm[i] != blocks[i]) std::printf("verified GetMany: key %d wrong\n", i);
    }
    d->SetGpuVerifiedReads(false);
    dn[0]->SetOffline(false);
    d->RunRepairTasks();
    const int rj = std::min(3, k - 1);  // the repaired node: data shard 3 (RS(2,1): shard 1)
    dn[size_t(rj)]->server().Wipe();
    // per-key RepairDataNode onto the wiped node, the lone-caller path on and off, alternated
    // twice; best of each
    double rep1 = 1e30, rep1n = 1e30;
    for (int rep = 0; rep < 2; rep++)
        for (bool lone : {true, false}) {
            dn[size_t(rj)]->server().Wipe();
            d->SetLoneCallerPaths(lone);
            t0 = clk::now();
            d->RepairDataNode(0, rj);
            (lone ? rep1 : rep1n) = std::min(lone ? rep1 : rep1n, secs(t0));
        }
    d->SetLoneCallerPaths(true);
    dn[size_t(rj)]->server().Wipe();
    size_t rep = 0;
    d->SetPhaseTiming(true);
    // BENCH_DAGNODE_TRACE=1: the batched repair's phase intervals as a TRACE line (thread index,
    // phase id: 0 fetch, 1 stage, 2 codec, 3 put, 4 wait for the fetch ahead, 5 wait for the writes;
    // start and end in ms)
    const bool trace = std::getenv("BENCH_DAGNODE_TRACE") != nullptr;
    d->SetPhaseTrace(trace);
    d->ResetPhases();
    t0 = clk::now();
    d->RepairDataNodeBatched(0, rj, 256, &rep);
    const double repb = secs(t0);
    if (trace) {
        const auto ev = d->PhaseEvents();
        std::vector<uint64_t> tids;
        std::string out;
        for (const auto& e : ev) {
            size_t ti = std::find(tids.begin(), tids.end(), e.thread) - tids.begin();
            if (ti == tids.size()) tids.push_back(e.thread);
            char buf[96];
            std::snprintf(buf, sizeof buf, "%s[%zu,%d,%.3f,%.3f]", out.empty() ? "" : ",", ti, e.phase, e.t0 * 1e3, e.t1 * 1e3);
            out += buf;
        }
        std::printf("TRACE {\"leg\": \"repair_batched\", \"k\": %d, \"m\": %d, \"B\": %zu, \"wall_ms\": %.3f, \"events\": [%s]}\n",
                    k, m, B, repb * 1e3, out.c_str());
        d->SetPhaseTrace(false);
    }
    phase_json("repair_batched", repb);
    d->SetPhaseTiming(false);
    // mutcask-backed datanodes (server.go:207): every value also carries a CRC-32 of the whole
    // entry (cask.go:73-79).  Put / PutMany with the entry CRC-16 from the GPU pass and the
    // value CRC-32 from each datanode (the default), against the datanodes computing both, and
    // against both from the GPU.
    double putm = 0, putmh = 0, put1m = 0, put1mh = 0, putm32 = 0, put1m32 = 0, c32 = 0;
    {
        DagNodeConfig mc = cfg;
        std::vector<std::shared_ptr<DataNodeClient>> mcl;
        for (int i = 0; i < k + m; i++) mcl.push_back(std::make_shared<InProcDataNode>(cfg.nodes[i], KvEngine::Mutcask));
        std::unique_ptr<DagNode> md;
        if (!DagNode::New(mc, mcl, &md).ok()) return 2;
        md->HealthCheckAll();
        md->PutMany({"warm"}, {blocks[0]});
        md->SetGpuChecksums(false);
        t0 = clk::now();
        for (int i = 0; i < N; i++) md->Put(keys[i], blocks[i]);
        put1mh = secs(t0);
        t0 = clk::now();
        md->PutMany(keys, blocks);
        putmh = secs(t0);
        md->SetGpuChecksums(true);
        md->Put("warm", blocks[0]);
        t0 = clk::now();
        for (int i = 0; i < N; i++) md->Put(keys[i], blocks[i]);
        put1m = secs(t0);
        t0 = clk::now();
        md->PutMany(keys, blocks);
        putm = secs(t0);
        md->SetGpuValueChecksums(true);  // the CRC-32 from the GPU pass as well
        t0 = clk::now();
        for (int i = 0; i < N; i++) md->Put(keys[i], blocks[i]);
        put1m32 = secs(t0);
        t0 = clk::now();
        md->PutMany(keys, blocks);
        putm32 = secs(t0);
        t0 = clk::now();
        volatile uint32_t s32 = 0;
        for (int i = 0; i < N; i++) s32 ^= crc32_ieee(blocks[i].data(), blocks[i].size());
        c32 = secs(t0);
    }
    std::printf("RS(%d,%d) %d blocks x %zu B (%.2f GiB payload), in-process datanodes\n", k, m, N, B, gib);
    std::printf("Put per block      %8.2f GiB/s (datanode CRC: %.2f)\n", gib / put1, gib / put1h);
    std::printf("PutMany (batched)  %8.2f GiB/s (datanode CRC: %.2f)\n", gib / putb, gib / putbh);
    std::printf("Put, %d threads    %8.2f GiB/s (%ld encodes in %ld coalesced GPU batches)\n", T, gib / putT, calls,
                batches);
    std::printf("Get, 1 lost shard  %8.2f GiB/s\nGetMany (batched)  %8.2f GiB/s (batch %zu)\n", gib / get1, gib / getb,
                best_batch);
    std::printf("Get / GetMany, GPU-verified reads %6.2f / %.2f GiB/s\n", gib / get1v, gib / getbv);
    std::printf("Get, %d threads    %8.2f GiB/s (%ld reconstructs in %ld coalesced GPU batches)\n", T, gib / getT,
                gcalls, gbatches);
    std::printf("RepairDataNode     %8.2f GiB/s (of block payload)\nRepair batched     %8.2f GiB/s (%zu keys)\n",
                gib / rep1, gib / repb, rep);
    std::printf("Put, mutcask       %8.2f GiB/s (datanode CRCs: %.2f; CRC-32 on the GPU too: %.2f)\n", gib / put1m,
                gib / put1mh, gib / put1m32);
    std::printf("PutMany, mutcask   %8.2f GiB/s (datanode CRCs: %.2f; CRC-32 on the GPU too: %.2f)\n", gib / putm,
                gib / putmh, gib / putm32);
    std::printf("CRC-16 alone       %8.2f GiB/s (one core, block bytes, carry-less folding)\n", gib / crc);
    std::printf("CRC-32 alone       %8.2f GiB/s (one core, block bytes, carry-less folding)\n", gib / c32);
#ifdef FAKE_RSMI_FAST
    const char* threads = std::getenv("FAKE_RSMI_THREADS") ? std::getenv("FAKE_RSMI_THREADS") : std::getenv("OMP_NUM_THREADS");
    std::printf("RESULT {\"codec\": \"cpu\", \"isa\": \"%s\", \"threads\": \"%s\", ", rs_cpu_isa(), threads ? threads : "all");
#else
    std::printf("RESULT {\"codec\": \"gpu\", ");
#endif
    std::printf("\"k\": %d, \"m\": %d, \"B\": %zu, \"N\": %d, \"put\": %.3f, \"putmany\": %.3f, \"put_threads\": %.3f, "
                "\"get\": %.3f, \"getmany\": %.3f, \"get_threads\": %.3f, \"repair\": %.3f, \"repair_batched\": %.3f, "
                "\"put_nolone\": %.3f, \"get_nolone\": %.3f, \"repair_nolone\": %.3f, \"put_threads_calls\": %ld, "
                "\"put_threads_batches\": %ld, \"get_threads_calls\": %ld, \"get_threads_batches\": %ld}\n",
                k, m, B, N, gib / put1, gib / putb, gib / putT, gib / get1, gib / getb, gib / getT, gib / rep1, gib / repb,
                gib / put1n, gib / get1n, gib / rep1n, calls, batches, gcalls, gbatches);
#ifdef FAKE_RSMI_FAST
    std::printf("PHASES {\"codec\": \"cpu\", \"k\": %d, \"m\": %d, \"B\": %zu, %s}\n", k, m, B, phases.c_str());
#else
    std::printf("PHASES {\"codec\": \"gpu\", \"k\": %d, \"m\": %d, \"B\": %zu, %s}\n", k, m, B, phases.c_str());
#endif
    return 0;
}
