#!/usr/bin/env python3
"""bench.py -- device-resident RS encode + reconstruct throughput on MI355X.

Default workload (BASELINE.json configs[2], the metric's own config): RS(10,4) over
256 KiB blocks, 4096 blocks per GPU (1 GiB of payload), resident in HBM.  Block b holds
BASELINE.md's synthetic bytes: splitmix64 seeded with 0xF11EDA6 ^ b (b = the block's index in
the whole job), generated on the device.  One step = encode every block
(dag/node/dagnode/erasure.go:60) then ReconstructData of a lost data shard 0 for every block
(erasure.go:82, the DagNode.Get path), both through the C-ABI (include/rsmi.h) on one HIP
stream.  After the timed steps the run checks itself: every lost row is erased and rebuilt
and compared with its original bytes on the device, every data row is compared with a fresh
copy of the generator's output, and the parity of sampled blocks is compared with the CPU
oracle (test infrastructure, never the thing measured).  A mismatch exits non-zero.
`--config` selects the other BASELINE configs, `--layout split` the contiguous Split layout
(rows back to back at pitch S, as blocks arrive from the Put path) and `--fused-crc` the
encode with the datanode CRC-16 of every shard fused in (DagNode.Put's form) as side lines.

Multi-GPU: one process per GPU.  `--gpus N` without a launcher spawns the N ranks itself
(before anything touches the GPU); under torchrun WORLD_SIZE must equal N.  Blocks are
independent (node.go:358-408), so every rank codes its own contiguous share of the job's
blocks (weak scaling) and no data-path collective exists; gloo carries only the timing
barrier, the max-over-ranks reduction and the per-rank roofline figures.

Prints ONE JSON line (rank 0).  roofline.achieved is the encode kernel's algorithmic bytes
((k+m)*S per block) per launch divided by its average launch time, measured with HIP events
on the launch stream inside the timed region; cpu_baseline times the oracle's multi-threaded
SIMD restatement (oracle/rs_cpu_fast.c) on the same blocks on this host's cores.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))

# numpy and torch load after the launcher decision (main) or on import as a module: the launcher
# of `--gpus N` must not map or initialise the HIP runtime before it spawns the ranks (torch links
# libamdhip64, so importing it maps the runtime).
np = torch = None


def _heavy_imports():
    global np, torch
    import numpy
    import torch as _torch

    np, torch = numpy, _torch


if __name__ != "__main__":
    _heavy_imports()

METRIC = "GiB/s device-resident RS encode+reconstruct, 256 KiB blocks; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
SEED = 0xF11EDA6  # splitmix64, seed 0xF11EDA6 ^ block index

# BASELINE.json configs -> (k, m, block KiB, blocks per GPU, lost shards for the reconstruct leg)
CONFIGS = {
    "rs10_4_256k": (10, 4, 256, 4096, "0"),      # configs[2]: the headline (default)
    "rs4_2_256k": (4, 2, 256, 4096, ""),         # configs[1]: encode only
    "rs10_4_1m": (10, 4, 1024, 1024, ""),        # configs[3]: encode only, 1024 blocks/GPU
    "rs16_4_4m": (16, 4, 4096, 256, "0,9"),      # configs[4]: encode + 2-shard Reconstruct
    "rs2_1_256k": (2, 1, 256, 4096, "1"),        # configs[0] shape on the device
}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="rs10_4_256k", choices=sorted(CONFIGS))
    p.add_argument("--blocks", type=int, default=0, help="blocks per GPU (0 = config default)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline time budget (0 = skip)")
    p.add_argument("--settle-ms", type=float, default=200.0,
                   help="untimed run of the step before the warmup steps, past the GPU's start-up power "
                        "transient (DESIGN.md section 5); 0 = off")
    p.add_argument("--sustained-steps", type=int, default=200,
                   help="after the K timed steps, also time this many back to back (reported as "
                        "`sustained`, never `value`); 0 = off")
    p.add_argument("--layout", choices=("pitched", "split"), default="pitched",
                   help="pitched: rows at rsmi_recommended_pitch (the batch API's layout); split: the "
                        "contiguous Split layout, rows back to back at pitch S")
    p.add_argument("--fused-crc", action="store_true",
                   help="side line: the encode also returns the datanode CRC-16 of every shard "
                        "(rsmi_encode_batch_dev_crc, DagNode.Put's form)")
    p.add_argument("--pitch", type=int, default=0, help="diagnostic: row pitch in HBM (0 = rsmi_recommended_pitch)")
    p.add_argument("--option", action="append", default=[], metavar="KEY=VALUE",
                   help="diagnostic: any rsmi_set_option knob, repeatable")
    p.add_argument("--share-device", action="store_true",
                   help="rehearsal only: every rank uses cuda:0 (multi-rank path on a 1-GPU box)")
    p.add_argument("--copy-inclusive", action="store_true",
                   help="also time host->device->host through pinned buffers (reported, never `value`)")
    p.add_argument("--group", default="", metavar="DEVS",
                   help="with --copy-inclusive: also run the host batch through one device group "
                        "(rsmi_group_*, one process over several GPUs) of these devices, e.g. 0,1,2,3 or "
                        "0,0 (two contexts on one GPU); 'all' = every visible GPU")
    p.add_argument("--event-every", type=int, default=5, metavar="N",
                   help="time the kernels of every N-th timed step with HIP events (3 per sampled step); "
                        "each event between kernels costs the step ~3 us (tools/eventgap.py), so the "
                        "other steps run uninstrumented.  1 = every step")
    p.add_argument("--no-verify", action="store_true", help="skip the post-run self check")
    p.add_argument("--mock", action="store_true",
                   help="test only: a CPU stand-in for the device step, to exercise the launcher, the "
                        "ranks and the JSON line on a host without a GPU; never a measurement")
    a = p.parse_args(argv)
    if a.steps < 1 or a.warmup < 0 or a.event_every < 1:
        p.error("--steps and --event-every must be at least 1, --warmup at least 0")
    return a


# ---------------------------------------------------------------- launcher and ranks
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(a):
    """--gpus N with no launcher: start N ranks of this script, one per GPU, and exit with the
    first failing rank's code.  Nothing here maps or initialises the HIP runtime: numpy and
    torch are not imported yet, and the GPUs are counted from sysfs (rsmi.multi.visible_gpu_count,
    honouring ROCR/HIP_VISIBLE_DEVICES), or by a child process where sysfs has no KFD topology.
    --share-device (a rehearsal on one GPU) needs one visible GPU, --mock none."""
    from rsmi import multi

    need = 0 if a.mock else (1 if a.share_device else a.gpus)
    have = None
    if need:
        have = multi.visible_gpu_count()
        if have is None:  # no KFD topology in sysfs: a child process counts (and initialises HIP)
            out = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                                 capture_output=True, text=True)
            have = int(out.stdout.strip() or "0") if out.returncode == 0 else 0
    probe = os.environ.get("RSMI_BENCH_LAUNCH_PROBE")
    if probe:  # test hook: what this process has mapped and opened at spawn time
        _launch_probe(probe, have)
    if need and have < need:
        raise SystemExit(f"bench.py --gpus {a.gpus}: only {have} GPU(s) visible")
    port = _free_port()
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus),
                   LOCAL_WORLD_SIZE=str(a.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code and not rc:
                rc = code
                for q in procs:  # one rank failed: the others would wait at a barrier forever
                    q.terminate()
        time.sleep(0.05)
    return rc


def _launch_probe(path, have):
    """Record the launcher's state just before it spawns ranks: shared objects of the HIP / HSA
    runtimes mapped into this process (/proc/self/maps), descriptors open on /dev/kfd (the
    runtime opens it when it initialises), and whether torch or numpy were imported."""
    with open("/proc/self/maps") as f:
        maps = sorted({ln.split()[-1] for ln in f if len(ln.split()) >= 6})
    hip = [m for m in maps if any(x in os.path.basename(m) for x in ("libamdhip64", "libhsa-runtime"))]
    kfd = 0
    for fd in os.listdir("/proc/self/fd"):
        try:
            kfd += os.readlink(f"/proc/self/fd/{fd}") == "/dev/kfd"
        except OSError:
            pass
    with open(path, "w") as f:
        json.dump({"gpus_counted": have, "hip_libs_mapped": hip, "kfd_fds": kfd,
                   "torch_imported": "torch" in sys.modules, "numpy_imported": "numpy" in sys.modules}, f)


_JSON_OUT = None  # multi-rank: the real stdout, kept for the one JSON line


def emit(line):
    """The run's JSON line, alone on stdout."""
    if _JSON_OUT is not None:
        _JSON_OUT.write(line + "\n")
        _JSON_OUT.flush()
    else:
        print(line, flush=True)


def dist_setup():
    global _JSON_OUT
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        # gloo and the runtime print connection chatter on fd 1; send everything but the JSON
        # line to stderr, so stdout carries exactly one line under any launcher
        sys.stdout.flush()
        _JSON_OUT = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def max_over_ranks(x, world):
    if world == 1:
        return x
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def finish(world):
    """Every rank waits for rank 0's CPU leg, then leaves the process group together (a rank
    that exits while a peer still talks to gloo can abort in the group's destructor)."""
    if world > 1:
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()


def gather(obj, world):
    if world == 1:
        return [obj]
    import torch.distributed as dist

    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def partition_blocks(nblocks, world, rank):
    from rsmi import multi

    return multi.partition_blocks(nblocks, world, rank)


# ---------------------------------------------------------------- synthetic blocks
_GAMMA, _C1, _C2 = 0x9E3779B97F4A7C15, 0xBF58476D1CE4E5B9, 0x94D049BB133111EB


def _s64(x):
    return x - (1 << 64) if x >= 1 << 63 else x


def _lsr(x, s):
    return (x >> s) & ((1 << (64 - s)) - 1)  # logical shift on int64


def splitmix_blocks(ids, nbytes, device):
    """Block b's first nbytes bytes of splitmix64 seeded with SEED ^ b, for every b in ids:
    (len(ids), nbytes) uint8, byte-identical to tests/oracle_lib.splitmix64_bytes."""
    n = (nbytes + 7) // 8
    seeds = torch.as_tensor([SEED ^ int(b) for b in ids], dtype=torch.int64, device=device)
    i = torch.arange(1, n + 1, dtype=torch.int64, device=device)
    x = seeds[:, None] + i[None, :] * _s64(_GAMMA)  # int64 arithmetic wraps mod 2^64
    x = (x ^ _lsr(x, 30)) * _s64(_C1)
    x = (x ^ _lsr(x, 27)) * _s64(_C2)
    x = x ^ _lsr(x, 31)
    return x.view(torch.uint8)[:, :nbytes]


class Layout:
    """Where row r of block b lives: base + b*bs + r*rs.  pitched: rs = the recommended pitch
    (multiple of 16); split: rs = S, rows back to back (the Split layout of erasure.go:55)."""

    def __init__(self, k, m, B, nb, kind, pitch=0):
        import rsmi

        self.k, self.m, self.n, self.B, self.nb = k, m, k + m, B, nb
        self.S = (B + k - 1) // k
        if kind == "split":
            self.rs = self.S
        else:
            self.rs = pitch or rsmi.recommended_pitch(self.S)
            assert self.rs >= self.S and self.rs % 16 == 0, "--pitch: a multiple of 16, at least S"
        self.bs = self.n * self.rs

    def rows(self, buf, r0, r1):
        """View (nb, r1 - r0, S) of rows r0..r1-1 of every block."""
        return buf.as_strided((self.nb, r1 - r0, self.S), (self.bs, self.rs, 1), r0 * self.rs)

    def fill(self, buf, first_block, device, chunk=256):
        """Data rows of every block from the generator, Split's zero padding past B."""
        k, S, B = self.k, self.S, self.B
        for b0 in range(0, self.nb, chunk):
            b1 = min(self.nb, b0 + chunk)
            blk = torch.zeros((b1 - b0, k * S), dtype=torch.uint8, device=device)
            blk[:, :B] = splitmix_blocks(range(first_block + b0, first_block + b1), B, device)
            sub = buf[b0 * self.bs:b1 * self.bs].as_strided((b1 - b0, k, S), (self.bs, self.rs, 1))
            sub.copy_(blk.view(b1 - b0, k, S))


# ---------------------------------------------------------------- CPU legs (rank 0 only)
def cpu_baseline(k, m, S, B, data_host, lost, data_only, seconds, world=1):
    """The oracle's SIMD restatement of the reference CPU path (test infrastructure, used here
    only as the reported baseline) on host cores, over the same blocks the GPU coded.  Timed at
    N = 1 only (rank 0, after the GPU legs): the multi-GPU lines carry none, so the scaling runs
    stay short."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as orc

    L = orc.lib()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 64))
    n = k + m
    nb = data_host.shape[0]
    data = np.ascontiguousarray(data_host)
    par = np.zeros((nb, m, S), dtype=np.uint8)
    shards = np.zeros((nb, n, S), dtype=np.uint8)
    shards[:, :k] = data
    present = np.array([0 if i in lost else 1 for i in range(n)], dtype=np.uint8)

    def one(th):
        L.rs_cpu_encode_batch(k, m, data.ctypes.data, k * S, par.ctypes.data, m * S, S, nb, th)
        if lost:
            L.rs_cpu_reconstruct_batch(k, m, shards.ctypes.data, n * S, S, nb, present.ctypes.data,
                                       1 if data_only else 0, th)

    def rate(th, budget):
        one(th)  # warm
        reps = 0
        t0 = time.perf_counter()
        while True:
            one(th)
            reps += 1
            el = time.perf_counter() - t0
            if el >= budget:
                return reps, el

    reps, el = rate(threads, seconds)
    reps1, el1 = rate(1, max(1.0, seconds / 4))  # the 1-core figure SURVEY.md 8(d) asks for
    what = "encode" + (f"+{'ReconstructData' if data_only else 'Reconstruct'}(lost {lost})" if lost else "")
    return {
        "value": round(reps * nb * B / el / 2**30, 3),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{reps} passes x the bench's own {nb} blocks of {B // 1024} KiB RS({k},{m}) {what}, "
                  f"oracle/rs_cpu_fast.c {L.rs_cpu_isa().decode()}, {threads} threads, {el:.1f} s",
        "single_core_value": round(reps1 * nb * B / el1 / 2**30, 3),
        "host_cpus": os.cpu_count(),
        "ranks": world,
    }


def load_traffic(label):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC pass."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
            return json.load(f).get(label)
    except Exception:
        return None


def load_trace_window(label):
    """The kernel's average duration (ms) over the timed window of the committed rocprofv3 kernel
    trace of this same command (tools/trace_window.py -> profiles/trace_window.json)."""
    try:
        with open(os.path.join(ROOT, "profiles", "trace_window.json")) as f:
            return json.load(f).get(label)
    except Exception:
        return None


def copy_inclusive(codec, k, m, S, nb, lost, data_only, world, group=None):
    """Host-resident encode(+reconstruct) through page-locked buffers (the zero-copy direct
    path).  Every rank runs each leg at the same time, so the aggregate shows
    what the ranks' PCIe links and the shared host memory give together.  PCIe-bound; reported
    in DESIGN.md, never `value`."""
    import ctypes

    import rsmi

    L = rsmi.lib()
    n = k + m
    din = L.rsmi_host_alloc(nb * k * S)
    dpar = L.rsmi_host_alloc(nb * m * S)
    dsh = L.rsmi_host_alloc(nb * n * S)
    arr = np.ctypeslib.as_array((ctypes.c_uint8 * (nb * n * S)).from_address(dsh))
    arr[:] = np.random.default_rng(3).integers(0, 256, size=arr.shape, dtype=np.uint8)
    ctypes.memmove(din, dsh, nb * k * S)
    present = [i not in lost for i in range(n)]
    B = k * S
    reps = 3

    def leg(f):
        f()  # warm
        barrier(world)
        t0 = time.perf_counter()
        for _ in range(reps):
            f()
        el = time.perf_counter() - t0
        return reps * nb * B * world / max_over_ranks(el, world) / 2**30

    res = {"blocks_per_rank": nb, "ranks": world}
    res["encode_GiBs"] = round(leg(lambda: codec.encode_batch_host_ptr(din, k * S, dpar, m * S, S, nb)), 2)
    if lost:
        res["reconstruct_GiBs"] = round(leg(lambda: codec.reconstruct_batch_host_ptr(
            dsh, n * S, S, nb, present, data_only)), 2)
        # mixed (BASELINE configs[4]): an encode stream and a reconstruct stream at once, each on
        # its own context (own HIP streams and staging), so one call's uploads overlap the
        # other's, and the D2H of either rides beside the H2D of both (PCIe is full duplex)
        import threading

        other = rsmi.Codec(k, m, codec.device)
        errs = []

        def both():
            def run(f):
                try:
                    f()
                except Exception as e:  # surfaced below
                    errs.append(e)

            th = [threading.Thread(target=run, args=(lambda: codec.encode_batch_host_ptr(din, k * S, dpar, m * S, S, nb),)),
                  threading.Thread(target=run, args=(lambda: other.reconstruct_batch_host_ptr(
                      dsh, n * S, S, nb, present, data_only),))]
            for t in th:
                t.start()
            for t in th:
                t.join()

        res["mixed_concurrent_GiBs"] = round(2 * leg(both), 2)
        other.close()
        if errs:
            raise errs[0]
    if group:
        # the same host batch spread over a device group from this one process: contiguous
        # block ranges, one member context (own streams and staging) and NUMA-bound worker each,
        # over buffers whose member ranges sit on the members' NUMA nodes (rsmi_group_host_alloc)
        with rsmi.DeviceGroup(k, m, group) as g:
            gin, gpar, gsh = g.host_alloc(k * S, nb), g.host_alloc(m * S, nb), g.host_alloc(n * S, nb)
            ctypes.memmove(gsh, dsh, nb * n * S)
            ctypes.memmove(gin, din, nb * k * S)
            gr = {"devices": list(group), "numa_nodes": [g.member_numa_node(i) for i in range(len(group))]}
            gr["encode_GiBs"] = round(leg(lambda: g.encode_batch_host_ptr(gin, k * S, gpar, m * S, S, nb)), 2)
            if lost:
                gr["reconstruct_GiBs"] = round(leg(lambda: g.reconstruct_batch_host_ptr(
                    gsh, n * S, S, nb, present, data_only)), 2)
            for q in (gin, gpar, gsh):
                g.host_free(q)
        res["group"] = gr
    for p in (din, dpar, dsh):
        L.rsmi_host_free(p)
    return res


# ---------------------------------------------------------------- verification
def verify(codec, lay, buf, first_block, lost, data_only, lost_ref, stream, raw=None, samples=16):
    """Self check after the timed steps.  Returns a dict; raises SystemExit on a mismatch."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as orc

    k, m, n, S, nb = lay.k, lay.m, lay.n, lay.S, lay.nb
    dev = buf.device
    rec_rows = [i for i in lost if i < k or not data_only]
    # 1. every rebuilt row of every block, on the device: erase, rebuild once, compare
    if rec_rows:
        for i in rec_rows:
            lay.rows(buf, i, i + 1).zero_()
        torch.cuda.synchronize()  # the zeroing ran on torch's stream, the rebuild runs on the bench's
        codec.reconstruct_batch_dev(buf.data_ptr(), lay.rs, lay.bs, S, nb, [i not in lost for i in range(n)],
                                    data_only, stream)
        torch.cuda.synchronize()
        for j, i in enumerate(rec_rows):
            if not torch.equal(lay.rows(buf, i, i + 1)[:, 0], lost_ref[:, j]):
                raise SystemExit(f"verify: rebuilt row {i} differs from the original bytes")
    # 2. every data row of every block against the generator (the kernels never write them)
    fresh = torch.zeros(lay.nb * lay.bs, dtype=torch.uint8, device=dev)
    lay.fill(fresh, first_block, dev)
    if not torch.equal(lay.rows(buf, 0, k), lay.rows(fresh, 0, k)):
        raise SystemExit("verify: data rows changed")
    del fresh
    # 3. parity (and CRCs) of sampled blocks against the CPU oracle
    rng = np.random.default_rng(first_block + 1)
    idx = sorted(set([0, nb - 1, nb // 2] + list(rng.integers(0, nb, size=max(0, samples - 3)))))
    rows = lay.rows(buf, 0, n)[idx].cpu().numpy()
    for j, b in enumerate(idx):
        blk = np.zeros(k * S, dtype=np.uint8)
        blk[:lay.B] = orc.splitmix64_bytes(SEED ^ (first_block + b), lay.B)
        want = orc.encode_fast(k, m, blk.reshape(1, k, S), threads=4)[0]
        if not np.array_equal(rows[j, k:], want):
            raise SystemExit(f"verify: parity of block {first_block + b} differs from the oracle")
    out = {"verified": True, "rebuilt_rows_checked": nb * len(rec_rows), "data_rows_checked": nb * k,
           "oracle_blocks": len(idx)}
    if raw is not None:
        got = raw[idx].cpu().numpy().astype(np.int64) & 0xFFFFFFFF
        import rsmi

        for j in range(len(idx)):
            for r in range(n):
                if rsmi.crc16_entry(b"", int(got[j, r]), S) != orc.crc16_ibm(rows[j, r].tobytes()):
                    raise SystemExit(f"verify: CRC-16 of block {first_block + idx[j]} row {r} differs")
        out["crc_blocks_checked"] = len(idx)
    return out


# ---------------------------------------------------------------- main
def run_mock(a, world, rank):
    """CPU stand-in for the device step (test only): a tiny RS(4,2) batch through the oracle, so
    the launcher, the ranks, the reductions and the JSON line run on a host without a GPU."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as orc

    k, m, S, nb = 4, 2, 4096, 8
    start, count = partition_blocks(nb * world, world, rank)
    data = np.stack([orc.splitmix64_bytes(SEED ^ b, k * S) for b in range(start, start + count)]).reshape(count, k, S)
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        orc.encode_fast(k, m, data, threads=1)
    el = max_over_ranks(time.perf_counter() - t0, world)
    per = gather({"rank": rank, "blocks": count}, world)
    if rank == 0:
        cpu = (cpu_baseline(k, m, S, k * S, data, [], True, min(a.cpu_seconds, 0.2), world)
               if a.cpu_seconds > 0 and world == 1 else None)
        emit(json.dumps({"metric": "mock", "mock": True, "value": round(nb * world * k * S * a.steps / el / 2**30, 4),
                          "unit": "GiB/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                          "ms_per_step": round(el * 1e3 / a.steps, 4), "higher_is_better": True, "scaling": "weak",
                          "vs_baseline": None, "dtype": "u8", "data": "mock (CPU stand-in, orchestration test only)",
                          "config": {"ranks": per}, "cpu_baseline": cpu}))


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return launch(a)
    _heavy_imports()
    world, rank, local = dist_setup()
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}")
    if a.mock:
        run_mock(a, world, rank)
        finish(world)
        return 0
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU (no CPU fallback)")
    import rsmi

    if a.share_device:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    k, m, bkib, nb_default, lost_s = CONFIGS[a.config]
    n = k + m
    B = bkib * 1024
    nb = a.blocks or nb_default
    lay = Layout(k, m, B, nb, a.layout, a.pitch)
    S, rs, bs = lay.S, lay.rs, lay.bs
    lost = [int(x) for x in lost_s.split(",") if x != ""]
    present = [i not in lost for i in range(n)]
    data_only = all(i < k for i in lost)
    rec_rows = [i for i in lost if i < k or not data_only]
    first_block, _ = partition_blocks(nb * world, world, rank)  # this rank's blocks of the job

    buf = torch.zeros(nb * bs + 64, dtype=torch.uint8, device=dev)
    lay.fill(buf, first_block, dev)
    lost_ref = torch.stack([lay.rows(buf, i, i + 1)[:, 0].clone() for i in rec_rows], 1) if rec_rows else None
    base = buf.data_ptr()
    raw = torch.zeros((nb, n), dtype=torch.int32, device=dev) if a.fused_crc else None

    codec = rsmi.Codec(k, m, local)
    for kv in a.option:
        key, val = kv.split("=", 1)
        codec.set_option(key, int(val))
    stream = torch.cuda.Stream(device=dev)
    sh = stream.cuda_stream

    if a.fused_crc:
        def encode():
            codec.encode_batch_dev_crc(base, rs, bs, base + k * rs, rs, bs, S, nb, raw.data_ptr(), sh)
    else:
        def encode():
            codec.encode_batch_dev(base, rs, bs, base + k * rs, rs, bs, S, nb, sh)

    def reconstruct():
        if lost:
            codec.reconstruct_batch_dev(base, rs, bs, S, nb, present, data_only, sh)

    # Settle: on a freshly loaded MI355X the encode kernel slows by up to 25 % for ~10 ms,
    # starting a few ms after the first launch, then returns to its steady rate (per-dispatch
    # traces in profiles/r01/README.md).  Run the untimed step for settle_ms of wall time first.
    settle_steps = 0
    if a.settle_ms > 0:
        t_end = time.perf_counter() + a.settle_ms / 1e3
        while time.perf_counter() < t_end:
            for _ in range(4):
                encode()
                reconstruct()
            settle_steps += 4
            torch.cuda.synchronize()
    for _ in range(a.warmup):
        encode()
        reconstruct()
    torch.cuda.synchronize()
    encode()
    enc_kernel = codec.last_kernel()
    reconstruct()
    rec_kernel = codec.last_kernel() if lost else None
    torch.cuda.synchronize()

    def timed(steps, every):
        # every `every`-th step is instrumented with three HIP events on the kernels' stream
        # (before the encode, between the kernels, after the reconstruct): the encode's time is
        # ev[0]->ev[1], the reconstruct's ev[1]->ev[2]; the other steps run without events, whose
        # cost between kernels (~3 us each) is instrumentation, not work (tools/eventgap.py)
        every = max(1, every)
        sampled = list(range(0, steps, every))
        evs = {i: [torch.cuda.Event(enable_timing=True) for _ in range(3)] for i in sampled}
        barrier(world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            ev = evs.get(i)
            if ev:
                ev[0].record(stream)
            encode()
            if ev:
                ev[1].record(stream)
            reconstruct()
            if ev:
                ev[2].record(stream)
        torch.cuda.synchronize()
        barrier(world)
        el = time.perf_counter() - t0
        enc_t = sorted(evs[i][0].elapsed_time(evs[i][1]) for i in sampled)
        rec_t = sorted(evs[i][1].elapsed_time(evs[i][2]) for i in sampled)
        return el, enc_t, rec_t

    el, enc_t, rec_t = timed(a.steps, a.event_every)
    el_max = max_over_ranks(el, world)
    sus = None
    if a.sustained_steps > 0:
        sel, _, _ = timed(a.sustained_steps, a.sustained_steps)
        sus = {"steps": a.sustained_steps,
               "value": round(nb * B * a.sustained_steps * world / max_over_ranks(sel, world) / 2**30, 2)}

    enc_ms, rec_ms = sum(enc_t) / len(enc_t), sum(rec_t) / len(rec_t)
    enc_bytes = nb * (k + m) * S
    rec_bytes = nb * (k + len(rec_rows)) * S
    enc_gbs = enc_bytes / (enc_ms * 1e-3) / 1e9
    rec_gbs = rec_bytes / (rec_ms * 1e-3) / 1e9 if lost else None

    ver = {"verified": False, "skipped": True}
    if not a.no_verify:
        ver = verify(codec, lay, buf, first_block, lost, data_only, lost_ref, sh, raw)
    per_rank = gather({"rank": rank, "encode_GBs": enc_gbs, "reconstruct_GBs": rec_gbs,
                       "verified": ver["verified"]}, world)

    value = nb * B * a.steps * world / el_max / 2**30
    headline = a.config == "rs10_4_256k" and a.layout == "pitched" and not a.fused_crc
    what = f"RS({k},{m}) encode" + (" with fused CRC-16 of every shard" if a.fused_crc else "") + (
        f" + {'ReconstructData' if data_only else 'Reconstruct'} of lost shard(s) {lost}" if lost else "")
    fr = [p["encode_GBs"] / HBM_PEAK_GBS for p in per_rank]
    out = {
        "metric": METRIC if headline else f"GiB/s device-resident {what}, {bkib} KiB blocks, {a.layout} layout",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(el_max * 1e3 / a.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: splitmix64(0xF11EDA6 ^ block) per block, generated in HBM (BASELINE.md)",
        "config": {
            "workload": f"{what}, {bkib} KiB blocks" + (" (BASELINE configs[2])" if headline else f" ({a.config})"),
            "blocks_per_gpu": nb,
            "block_bytes": B,
            "shard_bytes": S,
            "layout": a.layout,
            "row_pitch": rs,
            "settle": {"ms": a.settle_ms, "steps": settle_steps},
            "parallelism": f"independent blocks, {world} GPU(s), one process each, no collective",
            **({"options": a.option} if a.option else {}),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(enc_gbs, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(enc_gbs / HBM_PEAK_GBS, 4),
            "traffic": load_traffic(enc_kernel) if headline else None,
            "traffic_source": ("profiles/pmc_traffic.json: rocprofv3 FETCH_SIZE + WRITE_SIZE passes over this "
                               "kernel (tools/gpu_session.sh prof), per launch, gfx950-corrected; refreshed each "
                               "evidence session, not measured in this run") if headline else None,
            "kernel": enc_kernel + (" + its CRC-16 combine kernel" if a.fused_crc else ""),
            "algorithmic_bytes_per_launch": enc_bytes,
            "avg_launch_ms": round(enc_ms, 4),
            "median_launch_ms": round(enc_t[len(enc_t) // 2], 4),
            "launches_timed": len(enc_t),
            "timing": ("avg_launch_ms / achieved: HIP events on the kernels' stream around each kernel of every "
                       f"{a.event_every}th step, event-inflated (~3 %: the encode and reconstruct averages sum to more "
                       "than ms_per_step, which is timed without events); trace_window_avg_ms: the same kernel's "
                       "average over the timed window of the committed rocprofv3 kernel trace of this command "
                       "(profiles/trace_window.json, tools/gpu_session.sh prof), not measured in this run"),
            "trace_window_avg_ms": load_trace_window(enc_kernel) if headline else None,
            "per_rank_frac": {"min": round(min(fr), 4), "max": round(max(fr), 4),
                              "mean": round(sum(fr) / len(fr), 4)},
        },
        "cpu_baseline": None,
        "verify": {**ver, "ranks_verified": sum(1 for p in per_rank if p["verified"])},
    }
    if sus:
        out["sustained"] = sus
    if lost:
        out["reconstruct"] = {
            "kernel": rec_kernel,
            "achieved_GBs": round(rec_gbs, 1),
            "frac": round(rec_gbs / HBM_PEAK_GBS, 4),
            "algorithmic_bytes_per_launch": rec_bytes,
            "avg_launch_ms": round(rec_ms, 4),
            "trace_window_avg_ms": load_trace_window(rec_kernel) if headline else None,
        }
    if a.copy_inclusive:
        group = None
        if a.group and world == 1:
            group = (list(range(torch.cuda.device_count())) if a.group == "all"
                     else [int(x) for x in a.group.split(",")])
        out["copy_inclusive"] = copy_inclusive(codec, k, m, S, min(nb, max(1, (1 << 30) // B)), lost, data_only,
                                               world, group)
    if rank == 0 and a.cpu_seconds > 0 and world == 1:
        # the GPU legs are done, so the host cores are free (N = 1 only: the multi-GPU lines carry
        # no CPU figure)
        data_host = lay.rows(buf, 0, k).cpu().numpy()  # the bench's own blocks
        out["cpu_baseline"] = cpu_baseline(k, m, S, B, data_host, lost, data_only, a.cpu_seconds, world)
    if rank == 0:
        emit(json.dumps(out))
    codec.close()
    finish(world)
    return 0


if __name__ == "__main__":
    sys.exit(main())
