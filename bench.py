#!/usr/bin/env python3
"""bench.py -- device-resident RS encode + reconstruct throughput on MI355X.

Default workload (BASELINE.json configs[2], the metric's own config): RS(10,4) over
256 KiB blocks, 4096 blocks per GPU (1 GiB of payload), synthetic uniform random bytes
already resident in HBM.  One step = encode every block (dag/node/dagnode/erasure.go:60)
then ReconstructData of a lost data shard 0 for every block (erasure.go:82, the
DagNode.Get path), both through the C-ABI (include/rsmi.h) on one HIP stream.
`--config` selects the other BASELINE configs for side measurements (not the headline).

Multi-GPU: one process per GPU (torchrun); blocks are independent, so every rank codes
its own blocks (weak scaling) and no data-path collective exists.  gloo carries only
the timing barrier and the max-over-ranks reduction.

Prints ONE JSON line (rank 0).  roofline.achieved is the encode kernel's algorithmic
bytes ((k+m)*S per block) per launch divided by its average launch time, measured with
HIP events on the launch stream inside the timed region; cpu_baseline times the
oracle's multi-threaded SIMD restatement (oracle/rs_cpu_fast.c) on a bounded sample on
this host's cores.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import rsmi  # noqa: E402

METRIC = "GiB/s device-resident RS encode+reconstruct, 256 KiB blocks; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

# BASELINE.json configs -> (k, m, block KiB, blocks per GPU, lost shards for the reconstruct leg)
CONFIGS = {
    "rs10_4_256k": (10, 4, 256, 4096, "0"),      # configs[2]: the headline (default)
    "rs4_2_256k": (4, 2, 256, 4096, ""),         # configs[1]: encode only
    "rs10_4_1m": (10, 4, 1024, 1024, ""),        # configs[3]: encode only, 1024 blocks/GPU
    "rs16_4_4m": (16, 4, 4096, 256, "0,9"),      # configs[4]: encode + 2-shard Reconstruct
    "rs2_1_256k": (2, 1, 256, 4096, "1"),        # configs[0] shape on the device
}


def parse():
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
    p.add_argument("--chunks-per-lane", type=int, default=0)
    p.add_argument("--nontemporal", type=int, default=-1)
    p.add_argument("--pitch", type=int, default=0, help="diagnostic: row pitch in HBM (0 = rsmi_recommended_pitch)")
    p.add_argument("--option", action="append", default=[], metavar="KEY=VALUE",
                   help="diagnostic: any rsmi_set_option knob, repeatable (A/B in the bench's own context)")
    p.add_argument("--share-device", action="store_true",
                   help="rehearsal only: every rank uses cuda:0 (multi-rank path on a 1-GPU box)")
    p.add_argument("--copy-inclusive", action="store_true",
                   help="also time host->device->host through pinned buffers (reported, never `value`)")
    return p.parse_args()


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

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


def cpu_baseline(k, m, B, lost, data_only, seconds):
    """Oracle SIMD restatement of the reference CPU path on host cores, bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as orc

    L = orc.lib()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 64))
    S = (B + k - 1) // k
    n = k + m
    nb = max(16, min(256, (256 << 20) // (n * S)))
    shards = np.zeros((nb, n, S), dtype=np.uint8)
    shards[:, :k, :] = np.random.default_rng(7).integers(0, 256, size=(nb, k, S), dtype=np.uint8)
    present = np.array([0 if i in lost else 1 for i in range(n)], dtype=np.uint8)
    data = np.ascontiguousarray(shards[:, :k])
    par = np.zeros((nb, m, S), dtype=np.uint8)

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
    gibs = reps * nb * B / el / 2**30
    reps1, el1 = rate(1, max(1.0, seconds / 4))  # the 1-core figure SURVEY.md 8(d) asks for
    what = "encode" + (f"+{'ReconstructData' if data_only else 'Reconstruct'}(lost {lost})" if lost else "")
    return {
        "value": round(gibs, 3),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{reps} passes x {nb} blocks of {B // 1024} KiB RS({k},{m}) {what}, "
                  f"oracle/rs_cpu_fast.c {L.rs_cpu_isa().decode()}, {threads} threads, {el:.1f} s",
        "single_core_value": round(reps1 * nb * B / el1 / 2**30, 3),
    }


def load_traffic(label):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC pass."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(label)
    except Exception:
        return None


def copy_inclusive(codec, k, m, S, nb, lost, data_only):
    """Host-resident encode(+reconstruct) through pinned buffers: H2D/compute/D2H overlapped
    over the library's 3 streams.  PCIe-bound; reported in DESIGN.md, never `value`."""
    import ctypes

    L = rsmi.lib()
    n = k + m
    din = L.rsmi_host_alloc(nb * k * S)
    dpar = L.rsmi_host_alloc(nb * m * S)
    dsh = L.rsmi_host_alloc(nb * n * S)
    arr = np.ctypeslib.as_array((ctypes.c_uint8 * (nb * n * S)).from_address(dsh))
    arr[:] = np.random.default_rng(3).integers(0, 256, size=arr.shape, dtype=np.uint8)
    ctypes.memmove(din, dsh, nb * k * S)
    present = [i not in lost for i in range(n)]
    codec.encode_batch_host_ptr(din, k * S, dpar, m * S, S, nb)
    if lost:
        codec.reconstruct_batch_host_ptr(dsh, n * S, S, nb, present, data_only)
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        codec.encode_batch_host_ptr(din, k * S, dpar, m * S, S, nb)
    t1 = time.perf_counter()
    for _ in range(reps if lost else 0):
        codec.reconstruct_batch_host_ptr(dsh, n * S, S, nb, present, data_only)
    t2 = time.perf_counter()
    B = k * S
    res = {"blocks": nb, "encode_GiBs": round(reps * nb * B / (t1 - t0) / 2**30, 2)}
    if lost:
        res["reconstruct_GiBs"] = round(reps * nb * B / (t2 - t1) / 2**30, 2)
        res["enc_plus_rec_GiBs"] = round(reps * nb * B / (t2 - t0) / 2**30, 2)
        # mixed (BASELINE configs[4]): an encode stream and a reconstruct stream at once, each on
        # its own context (own HIP streams and staging), so one call's uploads overlap the
        # other's, and the D2H of either rides beside the H2D of both (PCIe is full duplex)
        import threading

        other = rsmi.Codec(k, m, codec.device)
        other.reconstruct_batch_host_ptr(dsh, n * S, S, nb, present, data_only)
        errs = []

        def run(f):
            try:
                for _ in range(reps):
                    f()
            except Exception as e:  # surfaced below
                errs.append(e)

        th = [threading.Thread(target=run, args=(lambda: codec.encode_batch_host_ptr(din, k * S, dpar, m * S, S, nb),)),
              threading.Thread(target=run, args=(lambda: other.reconstruct_batch_host_ptr(
                  dsh, n * S, S, nb, present, data_only),))]
        t3 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        t4 = time.perf_counter()
        other.close()
        if errs:
            raise errs[0]
        res["mixed_concurrent_GiBs"] = round(2 * reps * nb * B / (t4 - t3) / 2**30, 2)
    for p in (din, dpar, dsh):
        L.rsmi_host_free(p)
    return res


def main():
    a = parse()
    world, rank, local = dist_setup()
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU (no CPU fallback)")
    if a.share_device:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    k, m, bkib, nb_default, lost_s = CONFIGS[a.config]
    n = k + m
    B = bkib * 1024
    S = (B + k - 1) // k
    rs = rsmi.recommended_pitch(S)  # power-of-two shard slots in HBM (DESIGN.md "Layout")
    if a.pitch:
        assert a.pitch >= S and a.pitch % 16 == 0, "--pitch: a multiple of 16 bytes, at least the shard size"
        rs = a.pitch
    bs = n * rs
    nb = a.blocks or nb_default
    lost = [int(x) for x in lost_s.split(",") if x != ""]
    present = [i not in lost for i in range(n)]
    data_only = all(i < k for i in lost)

    # synthetic blocks resident in HBM; Split's zero padding in the last data row
    g = torch.Generator(device=dev)
    g.manual_seed(0xF11EDA6 + rank)
    buf = torch.randint(0, 256, (nb, n, rs), dtype=torch.uint8, device=dev, generator=g)
    pad = k * S - B
    if pad:
        buf[:, k - 1, S - pad:S] = 0
    base = buf.data_ptr()

    codec = rsmi.Codec(k, m, local)
    if a.chunks_per_lane:
        codec.set_option("chunks_per_lane", a.chunks_per_lane)
    if a.nontemporal >= 0:
        codec.set_option("nontemporal", a.nontemporal)
    for kv in a.option:
        key, val = kv.split("=", 1)
        codec.set_option(key, int(val))
    stream = torch.cuda.Stream(device=dev)
    sh = stream.cuda_stream

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

    # two HIP events per step (before / after the encode launch) plus one at the end: the
    # encode kernel's time is ev_b[i]->ev_a[i], the reconstruct's ev_a[i]->ev_b[i+1]
    ev_b = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    ev_a = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        ev_b[i].record(stream)
        encode()
        ev_a[i].record(stream)
        reconstruct()
    ev_b[a.steps].record(stream)
    torch.cuda.synchronize()
    barrier(world)
    el = time.perf_counter() - t0
    el_max = max_over_ranks(el, world)

    enc_t = sorted(ev_b[i].elapsed_time(ev_a[i]) for i in range(a.steps))
    rec_t = sorted(ev_a[i].elapsed_time(ev_b[i + 1]) for i in range(a.steps))
    enc_ms, rec_ms = sum(enc_t) / a.steps, sum(rec_t) / a.steps
    r = len([i for i in lost if i < k or not data_only])
    enc_bytes = nb * (k + m) * S
    rec_bytes = nb * (k + r) * S
    enc_gbs = enc_bytes / (enc_ms * 1e-3) / 1e9

    total_payload = nb * B * a.steps * world
    value = total_payload / el_max / 2**30
    headline = a.config == "rs10_4_256k"
    what = f"RS({k},{m}) encode" + (
        f" + {'ReconstructData' if data_only else 'Reconstruct'} of lost shard(s) {lost}" if lost else "")
    out = {
        "metric": METRIC if headline else f"GiB/s device-resident {what}, {bkib} KiB blocks",
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
        "data": "synthetic (uniform random bytes, torch.randint in HBM)",
        "config": {
            "workload": f"{what}, {bkib} KiB blocks" + (" (BASELINE configs[2])" if headline else f" ({a.config})"),
            "blocks_per_gpu": nb,
            "block_bytes": B,
            "shard_bytes": S,
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
            "kernel": enc_kernel,
            "algorithmic_bytes_per_launch": enc_bytes,
            "avg_launch_ms": round(enc_ms, 4),
            "median_launch_ms": round(enc_t[a.steps // 2], 4),
        },
        "cpu_baseline": None,
    }
    if lost:
        out["reconstruct"] = {
            "kernel": rec_kernel,
            "achieved_GBs": round(rec_bytes / (rec_ms * 1e-3) / 1e9, 1),
            "frac": round(rec_bytes / (rec_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "algorithmic_bytes_per_launch": rec_bytes,
            "avg_launch_ms_incl_event_gap": round(rec_ms, 4),
        }
    if a.copy_inclusive:
        out["copy_inclusive"] = copy_inclusive(codec, k, m, S, min(nb, max(1, (1 << 30) // B)), lost, data_only)
    if rank == 0 and world == 1 and a.cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline(k, m, B, lost, data_only, a.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    codec.close()
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
