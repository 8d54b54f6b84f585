#!/usr/bin/env python3
"""bench.py -- device-resident RS encode + reconstruct throughput on MI355X.

Workload (BASELINE.json configs[2], the metric's own config): RS(10,4) over 256 KiB
blocks, 4096 blocks per GPU (1 GiB of payload), synthetic uniform random bytes already
resident in HBM.  One step = encode every block (dag/node/dagnode/erasure.go:60) then
ReconstructData of a lost data shard 0 for every block (erasure.go:82, the DagNode.Get
path), both through the C-ABI (include/rsmi.h) on one HIP stream.

Multi-GPU: one process per GPU (torchrun); blocks are independent, so every rank codes
its own 4096 blocks (weak scaling) and no data-path collective exists.  gloo carries
only the timing barrier and the max-over-ranks reduction.

Prints ONE JSON line (rank 0).  roofline.achieved is the encode kernel's algorithmic
bytes ((k+m)*S per block) per launch divided by its average launch time measured with
HIP events on the launch stream; cpu_baseline times the oracle's multi-threaded SIMD
restatement (oracle/rs_cpu_fast.c) on a bounded sample on this host's cores.
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


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--m", type=int, default=4)
    p.add_argument("--block-kib", type=int, default=256)
    p.add_argument("--blocks", type=int, default=4096, help="blocks per GPU")
    p.add_argument("--lost", type=str, default="0", help="comma list of lost shards for the reconstruct leg")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline time budget (0 = skip)")
    p.add_argument("--chunks-per-lane", type=int, default=0)
    p.add_argument("--nontemporal", type=int, default=-1)
    p.add_argument("--copy-inclusive", action="store_true", help="also time host->device->host (pinned) and print it")
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


def cpu_baseline(k, m, B, lost, seconds):
    """Oracle SIMD restatement of the reference CPU path on host cores, bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as orc

    L = orc.lib()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 64))
    S = (B + k - 1) // k
    n = k + m
    nb = 256
    shards = np.zeros((nb, n, S), dtype=np.uint8)
    shards[:, :k, :] = np.random.default_rng(7).integers(0, 256, size=(nb, k, S), dtype=np.uint8)
    present = np.array([0 if i in lost else 1 for i in range(n)], dtype=np.uint8)
    data = np.ascontiguousarray(shards[:, :k])
    par = np.zeros((nb, m, S), dtype=np.uint8)
    L.rs_cpu_encode_batch(k, m, data.ctypes.data, k * S, par.ctypes.data, m * S, S, nb, threads)  # warm
    reps = 0
    t0 = time.perf_counter()
    while True:
        L.rs_cpu_encode_batch(k, m, data.ctypes.data, k * S, par.ctypes.data, m * S, S, nb, threads)
        L.rs_cpu_reconstruct_batch(k, m, shards.ctypes.data, n * S, S, nb, present.ctypes.data, 1, threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    gibs = reps * nb * B / el / 2**30
    return {
        "value": round(gibs, 3),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{reps} passes x {nb} blocks of {B // 1024} KiB RS({k},{m}) encode+ReconstructData(lost {lost}), "
                  f"oracle/rs_cpu_fast.c {L.rs_cpu_isa().decode()}, {threads} threads, {el:.1f} s",
    }


def load_traffic(label):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC pass."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(label)
    except Exception:
        return None


def main():
    a = parse()
    world, rank, local = dist_setup()
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU (no CPU fallback)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    k, m, n = a.k, a.m, a.k + a.m
    B = a.block_kib * 1024
    S = (B + k - 1) // k
    rs = rsmi.recommended_pitch(S)  # power-of-two shard slots in HBM (DESIGN.md "Layout")
    bs = n * rs
    nb = a.blocks
    lost = [int(x) for x in a.lost.split(",") if x != ""]
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
    stream = torch.cuda.Stream(device=dev)
    sh = stream.cuda_stream

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        codec.encode_batch_dev(base, rs, bs, base + k * rs, rs, bs, S, nb, sh)
        if ev is not None:
            ev[1].record(stream)
        codec.reconstruct_batch_dev(base, rs, bs, S, nb, present, data_only, sh)
        if ev is not None:
            ev[2].record(stream)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    codec.encode_batch_dev(base, rs, bs, base + k * rs, rs, bs, S, nb, sh)
    enc_kernel = codec.last_kernel()
    codec.reconstruct_batch_dev(base, rs, bs, S, nb, present, data_only, sh)
    rec_kernel = codec.last_kernel()
    torch.cuda.synchronize()

    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(a.steps)]
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(events[i])
    torch.cuda.synchronize()
    barrier(world)
    el = time.perf_counter() - t0
    el_max = max_over_ranks(el, world)

    enc_ms = sum(e[0].elapsed_time(e[1]) for e in events) / a.steps
    rec_ms = sum(e[1].elapsed_time(e[2]) for e in events) / a.steps
    r = len([i for i in lost if i < k or not data_only])
    enc_bytes = nb * (k + m) * S
    rec_bytes = nb * (k + r) * S
    enc_gbs = enc_bytes / (enc_ms * 1e-3) / 1e9
    rec_gbs = rec_bytes / (rec_ms * 1e-3) / 1e9

    total_payload = nb * B * a.steps * world
    value = total_payload / el_max / 2**30
    ms_per_step = el_max * 1e3 / a.steps

    traffic = load_traffic(enc_kernel)
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (uniform random bytes, torch.randint in HBM)",
        "config": {
            "workload": f"RS({k},{m}) encode + ReconstructData of lost shard(s) {lost}, {a.block_kib} KiB blocks "
                        f"(BASELINE configs[2])",
            "blocks_per_gpu": nb,
            "block_bytes": B,
            "shard_bytes": S,
            "row_pitch": rs,
            "parallelism": f"independent blocks, {world} GPU(s), no collective",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(enc_gbs, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(enc_gbs / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "kernel": enc_kernel,
            "algorithmic_bytes_per_launch": enc_bytes,
            "avg_launch_ms": round(enc_ms, 4),
        },
        "reconstruct": {
            "kernel": rec_kernel,
            "achieved_GBs": round(rec_gbs, 1),
            "frac": round(rec_gbs / HBM_PEAK_GBS, 4),
            "algorithmic_bytes_per_launch": rec_bytes,
            "avg_launch_ms": round(rec_ms, 4),
        },
        "cpu_baseline": None,
    }
    if a.copy_inclusive:
        out["copy_inclusive"] = copy_inclusive(codec, k, m, S, min(nb, 1024), lost, data_only)
    if rank == 0 and world == 1 and a.cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline(k, m, B, lost, a.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    codec.close()
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


def copy_inclusive(codec, k, m, S, nb, lost, data_only):
    """Host-resident encode+reconstruct through pinned buffers (H2D/compute/D2H overlapped)."""
    import ctypes

    L = rsmi.lib()
    n = k + m
    din = L.rsmi_host_alloc(nb * k * S)
    dpar = L.rsmi_host_alloc(nb * m * S)
    dsh = L.rsmi_host_alloc(nb * n * S)
    arr = np.ctypeslib.as_array((ctypes.c_uint8 * (nb * k * S)).from_address(din))
    arr[:] = np.random.default_rng(3).integers(0, 256, size=arr.shape, dtype=np.uint8)
    present = [i not in lost for i in range(n)]
    codec.encode_batch_host_ptr(din, k * S, dpar, m * S, S, nb)
    codec.reconstruct_batch_host_ptr(dsh, n * S, S, nb, present, data_only)
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        codec.encode_batch_host_ptr(din, k * S, dpar, m * S, S, nb)
    t1 = time.perf_counter()
    for _ in range(reps):
        codec.reconstruct_batch_host_ptr(dsh, n * S, S, nb, present, data_only)
    t2 = time.perf_counter()
    B = k * S
    res = {
        "encode_GiBs": round(reps * nb * B / (t1 - t0) / 2**30, 2),
        "reconstruct_GiBs": round(reps * nb * B / (t2 - t1) / 2**30, 2),
        "enc_plus_rec_GiBs": round(reps * nb * B / (t2 - t0) / 2**30, 2),
        "blocks": nb,
    }
    for p in (din, dpar, dsh):
        L.rsmi_host_free(p)
    return res


if __name__ == "__main__":
    main()
