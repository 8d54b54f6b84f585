#!/usr/bin/env python3
"""A/B sweep of RS kernel variants against memory ceilings, interleaved in one process.

Usage: python tools/sweep.py [--k 10 --m 4 --blocks 4096 --rounds 7]
Prints one line per variant: median ms per launch and algorithmic GB/s.
"""
import argparse
import ctypes
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))

import torch  # noqa: E402

import rsmi  # noqa: E402

MEMBW_SO = os.path.join(ROOT, "tools", "build", "libmembw.so")


def membw():
    if not os.path.exists(MEMBW_SO):
        os.makedirs(os.path.dirname(MEMBW_SO), exist_ok=True)
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                               os.path.join(ROOT, "tools", "membw.hip"), "-o", MEMBW_SO])
    L = ctypes.CDLL(MEMBW_SO)
    L.membw_copy_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
    L.membw_rows_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                    ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int,
                                    ctypes.c_void_p]
    return L


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--m", type=int, default=4)
    p.add_argument("--block-kib", type=int, default=256)
    p.add_argument("--blocks", type=int, default=4096)
    p.add_argument("--rounds", type=int, default=7)
    p.add_argument("--iters", type=int, default=5)
    a = p.parse_args()
    k, m, n = a.k, a.m, a.k + a.m
    B = a.block_kib * 1024
    S = (B + k - 1) // k
    rs = (S + 255) // 256 * 256
    nb = a.blocks
    buf = torch.randint(0, 256, (nb, n, rs), dtype=torch.uint8, device="cuda")
    base = buf.data_ptr()
    stream = torch.cuda.Stream()
    sh = stream.cuda_stream
    L = membw()
    copy_bytes = 1 << 30
    cin = torch.empty(copy_bytes, dtype=torch.uint8, device="cuda")
    cout = torch.empty(copy_bytes, dtype=torch.uint8, device="cuda")
    codec = rsmi.Codec(k, m)
    enc_bytes = nb * n * S
    rec_bytes = nb * (k + 1) * S
    present = [i != 0 for i in range(n)]

    variants = {}

    def add_enc(name, d, nt, wpc):
        def run():
            codec.set_option("chunks_per_lane", d)
            codec.set_option("nontemporal", nt)
            codec.set_option("waves_per_cu", wpc)
            codec.encode_batch_dev(base, rs, n * rs, base + k * rs, rs, n * rs, S, nb, sh)
        variants[name] = (run, enc_bytes)

    def add_rec(name, d, nt, wpc):
        def run():
            codec.set_option("chunks_per_lane", d)
            codec.set_option("nontemporal", nt)
            codec.set_option("waves_per_cu", wpc)
            codec.reconstruct_batch_dev(base, rs, n * rs, S, nb, present, True, sh)
        variants[name] = (run, rec_bytes)

    for d in (1, 2):
        for nt in (0, 1):
            for wpc in (0, 8, 32):
                add_enc(f"enc D={d} NT={nt} wpc={wpc}", d, nt, wpc)
    for d in (1, 2):
        for nt in (0, 1):
            add_rec(f"rec1 D={d} NT={nt}", d, nt, 0)
    for grid in (1024, 2048, 8192):
        variants[f"copy 1GiB grid={grid}"] = (
            lambda g=grid: L.membw_copy_launch(cin.data_ptr(), cout.data_ptr(), copy_bytes, g, sh), 2 * copy_bytes)
    for grid in (1024, 2048, 4096):
        variants[f"rows_xor K={k} M={m} grid={grid}"] = (
            lambda g=grid: L.membw_rows_launch(k, m, base, base + k * rs, n * rs, rs, n * rs, S, nb, g, sh), enc_bytes)
        variants[f"rows_xor K={k} M=1 grid={grid}"] = (
            lambda g=grid: L.membw_rows_launch(k, 1, base + rs, base, n * rs, rs, n * rs, S, nb, g, sh), rec_bytes)

    times = {name: [] for name in variants}
    with torch.cuda.stream(stream):
        for name, (fn, _) in variants.items():
            fn()
        torch.cuda.synchronize()
        for r in range(a.rounds):
            for name, (fn, _) in variants.items():
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.iters):
                    fn()
                e1.record(stream)
                e1.synchronize()
                times[name].append(e0.elapsed_time(e1) / a.iters)
    print(f"RS({k},{m}) B={B} S={S} blocks={nb}")
    for name, (_, nbytes) in variants.items():
        med = statistics.median(times[name])
        print(f"{name:40s} {med:8.4f} ms  {nbytes / med / 1e6:8.1f} GB/s  min {min(times[name]):.4f}")


if __name__ == "__main__":
    main()
