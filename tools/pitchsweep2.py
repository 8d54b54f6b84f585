#!/usr/bin/env python3
"""Diagnostic: XOR-ceiling and encode throughput vs row pitch (full grids: one tile per wave)."""
import ctypes
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))
from sweep import membw  # noqa: E402
import rsmi  # noqa: E402


def run(k, m, S, nb, pitches, L, sh, rounds=3):
    n = k + m
    maxp = max(pitches)
    buf = torch.randint(0, 256, (nb * n * maxp + (1 << 20),), dtype=torch.uint8, device="cuda")
    b = buf.data_ptr()
    c = rsmi.Codec(k, m)
    enc = nb * n * S
    V = {}
    for p in pitches:
        if (k, m) in ((10, 4), (16, 4)):
            g = (nb * ((S + 1023) // 1024) + 3) // 4  # full grid (one tile per wave), as the encode launches
            V[f"K{k} xor p={p}"] = (lambda p=p, g=g: L.membw_rows_launch(k, m, 1, b, b + k * p, n * p, p, n * p, S, nb, g, sh), enc)
        V[f"K{k} enc p={p}"] = (lambda p=p: c.encode_batch_dev(b, p, n * p, b + k * p, p, n * p, S, nb, sh), enc)
    times = {x: [] for x in V}
    for f, _ in V.values():
        f()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    for r in range(rounds):
        for name, (f, _) in V.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(3):
                f()
            e1.record(st)
            e1.synchronize()
            times[name].append(e0.elapsed_time(e1) / 3)
    for name, (_, nbytes) in V.items():
        med = statistics.median(times[name])
        print(f"S={S:7d} {name:28s} {med:8.4f} ms {nbytes / med / 1e6:8.1f} GB/s", flush=True)
    del buf


def main():
    L = membw()
    L.membw_rows_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                    ctypes.c_int, ctypes.c_void_p]
    sh = torch.cuda.current_stream().cuda_stream
    K = 1024
    run(10, 4, 104858, 1024, [104864, 105472, 106496, 110592, 114688, 122880, 131072, 147456], L, sh)
    run(16, 4, 262144, 256, [262144, 262400, 266240, 270336, 294912], L, sh)
    run(10, 4, 26215, 4096, [26224, 26368, 26624, 27648, 28672, 32768, 36864], L, sh)


if __name__ == "__main__":
    main()
