#!/usr/bin/env python3
"""Diagnostic: encode vs XOR-pattern ceiling on random vs zero data, several row pitches."""
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


def main():
    L = membw()
    L.membw_rows_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                    ctypes.c_int, ctypes.c_void_p]
    stream = torch.cuda.Stream()
    sh = stream.cuda_stream
    k, m, n, nb, S = 10, 4, 14, 4096, 26215
    rnd = torch.randint(0, 256, (nb * n * 32768,), dtype=torch.uint8, device="cuda")
    zero = torch.zeros(nb * n * 32768, dtype=torch.uint8, device="cuda")
    c = rsmi.Codec(k, m)
    c.set_option("nontemporal", 1)
    enc = nb * n * S
    V = {}
    for dname, buf in (("rand", rnd), ("zero", zero)):
        base = buf.data_ptr()
        for p in (26368, 27648, 32768):
            V[f"xor10x4 NT=1 {dname} pitch={p}"] = (lambda b=base, p=p: L.membw_rows_launch(10, 4, 1, b, b + 10 * p, 14 * p, p, 14 * p, S, nb, 2048, sh), enc)
            for d in (1, 2):
                def f(b=base, p=p, d=d):
                    c.set_option("chunks_per_lane", d)
                    c.encode_batch_dev(b, p, n * p, b + k * p, p, n * p, S, nb, sh)
                V[f"enc D={d} NT=1 {dname} pitch={p}"] = (f, enc)
    times = {x: [] for x in V}
    with torch.cuda.stream(stream):
        for f, _ in V.values():
            f()
        torch.cuda.synchronize()
        for r in range(7):
            for name, (f, _) in V.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(4):
                    f()
                e1.record(stream)
                e1.synchronize()
                times[name].append(e0.elapsed_time(e1) / 4)
    for name, (_, nbytes) in V.items():
        med = statistics.median(times[name])
        print(f"{name:40s} {med:8.4f} ms {nbytes / med / 1e6:8.1f} GB/s")


if __name__ == "__main__":
    main()
