#!/usr/bin/env python3
"""Diagnostic: RS(10,4) XOR-pattern and encode throughput vs row pitch / block stride."""
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
    rnd = torch.randint(0, 256, (nb * n * 65536 + (1 << 20),), dtype=torch.uint8, device="cuda")
    b = rnd.data_ptr()
    c = rsmi.Codec(k, m)
    c.set_option("nontemporal", 1)
    enc = nb * n * S
    V = {}
    cases = [(p, n * p) for p in (26368, 26624, 28672, 30720, 32768, 33024, 34816, 36864, 40960, 49152, 65536)]
    cases += [(26368, n * 32768), (26368, n * 28672), (26368, 16 * 26368), (32768, n * 32768 + 4096),
              (26368, n * 26368 + 4096), (26368, n * 26368 + 65536)]
    for p, bs in cases:
        V[f"xor p={p} bs={bs}"] = (lambda p=p, bs=bs: L.membw_rows_launch(10, 4, 1, b, b + 10 * p, bs, p, bs, S, nb, 2048, sh), enc)
    for p, bs in [(26368, n * 26368), (32768, n * 32768), (26368, n * 32768), (28672, n * 28672), (36864, n * 36864)]:
        V[f"enc p={p} bs={bs}"] = (lambda p=p, bs=bs: c.encode_batch_dev(b, p, bs, b + k * p, p, bs, S, nb, sh), enc)
    times = {x: [] for x in V}
    with torch.cuda.stream(stream):
        for f, _ in V.values():
            f()
        torch.cuda.synchronize()
        for r in range(5):
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
