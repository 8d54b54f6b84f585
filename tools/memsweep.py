#!/usr/bin/env python3
"""Memory-ceiling sweep (diagnostic): copy and RS-pattern XOR kernels over layouts."""
import ctypes
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from sweep import membw  # noqa: E402


def main():
    L = membw()
    L.membw_copy_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                    ctypes.c_int, ctypes.c_void_p]
    L.membw_rows_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                    ctypes.c_int, ctypes.c_void_p]
    stream = torch.cuda.Stream()
    sh = stream.cuda_stream
    k, m, n, nb = 10, 4, 14, 4096
    S = 26215
    cb = 1 << 30
    cin = torch.empty(cb, dtype=torch.uint8, device="cuda")
    cout = torch.empty(cb, dtype=torch.uint8, device="cuda")
    big = torch.empty(nb * n * 32768 + (1 << 20), dtype=torch.uint8, device="cuda")
    base = big.data_ptr()
    V = {}
    for U in (1, 2, 4):
        for NT in (0, 1):
            for g in (256, 512, 1024, 2048):
                V[f"copy U={U} NT={NT} grid={g}"] = (lambda U=U, NT=NT, g=g: L.membw_copy_launch(U, NT, cin.data_ptr(), cout.data_ptr(), cb, g, sh), 2 * cb)
    enc = nb * n * S
    for pitch in (26368, 26624, 27648, 32768):
        for NT in (0, 1):
            for g in (1024, 4096):
                V[f"rows10x4 blockmajor pitch={pitch} NT={NT} grid={g}"] = (
                    lambda p=pitch, NT=NT, g=g: L.membw_rows_launch(10, 4, NT, base, base + 10 * p, 14 * p, p, 14 * p, S, nb, g, sh), enc)
    for pitch in (26368, 26624):
        for NT in (0, 1):
            g = 4096
            V[f"rows10x4 shardmajor pitch={pitch} NT={NT} grid={g}"] = (
                lambda p=pitch, NT=NT, g=g: L.membw_rows_launch(10, 4, NT, base, base + 10 * nb * p, p, nb * p, p, S, nb, g, sh), enc)
    for NT in (0, 1):
        V[f"rows1x1 (tile copy) NT={NT}"] = (lambda NT=NT: L.membw_rows_launch(1, 1, NT, base, base + 7 * nb * 26368, 26368, 26368, 26368, S, 7 * nb, 4096, sh), 2 * 7 * nb * S)
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
        print(f"{name:52s} {med:8.4f} ms {nbytes / med / 1e6:8.1f} GB/s")


if __name__ == "__main__":
    main()
