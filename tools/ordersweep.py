#!/usr/bin/env python3
"""Diagnostic: XOR-ceiling throughput vs tile width and tile->wave order (RS(10,4) pattern)."""
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
    L.membw_rows2_launch.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                           ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                                           ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
    st = torch.cuda.current_stream()
    sh = st.cuda_stream
    k, n, nb, S = 10, 14, 4096, 26215
    buf = torch.randint(0, 256, (nb * n * 32768 + (1 << 20),), dtype=torch.uint8, device="cuda")
    b = buf.data_ptr()
    V = {}
    for p in (32768, 26624):
        for M in (4, 1):
            nbytes = nb * (k + M) * S
            for W in (1, 2, 4):
                for order in (0, 1, 2):
                    for grid in (1024, 2048):
                        V[f"p={p} M={M} W={W} ord={order} g={grid}"] = (
                            lambda p=p, M=M, W=W, o=order, g=grid: L.membw_rows2_launch(
                                k, M, W, o, b, b + k * p, n * p, p, n * p, S, nb, g, sh), nbytes)
    times = {x: [] for x in V}
    for f, _ in V.values():
        assert f() == 0
    torch.cuda.synchronize()
    for r in range(3):
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
        print(f"{name:36s} {med:8.4f} ms {nbytes / med / 1e6:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
