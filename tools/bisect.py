#!/usr/bin/env python3
"""Diagnostic: feature bisection between the XOR ceiling and the encode kernel
(tools/membw.hip membw_rows3), RS(10,4) 256 KiB, 32 KiB pitch, beside the real kernels."""
import ctypes
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))
from sweep import membw  # noqa: E402
import rsmi  # noqa: E402


def main():
    L = membw()
    L.membw_rows3_launch.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                           ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                                           ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
    st = torch.cuda.current_stream()
    sh = st.cuda_stream
    k, m, n, S, nb, p = 10, 4, 14, 26215, 4096, 32768
    buf = torch.randint(0, 256, (nb * n * p + (1 << 20),), dtype=torch.uint8, device="cuda")
    b = buf.data_ptr()
    c = rsmi.Codec(k, m)
    present = [i != 0 for i in range(n)]
    V = {}
    for feat in range(8):
        for g in (1024, 2048):
            V[f"rows3 10r4w feat={feat} g={g}"] = (lambda f=feat, g=g: L.membw_rows3_launch(
                10, 4, f, b, b + k * p, n * p, p, n * p, S, nb, g, sh), nb * n * S)
        V[f"rows3 10r1w feat={feat} g=2048"] = (lambda f=feat: L.membw_rows3_launch(
            10, 1, f, b + p, b, n * p, p, n * p, S, nb, 2048, sh), nb * 11 * S)
    V["encode"] = (lambda: c.encode_batch_dev(b, p, n * p, b + k * p, p, n * p, S, nb, sh), nb * n * S)
    V["reconstruct 1"] = (lambda: c.reconstruct_batch_dev(b, p, n * p, S, nb, present, True, sh), nb * 11 * S)
    for f, _ in V.values():
        r = f()
        assert r in (0, None), r
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:
        for f, _ in V.values():
            f()
        torch.cuda.synchronize()
    times = {x: [] for x in V}
    for _ in range(5):
        for name, (f, _) in V.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(4):
                f()
            e1.record(st)
            e1.synchronize()
            times[name].append(e0.elapsed_time(e1) / 4)
    for name, (_, nbytes) in V.items():
        med = statistics.median(times[name])
        print(f"{name:32s} {med:8.4f} ms {nbytes / med / 1e6:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
