#!/usr/bin/env python3
"""Diagnostic: RS(10,4) over 1 MiB blocks (S = 104858): XOR ceiling by row pitch and tile
order (tools/membw.hip membw_rows2) beside the real encode at the same pitch."""
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
    L.membw_rows2_launch.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                           ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                                           ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
    st = torch.cuda.current_stream()
    sh = st.cuda_stream
    k, m, n = 10, 4, 14
    S = int(os.environ.get("S", "104858"))
    nb = int(os.environ.get("NB", "1024"))
    pitches = [int(x) for x in os.environ.get("PITCHES", "106496,110592,114688,122880,131072,139264,147456,"
                                                         "163840,180224,196608,229376,262144").split(",")]
    buf = torch.randint(0, 256, (nb * n * max(pitches) + (1 << 20),), dtype=torch.uint8, device="cuda")
    b = buf.data_ptr()
    c = rsmi.Codec(k, m)
    enc = nb * n * S
    V = {}
    for p in pitches:
        for order in (0, 1, 2):
            V[f"p={p} xor ord={order}"] = (lambda p=p, o=order: L.membw_rows2_launch(
                k, m, 1, o, b, b + k * p, n * p, p, n * p, S, nb, 2048, sh), enc)
        V[f"p={p} encode"] = (lambda p=p: c.encode_batch_dev(b, p, n * p, b + k * p, p, n * p, S, nb, sh), enc)
    t_end = time.perf_counter() + 0.3  # settle past the start-up transient
    while time.perf_counter() < t_end:
        for f, _ in V.values():
            f()
        torch.cuda.synchronize()
    times = {x: [] for x in V}
    for r in range(5):
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
        print(f"S={S} {name:28s} {med:8.4f} ms {nbytes / med / 1e6:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
