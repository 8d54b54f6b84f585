#!/usr/bin/env python3
"""Diagnostic: banded tile order (tools/membw.hip membw_rows_band) on the RS(10,4) XOR ceiling,
1 MiB blocks (S = 104858) against 256 KiB blocks (S = 26215): band width G (tiles of every
block run together) x row pitch, beside the real encode at each pitch.  Interleaved rounds,
medians."""
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
    L.membw_rows_band_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                     ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                     ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
    st = torch.cuda.current_stream()
    sh = st.cuda_stream
    k, m, n = 10, 4, 14
    cases = []
    for S, nb, pitches, Gs in ((104858, 1024, (106496, 131072, 139264), (0, 52, 26, 13, 8, 4)),
                               (26215, 4096, (26624, 32768), (0, 13, 8, 4))):
        for p in pitches:
            cases.append((S, nb, p, Gs))
    maxbytes = max(nb * n * p for S, nb, p, _ in cases)
    buf = torch.randint(0, 256, (maxbytes + (1 << 20),), dtype=torch.uint8, device="cuda")
    b = buf.data_ptr()
    c = rsmi.Codec(k, m)
    V = {}
    for S, nb, p, Gs in cases:
        enc = nb * n * S
        for G in Gs:
            V[f"S={S} p={p} xor G={G or 'all'}"] = (lambda S=S, nb=nb, p=p, G=G: L.membw_rows_band_launch(
                k, m, b, b + k * p, n * p, p, n * p, S, nb, G, 2048, sh), enc)
        V[f"S={S} p={p} encode"] = (lambda S=S, nb=nb, p=p: c.encode_batch_dev(b, p, n * p, b + k * p, p, n * p, S,
                                                                                nb, sh), enc)
    t_end = time.perf_counter() + 0.3
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
        print(f"{name:36s} {med:8.4f} ms {nbytes / med / 1e6:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
