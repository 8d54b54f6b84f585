#!/usr/bin/env python3
"""Diagnostic A/B: prefetch depth / XOR pairing / occupancy for RS(10,4) at 32 KiB pitch."""
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

if os.environ.get("RSMI_LIB"):  # e.g. the RSMI_DIAG_NOMATH build from `make -C tools diag`
    rsmi.LIB_PATH = os.environ["RSMI_LIB"]


def main():
    L = membw()
    L.membw_rows_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                    ctypes.c_int, ctypes.c_void_p]
    stream = torch.cuda.Stream()
    sh = stream.cuda_stream
    k, m, n, nb, S = 10, 4, 14, 4096, 26215
    p = int(os.environ.get("PITCH", "32768"))
    buf = torch.randint(0, 256, (nb * n * p,), dtype=torch.uint8, device="cuda")
    b = buf.data_ptr()
    c = rsmi.Codec(k, m)
    c.set_option("nontemporal", 1)
    enc, rec = nb * n * S, nb * (k + 1) * S
    present = [i != 0 for i in range(n)]
    V = {}
    V["xor10x4"] = (lambda: L.membw_rows_launch(10, 4, 1, b, b + 10 * p, n * p, p, n * p, S, nb, 2048, sh), enc)
    V["xor10x1"] = (lambda: L.membw_rows_launch(10, 1, 1, b + p, b, n * p, p, n * p, S, nb, 2048, sh), rec)
    pfs = [int(x) for x in os.environ.get("PFS", "0,4,8,10,505,504").split(",")]
    wpcs = [int(x) for x in os.environ.get("WPCS", "0,12,16,24").split(",")]
    for pf in pfs:
        for wpc in wpcs:
            def fe(pf=pf, wpc=wpc):
                c.set_option("prefetch", pf)
                c.set_option("waves_per_cu", wpc)
                c.encode_batch_dev(b, p, n * p, b + k * p, p, n * p, S, nb, sh)
            V[f"enc pf={pf} wpc={wpc}"] = (fe, enc)
        def fr(pf=pf):
            c.set_option("prefetch", pf)
            c.set_option("waves_per_cu", 0)
            c.reconstruct_batch_dev(b, p, n * p, S, nb, present, True, sh)
        V[f"rec pf={pf}"] = (fr, rec)
    times = {x: [] for x in V}
    labels = {}
    with torch.cuda.stream(stream):
        for name, (f, _) in V.items():
            f()
            labels[name] = c.last_kernel()
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
        print(f"{name:24s} {med:8.4f} ms {nbytes / med / 1e6:8.1f} GB/s  {labels[name] if 'xor' not in name else ''}")


if __name__ == "__main__":
    main()
