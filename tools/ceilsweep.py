#!/usr/bin/env python3
"""Diagnostic: split the RS(10,4) rows-pattern ceiling into its read and write halves and
try LDS-DMA staging of the reads (tools/membw.hip kinds 0/1/2), beside the real kernels."""
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
    L.membw_half_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                    ctypes.c_int, ctypes.c_void_p]
    L.membw_pol_launch.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                                         ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int,
                                                         ctypes.c_void_p]
    sh = torch.cuda.current_stream().cuda_stream
    k, m, n, S, nb = 10, 4, 14, 26215, 4096
    p = int(os.environ.get("PITCH", "32768"))
    buf = torch.randint(0, 256, (nb * n * p + (1 << 20),), dtype=torch.uint8, device="cuda")
    b = buf.data_ptr()
    c = rsmi.Codec(k, m)
    present = [0] + [1] * 13
    V = {}
    for g in (1024, 2048, 4096):
        V[f"xor 10r4w g{g}"] = (lambda g=g: L.membw_rows_launch(10, 4, 1, b, b + k * p, n * p, p, n * p, S, nb, g, sh), nb * n * S)
        V[f"ro 10r g{g}"] = (lambda g=g: L.membw_half_launch(0, 10, 0, b, b, n * p, p, n * p, S, nb, g, sh), nb * k * S)
        V[f"wo 4w g{g}"] = (lambda g=g: L.membw_half_launch(1, 0, 4, b, b + k * p, n * p, p, n * p, S, nb, g, sh), nb * m * S)
    for g in (512, 1024, 2048):
        V[f"lds 10r4w g{g}"] = (lambda g=g: L.membw_half_launch(2, 10, 4, b, b + k * p, n * p, p, n * p, S, nb, g, sh), nb * n * S)
        V[f"lds 10r1w g{g}"] = (lambda g=g: L.membw_half_launch(2, 10, 1, b + p, b, n * p, p, n * p, S, nb, g, sh), nb * 11 * S)
    for ntl, nts in ((0, 0), (0, 1), (1, 0), (1, 1), (1, 2), (1, 3)):
        if True:
            V[f"pol 10r4w L{ntl}S{nts}"] = (lambda a=ntl, z=nts: L.membw_pol_launch(10, 4, a, z, b, b + k * p, n * p, p, n * p, S, nb, 2048, sh), nb * n * S)
            V[f"pol 10r1w L{ntl}S{nts}"] = (lambda a=ntl, z=nts: L.membw_pol_launch(10, 1, a, z, b + p, b, n * p, p, n * p, S, nb, 2048, sh), nb * 11 * S)
    V["xor 10r1w g2048"] = (lambda: L.membw_rows_launch(10, 1, 1, b + p, b, n * p, p, n * p, S, nb, 2048, sh), nb * 11 * S)
    V["encode"] = (lambda: c.encode_batch_dev(b, p, n * p, b + k * p, p, n * p, S, nb, sh), nb * n * S)
    V["reconstruct 1"] = (lambda: c.reconstruct_batch_dev(b, p, n * p, S, nb, present, True, sh), nb * 11 * S)
    for f, _ in V.values():
        r = f()
        assert r in (0, None), r
    torch.cuda.synchronize()
    times = {x: [] for x in V}
    st = torch.cuda.current_stream()
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
        print(f"p={p} {name:24s} {med:8.4f} ms {nbytes / med / 1e6:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
