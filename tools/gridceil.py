#!/usr/bin/env python3
"""Diagnostic: the memory ceilings of DESIGN.md section 4 re-measured with full grids (one
work unit per wave, hardware dispatch) next to the persistent grids they were first measured
with -- float4 copy, the RS(10,4) encode pattern (10 row reads XOR-ed into 4 row writes),
its reads alone and its writes alone.  Interleaved rounds, medians."""
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
    L.membw_half_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                    ctypes.c_int, ctypes.c_void_p]
    L.membw_pol_launch.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                         ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                                         ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
    st = torch.cuda.current_stream()
    sh = st.cuda_stream
    k, m, n, nb, S, p = 10, 4, 14, 4096, 26215, 32768
    tiles = nb * ((S + 15) // 16 + 63) // 64
    cb = 1 << 30
    cin = torch.empty(cb, dtype=torch.uint8, device="cuda")
    cout = torch.empty(cb, dtype=torch.uint8, device="cuda")
    big = torch.randint(0, 256, (nb * n * p,), dtype=torch.uint8, device="cuda")
    b = big.data_ptr()
    full_copy = cb // 16 // 256
    V = {}
    for g in (2048, 8192, full_copy):
        V[f"copy float4 nt grid={g}"] = (lambda g=g: L.membw_copy_launch(1, 1, cin.data_ptr(), cout.data_ptr(), cb, g, sh),
                                         2 * cb)
    for g in (1024, 4096, (tiles + 3) // 4):
        V[f"rows 10r->4w nt grid={g}"] = (lambda g=g: L.membw_rows_launch(10, 4, 1, b, b + k * p, n * p, p, n * p, S, nb,
                                                                          g, sh), nb * n * S)
        V[f"reads alone 10r grid={g}"] = (lambda g=g: L.membw_half_launch(0, 10, 0, b, b, n * p, p, n * p, S, nb, g, sh),
                                          nb * k * S)
        V[f"writes alone 4w grid={g}"] = (lambda g=g: L.membw_half_launch(1, 0, 4, b, b + k * p, n * p, p, n * p, S, nb,
                                                                          g, sh), nb * m * S)
    g = (tiles + 3) // 4
    # the reconstruct's pattern: 10 rows read (nt), 1 row written (plain stores, the bench's policy)
    V[f"rows 10r->1w ntl plain-st grid={g}"] = (lambda: L.membw_pol_launch(10, 1, 1, 0, b + p, b, n * p, p, n * p, S, nb, g,
                                                                          sh), nb * (k + 1) * S)
    V["rows 10r->1w ntl plain-st grid=1024"] = (lambda: L.membw_pol_launch(10, 1, 1, 0, b + p, b, n * p, p, n * p, S, nb,
                                                                           1024, sh), nb * (k + 1) * S)
    for f, _ in V.values():
        f()
    torch.cuda.synchronize()
    times = {x: [] for x in V}
    for _ in range(7):
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
        print(f"{name:36s} {med * 1e3:8.1f} us {nbytes / med / 1e6:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
