#!/usr/bin/env python3
"""Diagnostic A/B: host batch calls (pinned rsmi_host_alloc buffers) with the zero-copy
write-back on and off, over the BASELINE shapes.  GiB/s of block payload."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))
import torch  # noqa: E402,F401
import rsmi  # noqa: E402

CASES = [(10, 4, 256, 2048, [0]), (4, 2, 256, 2048, [0]), (16, 4, 4096, 128, [0, 9]), (10, 4, 1024, 512, [0]),
         (2, 1, 256, 2048, [1])]


def main():
    L = rsmi.lib()
    for k, m, kib, nb, lost in CASES:
        n = k + m
        B = kib * 1024
        S = (B + k - 1) // k
        din, dpar, dsh = L.rsmi_host_alloc(nb * k * S), L.rsmi_host_alloc(nb * m * S), L.rsmi_host_alloc(nb * n * S)
        arr = np.ctypeslib.as_array((ctypes.c_uint8 * (nb * n * S)).from_address(dsh))
        arr[:] = np.random.default_rng(3).integers(0, 256, size=arr.shape, dtype=np.uint8)
        ctypes.memmove(din, dsh, nb * k * S)
        present = [i not in lost for i in range(n)]
        c = rsmi.Codec(k, m)
        res = {}
        # zero_copy 0/1/2 on the copy-engine pipeline; "direct" = one zero-copy UA kernel for
        # the whole call (small_call_bytes above the batch size)
        modes = (0, 1, 2, "direct")
        for zc in modes + modes:
            if zc == "direct":
                c.set_option("zero_copy", 1)
                c.set_option("small_call_bytes", 1 << 40)
            else:
                c.set_option("small_call_bytes", 0)
                c.set_option("zero_copy", zc)
            c.encode_batch_host_ptr(din, k * S, dpar, m * S, S, nb)
            t0 = time.perf_counter()
            for _ in range(3):
                c.encode_batch_host_ptr(din, k * S, dpar, m * S, S, nb)
            t1 = time.perf_counter()
            for _ in range(3):
                c.reconstruct_batch_host_ptr(dsh, n * S, S, nb, present, True)
            t2 = time.perf_counter()
            res.setdefault(zc, []).append((3 * nb * B / (t1 - t0) / 2**30, 3 * nb * B / (t2 - t1) / 2**30))
        for zc, v in res.items():
            e = max(x[0] for x in v)
            r = max(x[1] for x in v)
            print(f"RS({k},{m}) {kib:5d} KiB S={S:7d} zero_copy={zc!s:6s}: encode {e:6.2f} GiB/s, "
                  f"reconstruct{lost} {r:6.2f} GiB/s", flush=True)
        c.close()
        for p in (din, dpar, dsh):
            L.rsmi_host_free(p)


if __name__ == "__main__":
    main()
