#!/usr/bin/env python3
"""Diagnostic: the bench step (RS(10,4) encode then 1-row ReconstructData of 4096 x 256 KiB)
sequential on one stream, against the same blocks split in halves on two streams so one
half's encode overlaps the other half's reconstruct.  Medians over interleaved rounds."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))
import rsmi  # noqa: E402


def main():
    k, m, nb = 10, 4, 4096
    n, S, p = k + m, 26215, 32768
    present = [i != 0 for i in range(n)]
    buf = torch.randint(0, 256, (nb * n * p,), dtype=torch.uint8, device="cuda")
    b = buf.data_ptr()
    c = rsmi.Codec(k, m)
    s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()

    def enc(base, cnt, st):
        c.encode_batch_dev(base, p, n * p, base + k * p, p, n * p, S, cnt, st.cuda_stream)

    def rec(base, cnt, st):
        c.reconstruct_batch_dev(base, p, n * p, S, cnt, present, True, st.cuda_stream)

    def seq():
        enc(b, nb, s0)
        rec(b, nb, s0)

    half = nb // 2
    hb = b + half * n * p

    def ovl():
        enc(b, half, s0)
        enc(hb, half, s1)
        rec(b, half, s0)
        rec(hb, half, s1)

    V = {"sequential": seq, "two streams": ovl}
    for f in V.values():
        f()
    torch.cuda.synchronize()
    t = {x: [] for x in V}
    import time
    for _ in range(15):
        for name, f in V.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                f()
            torch.cuda.synchronize()
            t[name].append((time.perf_counter() - t0) / 10)
    for name in V:
        med = statistics.median(t[name])
        print(f"{name:12s} {med * 1e6:7.1f} us/step  {nb * 262144 / med / 2**30:7.1f} GiB/s payload", flush=True)


if __name__ == "__main__":
    main()
