#!/usr/bin/env python3
"""Diagnostic: device layout A/B for the bench workload (RS(10,4), 4096 x 256 KiB), one tile
per wave: block-major [block][row][pitch] (bench.py) against shard-major [row][block][pitch],
encode and 1-row ReconstructData alternating as in the bench step, medians."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))
import rsmi  # noqa: E402


def main():
    k, m, nb = 10, 4, 4096
    n, S = k + m, 26215
    sh = torch.cuda.current_stream().cuda_stream
    st = torch.cuda.current_stream()
    present = [i != 0 for i in range(n)]
    V = {}
    for p in (32768, 26624):
        for layout in ("block-major", "shard-major"):
            buf = torch.randint(0, 256, (nb * n * p,), dtype=torch.uint8, device="cuda")
            b = buf.data_ptr()
            rs, bs = (p, n * p) if layout == "block-major" else (nb * p, p)
            c = rsmi.Codec(k, m)
            V[(layout, p)] = (buf, c, lambda c=c, b=b, rs=rs, bs=bs: c.encode_batch_dev(b, rs, bs, b + k * rs, rs, bs,
                                                                                         S, nb, sh),
                              lambda c=c, b=b, rs=rs, bs=bs: c.reconstruct_batch_dev(b, rs, bs, S, nb, present, True, sh))
    for _, _, e, r in V.values():
        e()
        r()
    torch.cuda.synchronize()
    te = {x: [] for x in V}
    tr = {x: [] for x in V}
    for _ in range(9):
        for key, (_, _, e, r) in V.items():
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record(st)
            for _ in range(3):
                e()
            ev[1].record(st)
            for _ in range(3):
                r()
            ev[2].record(st)
            ev[2].synchronize()
            te[key].append(ev[0].elapsed_time(ev[1]) / 3)
            tr[key].append(ev[1].elapsed_time(ev[2]) / 3)
    for key in V:
        e, r = statistics.median(te[key]), statistics.median(tr[key])
        print(f"{key[0]:12s} pitch {key[1]:6d}: encode {e * 1e3:7.1f} us {nb * n * S / e / 1e6:7.1f} GB/s   "
              f"reconstruct {r * 1e3:7.1f} us {nb * (k + 1) * S / r / 1e6:7.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
