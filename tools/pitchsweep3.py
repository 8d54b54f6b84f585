#!/usr/bin/env python3
"""Diagnostic: encode throughput vs row pitch in 4 KiB steps (one tile per wave), for shard
sizes between the power-of-two cases, to find a pitch rule for rsmi_recommended_pitch."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))
import rsmi  # noqa: E402

TOTAL = 1 << 30  # shard bytes per launch, about the bench's


def run(k, m, S, pitches, sh):
    n = k + m
    nb = max(16, TOTAL // (n * S))
    buf = torch.randint(0, 256, (nb * n * max(pitches) + (1 << 20),), dtype=torch.uint8, device="cuda")
    b = buf.data_ptr()
    c = rsmi.Codec(k, m)
    V = {p: (lambda p=p: c.encode_batch_dev(b, p, n * p, b + k * p, p, n * p, S, nb, sh)) for p in pitches}
    for f in V.values():
        f()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    times = {p: [] for p in V}
    for _ in range(3):
        for p, f in V.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(3):
                f()
            e1.record(st)
            e1.synchronize()
            times[p].append(e0.elapsed_time(e1) / 3)
    res = {p: nb * n * S / statistics.median(t) / 1e6 for p, t in times.items()}
    best = max(res, key=res.get)
    line = " ".join(f"{p // 1024}K:{res[p]:.0f}" for p in pitches)
    print(f"RS({k},{m}) S={S} rec={rsmi.recommended_pitch(S) // 1024}K best={best // 1024}K ({res[best]:.0f})  {line}",
          flush=True)
    del buf


def main():
    sh = torch.cuda.current_stream().cuda_stream
    for k, m, S in ((10, 4, 104858), (10, 4, 52429), (10, 4, 78644), (10, 4, 157287), (10, 4, 209716),
                    (16, 4, 65537), (4, 2, 98304)):
        lo = (S + 4095) // 4096 * 4096
        pitches = list(range(lo, lo + S // 2 + 4096, 4096))
        pw = 1
        while pw < S:
            pw <<= 1
        if pw not in pitches:
            pitches.append(pw)
        run(k, m, S, pitches, sh)


if __name__ == "__main__":
    main()
