#!/usr/bin/env python3
"""Diagnostic: the unaligned-window (UA) kernels on the Split layout itself (rows back to
back at pitch S, odd for RS(10,4)) against the aligned kernels on the recommended pitch,
device-resident, interleaved rounds, medians."""
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))
import rsmi  # noqa: E402


def main():
    st = torch.cuda.current_stream()
    sh = st.cuda_stream
    V = {}
    keep = []
    for k, m, B, nb in ((10, 4, 262144, 4096), (10, 4, 1 << 20, 1024), (4, 2, 262144, 4096)):
        n = k + m
        S = (B + k - 1) // k
        c = rsmi.Codec(k, m)
        keep.append(c)
        present = [i != 0 for i in range(n)]
        for name, p in (("pitched", rsmi.recommended_pitch(S)), ("split", S)):
            buf = torch.randint(0, 256, (nb * n * p + 64,), dtype=torch.uint8, device="cuda")
            keep.append(buf)
            b = buf.data_ptr()
            V[f"RS({k},{m}) {B >> 10:5d}K {name:7s} encode"] = (
                lambda c=c, b=b, p=p, S=S, nb=nb, n=n, k=k: c.encode_batch_dev(b, p, n * p, b + k * p, p, n * p, S,
                                                                               nb, sh), nb * n * S, c)
            V[f"RS({k},{m}) {B >> 10:5d}K {name:7s} reconstruct"] = (
                lambda c=c, b=b, p=p, S=S, nb=nb, n=n, pr=present: c.reconstruct_batch_dev(b, p, n * p, S, nb, pr,
                                                                                           True, sh),
                nb * (k + 1) * S, c)
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:
        for f, _, _ in V.values():
            f()
        torch.cuda.synchronize()
    times = {x: [] for x in V}
    for _ in range(7):
        for name, (f, _, _) in V.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(3):
                f()
            e1.record(st)
            e1.synchronize()
            times[name].append(e0.elapsed_time(e1) / 3)
    for name, (f, nbytes, c) in V.items():
        f()
        torch.cuda.synchronize()
        med = statistics.median(times[name])
        print(f"{name:36s} {med * 1e3:8.1f} us {nbytes / med / 1e6:8.1f} GB/s  {c.last_kernel()}", flush=True)


if __name__ == "__main__":
    main()
