#!/usr/bin/env python3
"""Diagnostic A/B: cache policy (rsmi option "nontemporal" 1/2/3) per output width, over the
BASELINE shapes, interleaved in one process.  Feeds auto_cache_policy in rsmi_core.cpp."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))
import rsmi  # noqa: E402

# (k, m, block KiB, blocks, lost shards or None for encode)
CASES = [(10, 4, 256, 4096, None), (10, 4, 256, 4096, [0]), (10, 4, 256, 4096, [0, 1]),
         (10, 4, 256, 4096, [0, 1, 2]), (10, 4, 256, 4096, [0, 1, 2, 3]), (16, 4, 4096, 256, None),
         (16, 4, 4096, 256, [0, 9]), (4, 2, 256, 4096, None), (4, 2, 256, 4096, [0]), (2, 1, 256, 4096, None),
         (2, 1, 256, 4096, [1]), (10, 4, 1024, 1024, None)]


def main():
    sh = torch.cuda.current_stream().cuda_stream
    bufs, V = {}, {}
    for k, m, kib, nb, lost in CASES:
        n = k + m
        S = (kib * 1024 + k - 1) // k
        p = rsmi.recommended_pitch(S)
        key = (k, m, kib)
        if key not in bufs:
            bufs[key] = (torch.randint(0, 256, (nb * n * p,), dtype=torch.uint8, device="cuda"), rsmi.Codec(k, m))
        buf, c = bufs[key]
        b = buf.data_ptr()
        for nt in (1, 2, 3):
            if lost is None:
                f = (lambda c=c, b=b, p=p, n=n, k=k, S=S, nb=nb, nt=nt:
                     (c.set_option("nontemporal", nt), c.encode_batch_dev(b, p, n * p, b + k * p, p, n * p, S, nb, sh)))
                V[f"RS({k},{m}) {kib}K enc nt={nt}"] = (f, nb * n * S)
            else:
                present = [i not in lost for i in range(n)]
                f = (lambda c=c, b=b, p=p, n=n, S=S, nb=nb, nt=nt, present=present:
                     (c.set_option("nontemporal", nt), c.reconstruct_batch_dev(b, p, n * p, S, nb, present, True, sh)))
                V[f"RS({k},{m}) {kib}K rec{lost} nt={nt}"] = (f, nb * (k + len(lost)) * S)
    for f, _ in V.values():
        f()
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
        print(f"{name:36s} {med:8.4f} ms {nbytes / med / 1e6:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
