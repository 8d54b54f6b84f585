#!/usr/bin/env python3
"""Diagnostic: per-launch duration drift over a long run of the bench kernels."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))
import rsmi  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "both"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    k, m, nb, B = 10, 4, 4096, 256 * 1024
    n = k + m
    S = (B + k - 1) // k
    rs = rsmi.recommended_pitch(S)
    buf = torch.randint(0, 256, (nb, n, rs), dtype=torch.uint8, device="cuda")
    base = buf.data_ptr()
    c = rsmi.Codec(k, m)
    st = torch.cuda.current_stream()
    sh = st.cuda_stream
    present = [i != 0 for i in range(n)]
    evs = []
    for i in range(iters):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record(st)
        if mode in ("both", "enc"):
            c.encode_batch_dev(base, rs, n * rs, base + k * rs, rs, n * rs, S, nb, sh)
        e1.record(st)
        if mode in ("both", "rec"):
            c.reconstruct_batch_dev(base, rs, n * rs, S, nb, present, True, sh)
        e2.record(st)
        evs.append((e0, e1, e2))
    torch.cuda.synchronize()
    enc = [a.elapsed_time(b) for a, b, _ in evs]
    rec = [b.elapsed_time(c2) for _, b, c2 in evs]
    for lo in range(0, iters, max(1, iters // 10)):
        hi = min(iters, lo + max(1, iters // 10))
        print(f"iters {lo:4d}-{hi:4d}: enc {sum(enc[lo:hi]) / (hi - lo):.4f} ms  rec {sum(rec[lo:hi]) / (hi - lo):.4f} ms")


if __name__ == "__main__":
    main()
