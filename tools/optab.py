#!/usr/bin/env python3
"""Diagnostic A/B of one rsmi_set_option knob on the bench layout (RS(10,4) 256 KiB, 4096
blocks, 32 KiB pitch): encode and 1-row ReconstructData, interleaved rounds, medians; the
variants' outputs are compared byte for byte first.  usage: optab.py KEY V0 V1 [V2 ...]"""
import statistics
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))
import rsmi  # noqa: E402


def main():
    key, vals = sys.argv[1], [int(v) for v in sys.argv[2:]]
    k, m, n, nb = 10, 4, 14, int(os.environ.get("NB", "4096"))
    B = int(os.environ.get("B", "262144"))
    S = (B + k - 1) // k
    p = rsmi.recommended_pitch(S)
    st = torch.cuda.current_stream()
    sh = st.cuda_stream
    buf = torch.randint(0, 256, (nb, n, p), dtype=torch.uint8, device="cuda")
    base = buf.data_ptr()
    present = [i != 0 for i in range(n)]
    cs = {}
    ref = None
    orig = buf.clone()
    for v in vals:
        c = rsmi.Codec(k, m)
        c.set_option(key, v)
        cs[v] = c
        buf.copy_(orig)
        c.encode_batch_dev(base, p, n * p, base + k * p, p, n * p, S, nb, sh)
        torch.cuda.synchronize()
        row0 = buf[:, 0, :S].clone()
        buf[:, 0, :] = 0
        c.reconstruct_batch_dev(base, p, n * p, S, nb, present, True, sh)
        torch.cuda.synchronize()
        assert torch.equal(buf[:, 0, :S], row0), f"{key}={v}: reconstruct differs from the data"
        out = buf[:, :, :S].clone()
        if ref is None:
            ref = out
        else:
            assert torch.equal(out, ref), f"{key}={v} output differs"
    V = {}
    for v, c in cs.items():
        V[f"{key}={v} encode"] = (lambda c=c: c.encode_batch_dev(base, p, n * p, base + k * p, p, n * p, S, nb, sh),
                                  nb * n * S)
        V[f"{key}={v} reconstruct"] = (lambda c=c: c.reconstruct_batch_dev(base, p, n * p, S, nb, present, True, sh),
                                       nb * (k + 1) * S)
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:
        for f, _ in V.values():
            f()
        torch.cuda.synchronize()
    times = {x: [] for x in V}
    for _ in range(9):
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
        print(f"B={B} {name:28s} {med * 1e3:8.1f} us {nbytes / med / 1e6:8.1f} GB/s  "
              f"{[round(t * 1e3, 1) for t in sorted(times[name])][:3]}", flush=True)
    for v, c in cs.items():
        c.encode_batch_dev(base, p, n * p, base + k * p, p, n * p, S, nb, sh)
        print(key, v, c.last_kernel())


if __name__ == "__main__":
    main()
