#!/usr/bin/env python3
"""Diagnostic: grid size of the CRC rows kernels (rsmi option waves_per_cu; 0 = persistent,
occupancy x CUs) on the bench layout, interleaved rounds, medians."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))
import rsmi  # noqa: E402


def main():
    st = torch.cuda.current_stream()
    k, m, nb = 10, 4, 4096
    n, S = k + m, 26215
    p = rsmi.recommended_pitch(S)
    buf = torch.randint(0, 256, (nb, n, p), dtype=torch.uint8, device="cuda")
    out = torch.empty((nb, n), dtype=torch.int32, device="cuda")
    V = {}
    ref = {}
    for wpc in (0, 96, 128, 192, 256, 384):
        c = rsmi.Codec(k, m)
        c.set_option("waves_per_cu", wpc)
        for kind in ("crc16", "crc32"):
            f = getattr(c, kind + "_rows_dev")
            V[f"{kind} waves_per_cu={wpc}"] = (lambda f=f: f(buf.data_ptr(), p, n * p, n, S, nb, out.data_ptr(), n,
                                                             st.cuda_stream))
            V[f"{kind} waves_per_cu={wpc}"]()
            torch.cuda.synchronize()
            r = out.clone()
            assert kind not in ref or torch.equal(ref[kind], r), kind
            ref[kind] = r
    times = {x: [] for x in V}
    for _ in range(9):
        for name, f in V.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(3):
                f()
            e1.record(st)
            e1.synchronize()
            times[name].append(e0.elapsed_time(e1) / 3)
    for name in V:
        med = statistics.median(times[name])
        print(f"{name:32s} {med * 1e3:8.1f} us {nb * n * S / med / 1e6:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
