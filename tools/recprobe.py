#!/usr/bin/env python3
"""Diagnostic: the 1-row reconstruct's memory pattern (10 rows read nontemporal, 1 row written
with plain stores; tools/membw.hip membw_rows_pol, the GF math replaced by an XOR) with the
written row where ReconstructData writes it in the bench (row 0 of the same block, rows 1..10 read)
against a separate output buffer, next to its read-only and write-only halves and the real
reconstruct kernel.  RS(10,4) 256 KiB blocks x 4096 at the 32 KiB pitch.  Times in us."""
import ctypes
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))
import rsmi  # noqa: E402

L = ctypes.CDLL(os.path.join(ROOT, "tools", "build", "libmembw.so"))
U64, U32, VP = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p


def timeit(f, reps=30):
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    ts = []
    st = torch.cuda.current_stream()
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        f()
        e1.record(st)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts) * 1e3


def main():
    st = torch.cuda.current_stream().cuda_stream
    x = torch.empty(1 << 28, dtype=torch.uint8, device="cuda")
    for _ in range(200):  # past the start-up clock transient (profiles/r01/README.md)
        x.add_(1)
    torch.cuda.synchronize()
    del x
    k, m, B, nb = 10, 4, 262144, 4096
    n = k + m
    S = (B + k - 1) // k
    p = rsmi.recommended_pitch(S)
    buf = torch.randint(0, 256, (nb * n * p + 4096,), dtype=torch.uint8, device="cuda")
    sep = torch.zeros(nb * p + 4096, dtype=torch.uint8, device="cuda")
    b, o = buf.data_ptr(), sep.data_ptr()
    grid = (nb * ((S + 1023) // 1024) + 3) // 4
    alg = nb * 11 * S
    rows = {}
    for rep in range(3):
        cases = {
            "10r->1w, out = row 0 of the block (bench layout)": lambda: L.membw_pol_launch(
                10, 1, 1, 0, VP(b + p), VP(b), U64(n * p), U64(p), U64(n * p), U32(S), U64(nb), grid, VP(st)),
            "10r->1w, out = a separate buffer (pitch p per block)": lambda: L.membw_pol_launch(
                10, 1, 1, 0, VP(b + p), VP(o), U64(n * p), U64(p), U64(p), U32(S), U64(nb), grid, VP(st)),
            "10r->1w nt stores, out = row 0": lambda: L.membw_pol_launch(
                10, 1, 1, 1, VP(b + p), VP(b), U64(n * p), U64(p), U64(n * p), U32(S), U64(nb), grid, VP(st)),
            "10 rows read alone (rows 1..10)": lambda: L.membw_half_launch(
                0, 10, 0, VP(b + p), VP(o), U64(n * p), U64(p), U64(n * p), U32(S), U64(nb), grid, VP(st)),
            "1 row written alone (row 0, nt)": lambda: L.membw_half_launch(
                1, 0, 1, VP(b), VP(b), U64(n * p), U64(p), U64(n * p), U32(S), U64(nb), grid, VP(st)),
        }
        with rsmi.Codec(k, m) as c:
            present = [i != 0 for i in range(n)]
            cases["reconstruct kernel (rsmi_reconstruct_batch_dev, row 0)"] = lambda: c.reconstruct_batch_dev(
                b, p, n * p, S, nb, present, True, st)
            for name, f in cases.items():
                rows.setdefault(name, []).append(timeit(f))
    for name, ts in rows.items():
        t = statistics.median(ts)
        print(f"{name:58s} {t:7.1f} us  ({alg / t / 1e3:6.0f} GB/s of the 11-row bytes)  runs {', '.join(f'{x:.1f}' for x in ts)}")


if __name__ == "__main__":
    main()
