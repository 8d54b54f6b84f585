#!/usr/bin/env python3
"""Diagnostic: what the Split layout (rows back to back at odd pitch S) costs the coding
kernels' memory pattern, per access form (tools/membw.hip membw_split), next to the same
pattern at the recommended pitch (membw_rows) and the real kernels (rsmi).  RS(10,4)
256 KiB and 1 MiB blocks.  GB/s of algorithmic bytes (K + M rows of S per block)."""
import ctypes
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))
import rsmi  # noqa: E402

L = ctypes.CDLL(os.path.join(ROOT, "tools", "build", "libmembw.so"))


def timeit(f, reps=20):
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
    return statistics.median(ts) * 1e-3


def main():
    st = torch.cuda.current_stream().cuda_stream
    x = torch.empty(1 << 28, dtype=torch.uint8, device="cuda")
    for _ in range(200):  # past the start-up clock transient (profiles/r01/README.md)
        x.add_(1)
    torch.cuda.synchronize()
    del x
    for B, nb in ((262144, 4096), (1 << 20, 1024)):
        k, m = 10, 4
        n = k + m
        S = (B + k - 1) // k
        p = rsmi.recommended_pitch(S)
        buf = torch.randint(0, 256, (nb * n * p + 4096,), dtype=torch.uint8, device="cuda")
        b = buf.data_ptr()
        for K, M in ((10, 4), (10, 1)):
            byt = nb * (K + M) * S
            res = {}
            el = timeit(lambda: L.membw_rows_launch(K, M, 1, ctypes.c_void_p(b), ctypes.c_void_p(b + K * p),
                                                    ctypes.c_uint64(n * p), ctypes.c_uint64(p), ctypes.c_uint64(n * p),
                                                    ctypes.c_uint32(S), ctypes.c_uint64(nb), (nb * ((S + 1023) // 1024) + 3) // 4,
                                                    ctypes.c_void_p(st)))
            res["pitched XOR"] = byt / el / 1e9
            for mode, name in ((0, "split UA ld+st"), (1, "split aligned ld+st"), (2, "split UA ld, al st"),
                               (3, "split al ld, UA st")):
                el = timeit(lambda: L.membw_split_launch(K, M, mode, ctypes.c_void_p(b + 3), ctypes.c_void_p(b + 3 + K * S),
                                                         ctypes.c_uint64(n * S), ctypes.c_uint64(S), ctypes.c_uint64(n * S),
                                                         ctypes.c_uint32(S), ctypes.c_uint64(nb), ctypes.c_void_p(st)))
                res[name] = byt / el / 1e9
            for order in range(5):
                el = timeit(lambda: L.membw_split_order_launch(K, M, order, ctypes.c_void_p(b + 3), ctypes.c_void_p(b + 3 + K * S),
                                                               ctypes.c_uint64(n * S), ctypes.c_uint64(S), ctypes.c_uint64(n * S),
                                                               ctypes.c_uint32(S), ctypes.c_uint64(nb), ctypes.c_void_p(st)))
                res[f"split order {order}"] = byt / el / 1e9
            # the same XOR pattern at other row pitches (16-B aligned): which pitches are slow
            for pp in (S + 16 - S % 16, (S + 255) // 256 * 256, (S + 4095) // 4096 * 4096, p):
                el = timeit(lambda: L.membw_split_launch(K, M, 1, ctypes.c_void_p(b), ctypes.c_void_p(b + K * pp),
                                                         ctypes.c_uint64(n * pp), ctypes.c_uint64(pp), ctypes.c_uint64(n * pp),
                                                         ctypes.c_uint32(S), ctypes.c_uint64(nb), ctypes.c_void_p(st)))
                res[f"pitch {pp}"] = byt / el / 1e9
            c = rsmi.Codec(k, m)
            if M == 4:
                f_p = lambda: c.encode_batch_dev(b, p, n * p, b + k * p, p, n * p, S, nb, st)
                f_s = lambda: c.encode_batch_dev(b + 3, S, n * S, b + 3 + k * S, S, n * S, S, nb, st)
            else:
                pres = [i != 0 for i in range(n)]
                f_p = lambda: c.reconstruct_batch_dev(b, p, n * p, S, nb, pres, True, st)
                f_s = lambda: c.reconstruct_batch_dev(b + 3, S, n * S, S, nb, pres, True, st)
            res["kernel pitched"] = byt / timeit(f_p) / 1e9
            res["kernel split"] = byt / timeit(f_s) / 1e9
            c.close()
            print(f"B={B} K={K} M={M}: " + ", ".join(f"{x} {v:.0f}" for x, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
