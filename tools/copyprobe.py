#!/usr/bin/env python3
"""Diagnostic: hipMemcpy(2D)Async rates for pitched layouts (pinned host / device)."""
import ctypes
import time

import torch

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpy2DAsync.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                 ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
H2D, D2H, D2D = 1, 2, 3


def t(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    st = torch.cuda.current_stream().cuda_stream
    for S, pitch in ((26215, 32768), (104858, 106496), (262144, 262144), (26224, 32768), (26216, 32768)):
        rows = (1 << 30) // S // 4
        nbytes = rows * S
        host = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
        dev_lin = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        dev_p = torch.empty(rows * pitch, dtype=torch.uint8, device="cuda")
        r = {}
        r["h2d_1d"] = t(lambda: hip.hipMemcpyAsync(dev_lin.data_ptr(), host.data_ptr(), nbytes, H2D, st))
        r["h2d_2d"] = t(lambda: hip.hipMemcpy2DAsync(dev_p.data_ptr(), pitch, host.data_ptr(), S, S, rows, H2D, st))
        r["d2d_2d_in"] = t(lambda: hip.hipMemcpy2DAsync(dev_p.data_ptr(), pitch, dev_lin.data_ptr(), S, S, rows, D2D, st))
        r["d2d_2d_out"] = t(lambda: hip.hipMemcpy2DAsync(dev_lin.data_ptr(), S, dev_p.data_ptr(), pitch, S, rows, D2D, st))
        r["d2h_1d"] = t(lambda: hip.hipMemcpyAsync(host.data_ptr(), dev_lin.data_ptr(), nbytes, D2H, st))
        r["d2h_2d"] = t(lambda: hip.hipMemcpy2DAsync(host.data_ptr(), S, dev_p.data_ptr(), pitch, S, rows, D2H, st))
        print(f"S={S} pitch={pitch} MB={nbytes / 1e6:.0f}: " + "  ".join(f"{k} {nbytes / v / 1e9:.1f} GB/s" for k, v in r.items()), flush=True)


if __name__ == "__main__":
    main()
