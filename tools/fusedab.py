#!/usr/bin/env python3
"""Diagnostic A/B: the fused encode + CRC-16 (rsmi_encode_batch_dev_crc) next to the plain
encode, RS(10,4) 256 KiB x 4096, pitched (32 KiB) and Split layouts, in the library RSMI_LIB
names (tools/Makefile variants).  Median of 20 launches after a 300 ms settle."""
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))
import rsmi  # noqa: E402


def med(f, st, reps=40):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        f()
        e1.record(st)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return statistics.median(ts)


def main():
    # FUSED_SHAPE=k,m,blocks,block_bytes (default RS(10,4) 256 KiB x 4096)
    k, m, nb, B = (int(x) for x in os.environ.get("FUSED_SHAPE", "10,4,4096,262144").split(","))
    n, S = k + m, (B + k - 1) // k
    st = torch.cuda.current_stream()
    sh = st.cuda_stream
    c = rsmi.Codec(k, m)
    for kv in filter(None, os.environ.get("FUSED_OPT", "").split(",")):  # e.g. crc_parts=4
        key, val = kv.split("=")
        c.set_option(key, int(val))
    raw = torch.empty((nb, n), dtype=torch.int32, device="cuda")
    res = []
    for lay, rs in (("pitched", rsmi.recommended_pitch(S)), ("split", S)):
        buf = torch.randint(0, 256, (nb * n * rs + 64,), dtype=torch.uint8, device="cuda")
        b = buf.data_ptr()
        enc = lambda: c.encode_batch_dev(b, rs, n * rs, b + k * rs, rs, n * rs, S, nb, sh)
        fz = lambda: c.encode_batch_dev_crc(b, rs, n * rs, b + k * rs, rs, n * rs, S, nb, raw.data_ptr(), sh)
        t_end = time.perf_counter() + 0.3
        while time.perf_counter() < t_end:
            enc()
            fz()
            torch.cuda.synchronize()
        te, tf = med(enc, st), med(fz, st)
        res.append(f"{lay}: encode {te:.1f} us, fused {tf:.1f} us ({tf / te:.2f}x)")
        del buf
    tag = (os.path.basename(os.path.dirname(os.path.dirname(rsmi.LIB_PATH))) + f" RS({k},{m}) {B >> 10} KiB " +
           os.environ.get("FUSED_OPT", ""))
    print(tag + ": " + "; ".join(res), flush=True)


if __name__ == "__main__":
    main()
