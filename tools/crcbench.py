#!/usr/bin/env python3
"""Diagnostic: rs_crc16_rows_kernel / rs_crc32_rows_kernel bandwidth (R(row) of every shard row,
the datanode entry checksum's and the mutcask value checksum's device halves) over the bench layout: 4096 RS(10,4) 256 KiB blocks, 14 rows of
S = 26215 at 32 KiB pitch; and 1 MiB / 4 MiB shapes.  Bytes counted: rows x S read."""
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))
import rsmi  # noqa: E402


# env CRC_WPC (rows-kernel grid cap in waves per CU; 0 = default)
FOLDS = ["crc16", "crc16nib", "crc32"]  # crc16: the default fold (matrix cores); crc16nib: nibble tables
WPC = int(os.environ.get("CRC_WPC", "0"))
SPLIT = os.environ.get("CRC_SPLIT", "0") == "1"  # rows back to back at pitch S (the unaligned passes)


def main():
    st = torch.cuda.current_stream()
    for k, m, B, nb in ((10, 4, 262144, 4096), (10, 4, 1 << 20, 1024), (16, 4, 4 << 20, 256)):
        n = k + m
        S = (B + k - 1) // k
        p = S if SPLIT else rsmi.recommended_pitch(S)
        buf = torch.randint(0, 256, (nb, n, p), dtype=torch.uint8, device="cuda")
        out = torch.empty((nb, n), dtype=torch.int32, device="cuda")
        for fold in FOLDS:
            c = rsmi.Codec(k, m)
            if WPC:
                c.set_option("waves_per_cu", WPC)
            if fold == "crc16nib":
                c.set_option("crc16_fold", 0)
            if fold == "crc32":
                f = lambda: c.crc32_rows_dev(buf.data_ptr(), p, n * p, n, S, nb, out.data_ptr(), n, st.cuda_stream)
            else:
                f = lambda: c.crc16_rows_dev(buf.data_ptr(), p, n * p, n, S, nb, out.data_ptr(), n, st.cuda_stream)
            t_end = time.perf_counter() + 0.2
            while time.perf_counter() < t_end:
                f()
                torch.cuda.synchronize()
            ts = []
            for _ in range(20):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                f()
                e1.record(st)
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            med = statistics.median(ts)
            print(f"RS({k},{m}) B={B} nb={nb} rows={nb * n} S={S} {dict(crc32='crc32 (mutcask)', crc16='crc16 (datanode, matrix cores)', crc16nib='crc16 (datanode, nibble tables)')[fold]}: "
                  f"{med * 1e3:8.1f} us  {nb * n * S / med / 1e6:8.1f} GB/s", flush=True)
            c.close()


def fused_vs_separate(k=10, m=4, B=262144, nb=4096):
    """The bench layout: encode then a separate R(row) pass, against the encode with the CRC
    fused (rsmi_encode_batch_dev_crc)."""
    st = torch.cuda.current_stream()
    n = k + m
    S = (B + k - 1) // k
    p = rsmi.recommended_pitch(S)
    buf = torch.randint(0, 256, (nb, n, p), dtype=torch.uint8, device="cuda")
    raw = torch.empty((nb, n), dtype=torch.int32, device="cuda")
    b = buf.data_ptr()
    c = rsmi.Codec(k, m)
    cn = rsmi.Codec(k, m)
    cn.set_option("crc16_fused_fold", 0)  # the nibble-table fused variant, for A/B
    if WPC:
        c.set_option("waves_per_cu", WPC)
    sh = st.cuda_stream
    V = {
        "encode only": lambda: c.encode_batch_dev(b, p, n * p, b + k * p, p, n * p, S, nb, sh),
        "encode + separate CRC pass": lambda: (c.encode_batch_dev(b, p, n * p, b + k * p, p, n * p, S, nb, sh),
                                               c.crc16_rows_dev(b, p, n * p, n, S, nb, raw.data_ptr(), n, sh)),
        "encode with fused CRC": lambda: c.encode_batch_dev_crc(b, p, n * p, b + k * p, p, n * p, S, nb,
                                                                raw.data_ptr(), sh),
        "fused CRC, nibble fold": lambda: cn.encode_batch_dev_crc(b, p, n * p, b + k * p, p, n * p, S, nb,
                                                                  raw.data_ptr(), sh),
    }
    s2 = torch.cuda.Stream()

    def staged(parts):
        # encode part i on the main stream while the CRC pass of part i - 1 runs on s2
        q = nb // parts
        for i in range(parts):
            off = i * q * n * p
            c.encode_batch_dev(b + off, p, n * p, b + off + k * p, p, n * p, S, q, sh)
            e = torch.cuda.Event()
            e.record(st)
            s2.wait_event(e)
            c.crc16_rows_dev(b + off, p, n * p, n, S, q, raw.data_ptr() + i * q * n * 4, n, s2.cuda_stream)
        e = torch.cuda.Event()
        e.record(s2)
        st.wait_event(e)

    if "fused" not in sys.argv[1:]:
        for parts in (2, 4, 8):
            V[f"encode || CRC pass, {parts} parts"] = lambda parts=parts: staged(parts)
    t_end = time.perf_counter() + 0.2
    while time.perf_counter() < t_end:
        for f in V.values():
            f()
        torch.cuda.synchronize()
    ts = {x: [] for x in V}
    for _ in range(7):
        for name, f in V.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            f()
            e1.record(st)
            e1.synchronize()
            ts[name].append(e0.elapsed_time(e1))
    for name in V:
        med = statistics.median(ts[name])
        print(f"RS({k},{m}) {B // 1024} KiB x {nb}: {name:32s} {med * 1e3:8.1f} us  "
              f"{nb * n * S / med / 1e6:8.1f} GB/s of shard bytes", flush=True)
    c.close()
    cn.close()


if __name__ == "__main__":
    fused_vs_separate()
    fused_vs_separate(16, 4, 4 << 20, 256)
    if "fused" not in sys.argv[1:]:
        main()
