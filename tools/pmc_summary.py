#!/usr/bin/env python3
"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-launch HBM traffic.

gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE counts half the bytes of a wide
coalesced streaming read, so fetch bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is exact for
16-B-per-lane streaming stores (bytes = WRITE_SIZE * 1024).  Averaged over dispatches.
Usage: pmc_summary.py <fetch_counter_csv> <write_counter_csv> <out_json> [<labels...>]
"""
import csv
import json
import re
import statistics
import sys


def label(name):
    """The label rsmi_last_kernel reports for the coding kernels (rs_fast_kernel<K, MT, NT, WPS,
    UA, CRC> -> rs_fast_kernel<K=..,MT=..,NT=..>[,UA][,CRC]); every other rsmi:: kernel (the fused
    matrix-core encode + CRC-16, the combine kernels, the rows passes, repitch) by its name and
    template arguments; None for kernels outside the library (torch's generators)."""
    m = re.search(r"rs_fast_kernel<(\d+), (\d+), (\d+), (\d+), (true|false), (true|false)(?:, (true|false))?>", name)
    if m:
        return f"rs_fast_kernel<K={m.group(1)},MT={m.group(2)},NT={m.group(3)}>" + (
            ",UA" if m.group(5) == "true" else "") + (",CRC" if m.group(6) == "true" else "") + (
            ",TB" if m.group(7) == "true" else "")
    m = re.search(r"rsmi::(\w+)(<[^>]*>)?", name)
    if not m:
        return None
    return m.group(1) + (m.group(2) or "").replace(" ", "")


def per_kernel(path, counter):
    d = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        key = label(r["Kernel_Name"])
        if key:
            d.setdefault(key, []).append(float(r["Counter_Value"]))
    return {k: statistics.mean(v) for k, v in d.items()}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in fetch:
        fb = 2 * fetch[k] * 1024
        wb = write.get(k, 0.0) * 1024
        out[k] = int(fb + wb)
        print(f"{k}: fetch {fb / 1e6:.1f} MB (2x FETCH_SIZE), write {wb / 1e6:.1f} MB, traffic {out[k] / 1e6:.1f} MB/launch")
    json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
