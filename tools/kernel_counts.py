#!/usr/bin/env python3
"""Diagnostic: kernels of two rocprofv3 kernel traces side by side (tools/gpu_session.sh
kernarg_trace: the Dag Node bench with HIP_FORCE_DEV_KERNARG 0 and 1).  Per kernel name: the
dispatch count, the summed and median duration, and, per hardware queue, the summed idle gap
between one dispatch's end and the next dispatch's start on that queue."""
import csv
import statistics
import sys
from collections import defaultdict


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((r["Kernel_Name"], int(r["Queue_Id"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return rows


def short(name):
    name = name.replace("void ", "")
    cut = name.find("(")
    return (name[:cut] if cut > 0 else name)[:70]


def summary(rows):
    by = defaultdict(list)
    for n, _, s, e in rows:
        by[short(n)].append(e - s)
    gaps = defaultdict(int)
    per_q = defaultdict(list)
    for n, q, s, e in rows:
        per_q[q].append((s, e))
    for q, v in per_q.items():
        v.sort()
        for (s0, e0), (s1, _) in zip(v, v[1:]):
            if s1 > e0:
                gaps[q] += s1 - e0
    return by, gaps


def main():
    runs = [summary(load(p)) for p in sys.argv[1:]]
    names = sorted({n for by, _ in runs for n in by}, key=lambda n: -sum(runs[0][0].get(n, [0])))
    print("kernel".ljust(72) + "".join(f"| {'run ' + str(i)} count, sum ms, median us ".ljust(36) for i in range(len(runs))))
    for n in names:
        line = n.ljust(72)
        for by, _ in runs:
            d = by.get(n, [])
            line += f"| {len(d):7d} {sum(d) / 1e6:9.2f} {statistics.median(d) / 1e3 if d else 0:9.1f}".ljust(36)
        print(line)
    for i, (by, gaps) in enumerate(runs):
        tot = sum(len(v) for v in by.values())
        busy = sum(sum(v) for v in by.values())
        print(f"run {i}: {tot} dispatches, {busy / 1e6:.2f} ms of kernel time; idle gaps between dispatches per queue: "
              + ", ".join(f"q{q} {g / 1e6:.2f} ms" for q, g in sorted(gaps.items())))


if __name__ == "__main__":
    main()
