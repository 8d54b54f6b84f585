#!/usr/bin/env python3
"""Where a per-block host call's time goes, from a rocprofv3 --kernel-trace --hip-runtime-trace
run of tools/latency.cpp: per kernel name, the median of (launch API duration, launch API end ->
kernel start, kernel duration, kernel end -> the next hipStreamSynchronize's return), the
kernel matched to its launch by correlation id.  Usage: call_breakdown.py <dir with lat_*.csv>"""
import bisect
import csv
import re
import statistics
import sys
from collections import defaultdict


def main(d):
    api = list(csv.DictReader(open(f"{d}/lat_hip_api_trace.csv")))
    ker = list(csv.DictReader(open(f"{d}/lat_kernel_trace.csv")))
    launch = {r["Correlation_Id"]: r for r in api if r["Function"] in ("hipLaunchKernel", "hipExtLaunchKernel")}
    syncs = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in api
                   if r["Function"] in ("hipStreamSynchronize", "hipDeviceSynchronize"))
    sync_starts = [s for s, _ in syncs]
    rows = defaultdict(list)
    for k in ker:
        l = launch.get(k["Correlation_Id"])
        if not l:
            continue
        ks, ke = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
        ls, le = int(l["Start_Timestamp"]), int(l["End_Timestamp"])
        i = bisect.bisect_left(sync_starts, le)
        if i >= len(syncs):
            continue
        ss, se = syncs[i]
        name = re.sub(r"\(.*", "", k["Kernel_Name"]).replace("void rsmi::", "").replace("rsmi::", "")
        rows[name].append(((le - ls) / 1e3, (ks - le) / 1e3, (ke - ks) / 1e3, (se - ke) / 1e3, (se - ss) / 1e3))
    print(f"{'kernel':52s} {'n':>5} {'launch':>7} {'->start':>8} {'kernel':>7} {'end->ret':>9} {'sync':>7}  (us, medians)")
    for name, v in sorted(rows.items()):
        med = [statistics.median(x[i] for x in v) for i in range(5)]
        print(f"{name:52s} {len(v):5d} {med[0]:7.2f} {med[1]:8.2f} {med[2]:7.2f} {med[3]:9.2f} {med[4]:7.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
