#!/usr/bin/env python3
"""Diagnostic: average PMC counters per (kernel, grid) over rocprofv3 counter-collection CSVs.
Usage: pmc_table.py CSV... [--match SUBSTRING]"""
import collections
import csv
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else ""
if match:
    args.remove(match)
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in args:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if match not in k:
            continue
        agg[(k, r.get("Grid_Size", ""))][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (k, g), d in agg.items():
    print(f"{k} grid {g} (n={len(next(iter(d.values())))})")
    for c, v in sorted(d.items()):
        print(f"   {c:24s} {sum(v) / len(v):16.0f}")
