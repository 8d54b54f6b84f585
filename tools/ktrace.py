#!/usr/bin/env python3
"""Per-kernel average duration from a rocprofv3 kernel-trace CSV (skipping each kernel's first
`skip` dispatches).  Usage: ktrace.py <kernel_trace.csv> [skip]"""
import collections
import csv
import sys


def main():
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    per = collections.OrderedDict()
    for r in csv.DictReader(open(sys.argv[1])):
        name = r["Kernel_Name"]
        if "rsmi::" not in name:
            continue
        short = name.split("(")[0].replace("void ", "")
        per.setdefault((short, r["VGPR_Count"], r["LDS_Block_Size"]), []).append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for (k, v, lds), d in per.items():
        d = d[skip:] or d
        print(f"{k:70s} vgpr {v:>4s} lds {lds:>6s}  n {len(d):4d}  avg {sum(d) / len(d):8.1f} us  min {min(d):8.1f}")


if __name__ == "__main__":
    main()
