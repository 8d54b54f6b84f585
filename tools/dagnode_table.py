#!/usr/bin/env python3
"""Median and spread (min-max) of tools/dagnode_cpu_vs_gpu.sh's RESULT lines, GPU codec beside
CPU codec, per shape and Dag Node leg (GiB/s of block payload); with a second file of PHASES
lines, the median per-phase host time (ms: fetch / stage / codec / put, summed over threads, and
the leg's wall time) of the legs that report them."""
import json
import statistics
import sys

LEGS = [("put", "Put, per block"), ("putmany", "PutMany"), ("put_threads", "Put, 16 threads"),
        ("get", "Get, per block (1 lost shard)"), ("getmany", "GetMany"), ("get_threads", "Get, 16 threads"),
        ("repair", "RepairDataNode"), ("repair_batched", "RepairDataNodeBatched"),
        ("put_nolone", "Put, per block, lone-caller path off"), ("get_nolone", "Get, per block, lone-caller path off"),
        ("repair_nolone", "RepairDataNode, lone-caller path off")]


def phases(path):
    rows = [json.loads(l) for l in open(path) if l.strip()]
    shapes = []
    for r in rows:
        if (r["k"], r["m"], r["B"]) not in shapes:
            shapes.append((r["k"], r["m"], r["B"]))
    for k, m, B in shapes:
        print(f"\nRS({k},{m}) {B // 1024} KiB: per-phase host time, ms, median of runs (summed over threads)")
        print("| leg | codec | wall | fetch | stage | codec call | datanode puts |")
        print("|---|---|---|---|---|---|---|")
        for leg in ("put", "putmany", "put_threads", "get", "getmany", "get_threads", "repair_batched"):
            for codec in ("gpu", "cpu"):
                v = [r[leg] for r in rows if r["codec"] == codec and (r["k"], r["m"], r["B"]) == (k, m, B) and leg in r]
                if not v:
                    continue
                med = {f: 1e3 * statistics.median(x[f] for x in v) for f in ("wall", "fetch", "stage", "codec", "put")}
                print(f"| {leg} | {codec} | {med['wall']:.1f} | {med['fetch']:.1f} | {med['stage']:.1f} | "
                      f"{med['codec']:.1f} | {med['put']:.1f} |")


def main(path):
    rows = [json.loads(l) for l in open(path) if l.strip()]
    shapes = []
    for r in rows:
        s = (r["k"], r["m"], r["B"], r["N"])
        if s not in shapes:
            shapes.append(s)
    cpu = next((r for r in rows if r["codec"] == "cpu"), None)
    if cpu:
        print(f"CPU codec: oracle/rs_cpu_fast.c {cpu['isa']}, {cpu['threads']} threads per batch (one per block call)")
    for k, m, B, N in shapes:
        print(f"\nRS({k},{m}) {B // 1024} KiB blocks x {N}, {k + m} in-process datanodes; GiB/s, median [min-max] of runs")
        print(f"| leg | GPU codec (librsmi) | CPU codec | GPU / CPU |")
        print(f"|---|---|---|---|")
        for key, name in LEGS:
            cells, med = [], {}
            for codec in ("gpu", "cpu"):
                v = [r[key] for r in rows if r["codec"] == codec and (r["k"], r["m"], r["B"], r["N"]) == (k, m, B, N)
                     and key in r]
                if v:
                    med[codec] = statistics.median(v)
                    cells.append(f"{med[codec]:.2f} [{min(v):.2f}-{max(v):.2f}] ({len(v)})")
                else:
                    cells.append("-")
            ratio = f"{med['gpu'] / med['cpu']:.2f}x" if "gpu" in med and "cpu" in med and med["cpu"] else "-"
            print(f"| {name} | {cells[0]} | {cells[1]} | {ratio} |")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/dagnode_cmp.jsonl")
    if len(sys.argv) > 2:
        phases(sys.argv[2])
