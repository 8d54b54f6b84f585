#!/usr/bin/env python3
"""Median and spread (min-max) of tools/dagnode_cpu_vs_gpu.sh's RESULT lines, GPU codec beside
CPU codec, per shape and Dag Node leg (GiB/s of block payload)."""
import json
import statistics
import sys

LEGS = [("put", "Put, per block"), ("putmany", "PutMany"), ("put_threads", "Put, 16 threads"),
        ("get", "Get, per block (1 lost shard)"), ("getmany", "GetMany"), ("get_threads", "Get, 16 threads"),
        ("repair", "RepairDataNode"), ("repair_batched", "RepairDataNodeBatched")]


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
                v = [r[key] for r in rows if r["codec"] == codec and (r["k"], r["m"], r["B"], r["N"]) == (k, m, B, N)]
                if v:
                    med[codec] = statistics.median(v)
                    cells.append(f"{med[codec]:.2f} [{min(v):.2f}-{max(v):.2f}] ({len(v)})")
                else:
                    cells.append("-")
            ratio = f"{med['gpu'] / med['cpu']:.2f}x" if "gpu" in med and "cpu" in med and med["cpu"] else "-"
            print(f"| {name} | {cells[0]} | {cells[1]} | {ratio} |")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/dagnode_cmp.jsonl")
