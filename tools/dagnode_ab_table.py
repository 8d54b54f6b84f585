#!/usr/bin/env python3
"""Median [min-max] per library variant, shape and Dag Node leg (GiB/s of block payload) of
tools/dagnode_ab.sh's RESULT lines."""
import json
import statistics
import sys

LEGS = ["put", "putmany", "put_threads", "get", "getmany", "get_threads", "repair", "repair_batched"]


def main():
    rows = [json.loads(l) for l in open(sys.argv[1]) if l.strip()]
    shapes, variants = [], []
    for r in rows:
        if (r["k"], r["m"], r["B"]) not in shapes:
            shapes.append((r["k"], r["m"], r["B"]))
        if r["variant"] not in variants:
            variants.append(r["variant"])
    for k, m, B in shapes:
        print(f"\nRS({k},{m}) {B // 1024} KiB, GPU codec, GiB/s median [min-max] of runs")
        print("| leg | " + " | ".join(variants) + " |")
        print("|---" * (len(variants) + 1) + "|")
        for leg in LEGS:
            cells = []
            for v in variants:
                x = [r[leg] for r in rows if r["variant"] == v and (r["k"], r["m"], r["B"]) == (k, m, B) and leg in r]
                cells.append(f"{statistics.median(x):.2f} [{min(x):.2f}-{max(x):.2f}]" if x else "-")
            print(f"| {leg} | " + " | ".join(cells) + " |")
        for leg in ("put_threads", "get_threads"):
            cells = []
            for v in variants:
                x = [r for r in rows if r["variant"] == v and (r["k"], r["m"], r["B"]) == (k, m, B)
                     and r.get(leg + "_calls")]
                cells.append(f"{statistics.median(r[leg + '_batches'] / r[leg + '_calls'] for r in x):.2f}" if x else "-")
            print(f"| {leg} batches / calls | " + " | ".join(cells) + " |")


if __name__ == "__main__":
    main()
