#!/usr/bin/env python3
"""Summarise tools/bench_dagnode's TRACE line (BENCH_DAGNODE_TRACE=1): the batched repair's
phase intervals per thread.

    python tools/trace_timeline.py LOG [LOG ...]

Prints, per TRACE line: the wall time; per phase the summed time and the time any thread
spent in it (the union of its intervals); how long the calling thread (the one that stages and
codes) was busy, waiting for the fetch ahead and waiting for the writes; and the share of the
wall in which no stage or codec ran (the calling thread's idle or waiting time).
"""
import json
import sys

NAMES = {0: "fetch", 1: "stage", 2: "codec", 3: "put", 4: "wait fetch", 5: "wait writes"}


def union(iv):
    iv = sorted(iv)
    tot, cur0, cur1 = 0.0, None, None
    for a, b in iv:
        if cur1 is None or a > cur1:
            if cur1 is not None:
                tot += cur1 - cur0
            cur0, cur1 = a, b
        else:
            cur1 = max(cur1, b)
    if cur1 is not None:
        tot += cur1 - cur0
    return tot


def summarise(t):
    ev = t["events"]
    wall = t["wall_ms"]
    print(f"RS({t['k']},{t['m']}) B={t['B']}: wall {wall:.2f} ms, {len(ev)} intervals")
    for p in sorted(NAMES):
        iv = [(e[2], e[3]) for e in ev if e[1] == p]
        if not iv:
            continue
        s = sum(b - a for a, b in iv)
        print(f"  {NAMES[p]:12s} {len(iv):4d} x, sum {s:7.2f} ms, union {union(iv):7.2f} ms, "
              f"mean {s / len(iv):6.3f} ms")
    # the calling thread: the one with the stage intervals
    main = next((e[0] for e in ev if e[1] == 1), None)
    if main is not None:
        busy = union([(e[2], e[3]) for e in ev if e[0] == main and e[1] in (1, 2)])
        wait = union([(e[2], e[3]) for e in ev if e[0] == main and e[1] in (4, 5)])
        print(f"  calling thread: stage+codec {busy:.2f} ms, waiting {wait:.2f} ms, "
              f"other {wall - busy - wait:.2f} ms of {wall:.2f}")
        fetch = union([(e[2], e[3]) for e in ev if e[1] == 0])
        both = union([(e[2], e[3]) for e in ev if e[1] in (0, 1, 2)])
        print(f"  fetch and stage/codec overlap: {fetch + busy - both:.2f} ms "
              f"(fetch {fetch:.2f}, stage+codec {busy:.2f}, together {both:.2f})")


def main(paths):
    for p in paths:
        with open(p) as f:
            for line in f:
                if line.startswith("TRACE "):
                    summarise(json.loads(line[6:]))


if __name__ == "__main__":
    main(sys.argv[1:])
