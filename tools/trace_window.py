#!/usr/bin/env python3
"""Average rocprofv3 kernel-trace durations over bench.py's timed window.

bench.py launches the encode (and reconstruct) kernel once per step; the timed window is
the `steps` dispatches of each kernel after the settle steps, the warmup steps and one
label probe (the sustained run and the self check come after it).
Usage: trace_window.py <kernel_trace.csv> <bench.json> [out.json]
Prints, per kernel, the window average next to bench.py's own HIP-event average; out.json gets
{kernel label: window average in ms} (profiles/trace_window.json, which bench.py's roofline
block carries beside its event-timed figures).
"""
import csv
import json
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    bench = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
    steps = bench["steps"]
    first = bench["config"]["settle"]["steps"] + bench["warmup"] + 1
    per = {}
    for r in rows:
        m = re.search(r"rs_fast_kernel<(\d+), (\d+), (\d+), (\d+), (true|false), (true|false)(?:, (true|false))?>", r["Kernel_Name"])
        if not m:
            continue
        key = f"rs_fast_kernel<K={m.group(1)},MT={m.group(2)},NT={m.group(3)}>" + (",UA" if m.group(5) == "true" else "") + (
            ",CRC" if m.group(6) == "true" else "")
        per.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    ev = {bench["roofline"]["kernel"]: bench["roofline"]["avg_launch_ms"] * 1e3}
    if "reconstruct" in bench:
        rec = bench["reconstruct"]
        ev[rec["kernel"]] = rec.get("avg_launch_ms", rec.get("avg_launch_ms_incl_event_gap")) * 1e3
    # bench.py times every `every`-th step with HIP events (round 3; every step before)
    timed = bench["roofline"].get("launches_timed", steps)
    every = -(-steps // timed)
    summary = {}
    for k, d in per.items():
        w = d[first:first + steps]
        avg = sum(w) / len(w)
        ws = w[::every]
        avs = sum(ws) / len(ws)
        e = ev.get(k)
        extra = (f"; the {len(ws)} event-timed steps avg {avs:.1f} us, bench.py HIP events {e:.1f} us "
                 f"({(e / avs - 1) * 100:+.1f} %)") if e else ""
        print(f"{k}: {len(d)} dispatches, timed window ({len(w)} steps) avg {avg:.1f} us, "
              f"min {min(w):.1f}, max {max(w):.1f}{extra}")
        summary[k] = round(avg / 1e3, 4)
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
