#!/usr/bin/env python3
"""Diagnostic: does timing each kernel with HIP events cost the headline step time?  The bench's
step (RS(10,4) 256 KiB x 4096 encode + 1-row ReconstructData, pitched) run K times back to back
on one stream, alternating three forms: no events inside the loop, one event pair per step, and
bench.py's form (an event before each kernel).  Wall time per step over the K steps, median of
rounds.  Usage: eventgap.py [steps] [rounds]"""
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))
import rsmi  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    k, m, nb, B = 10, 4, 4096, 256 * 1024
    n, S = k + m, (B + k - 1) // k
    rs = rsmi.recommended_pitch(S)
    buf = torch.randint(0, 256, (nb, n, rs), dtype=torch.uint8, device="cuda")
    base = buf.data_ptr()
    c = rsmi.Codec(k, m)
    stream = torch.cuda.Stream()
    st = stream.cuda_stream
    present = [i != 0 for i in range(n)]

    def enc():
        c.encode_batch_dev(base, rs, n * rs, base + k * rs, rs, n * rs, S, nb, st)

    def rec():
        c.reconstruct_batch_dev(base, rs, n * rs, S, nb, present, True, st)

    def run(form):
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(2 * steps + 1)] if form else []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            if form == 2:
                evs[2 * i].record(stream)
            elif form == 1 and i == 0:
                evs[0].record(stream)
            enc()
            if form == 2:
                evs[2 * i + 1].record(stream)
            rec()
        if form:
            evs[2 * steps].record(stream)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e6

    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:
        enc()
        rec()
        torch.cuda.synchronize()
    # form 3: the K steps captured once as a HIP graph and replayed
    graph = None
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            for _ in range(steps):
                enc()
                rec()
        graph = g
    except Exception as e:  # the library's launches may not be capturable
        print("graph capture failed:", repr(e)[:200], flush=True)

    def run_graph():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        graph.replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e6

    res = {0: [], 1: [], 2: [], 3: []}
    for _ in range(rounds):
        for form in (0, 1, 2):
            res[form].append(run(form))
        if graph is not None:
            res[3].append(run_graph())
    names = {0: "no events", 1: "events around the loop", 2: "an event before each kernel (bench.py)",
             3: "the K steps as one HIP graph"}
    for form in (0, 1, 2, 3) if graph is not None else (0, 1, 2):
        v = res[form]
        print(f"{names[form]:42s} median {statistics.median(v):8.1f} us/step  [{min(v):.1f}-{max(v):.1f}]", flush=True)


if __name__ == "__main__":
    main()
