#!/usr/bin/env python3
"""Check the completion-flag release in the gfx950 assembly of the table-of-bases kernels.

Every kernel that counts its workgroups with a system-scope global_atomic_add (launch_done,
csrc/rs_kernels.hip) must have, in every wave, no vector store still outstanding when the
workgroup barrier before that atomic passes: on every straight-line path from a vector store to
the flag's s_barrier (the barrier whose next barrier-or-atomic in the text is the flag atomic)
there has to be an `s_waitcnt vmcnt(0)`.  The check is on program text: a store followed by a
flag barrier with no vmcnt(0) wait between them, inside one kernel that has the flag atomic, is
reported (stores before an earlier, LDS-only barrier still count as pending).

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC --cuda-device-only -S \
        filedag-storage_amd/csrc/rs_kernels_tb.hip -o /tmp/tb.s
    python tools/check_flag_fence.py /tmp/tb.s
"""
import re
import sys

STORE = re.compile(r"^\s*(global_store|flat_store|buffer_store)\w*")
WAIT0 = re.compile(r"^\s*s_waitcnt\b.*vmcnt\(0\)")
BARRIER = re.compile(r"^\s*s_barrier\b")
FLAG_ATOMIC = re.compile(r"^\s*global_atomic_add\b.*sc0 sc1")
FUNC = re.compile(r"^(_Z\w+):")


def kernels(lines):
    name, body = None, []
    for ln in lines:
        m = FUNC.match(ln)
        if m:
            if name:
                yield name, body
            name, body = m.group(1), []
        elif name:
            body.append(ln)
    if name:
        yield name, body


def check(path):
    with open(path) as f:
        lines = f.read().splitlines()
    checked = bad = 0
    barriers = 0
    for name, body in kernels(lines):
        # the function's text ends at its .Lfunc_end label
        end = next((i for i, ln in enumerate(body) if ln.startswith(".Lfunc_end")), len(body))
        body = body[:end]
        if not any(FLAG_ATOMIC.match(ln) for ln in body):
            continue
        checked += 1
        pending = False
        for i, ln in enumerate(body):
            if STORE.match(ln):
                pending = True
            elif WAIT0.match(ln):
                pending = False
            elif BARRIER.match(ln):
                # a flag barrier: the next barrier-or-flag-atomic in the text is the atomic
                nxt = next((b for b in body[i + 1:] if BARRIER.match(b) or FLAG_ATOMIC.match(b)), "")
                if FLAG_ATOMIC.match(nxt):
                    barriers += 1
                    if pending:
                        bad += 1
                        print(f"UNFENCED {name[:80]} line {i}: store reaches the flag barrier without vmcnt(0)")
                # stores before an LDS-only barrier stay pending: the flag barrier must drain them
    print(f"{checked} flag kernels, {barriers} barriers checked, {bad} unfenced")
    return 0 if checked and not bad else 1


if __name__ == "__main__":
    sys.exit(check(sys.argv[1] if len(sys.argv) > 1 else "/tmp/tb.s"))
