#!/usr/bin/env python3
"""Static per-kernel instruction breakdown of the gfx950 assembly (hipcc -save-temps .s).

Usage: isa_breakdown.py <file.s> <kernel-substring> [<kernel-substring> ...]
Counts every instruction of each matching kernel's body by class (GF selectors, v_perm,
3-input XORs, bit-form construction, MFMA, memory, scalar, waits) and prints one table.
The coding kernels are straight-line per tile (every row loop is unrolled), so a static count
is the per-tile issue count plus the prologue and the record / store epilogue."""
import re
import sys
from collections import Counter, OrderedDict

CLASSES = OrderedDict([
    ("v_perm", lambda op: op == "v_perm_b32"),
    ("v_bitop3", lambda op: op.startswith("v_bitop3")),
    ("v_xor", lambda op: op.startswith("v_xor")),
    ("v_and/or/bfe/shift", lambda op: re.match(r"v_(and|or|bfe|lshr|lshl|ashr|alignbit|alignbyte|and_or|lshl_or|or3|lshl_add)", op) is not None),
    ("v_mfma", lambda op: op.startswith("v_mfma")),
    ("v_cndmask/cmp", lambda op: op.startswith("v_cndmask") or op.startswith("v_cmp")),
    ("v_mov/readlane", lambda op: op.startswith("v_mov") or op.startswith("v_readfirstlane") or op.startswith("v_readlane") or op.startswith("v_accvgpr")),
    ("v_add/mul/mad", lambda op: re.match(r"v_(add|sub|mul|mad|lshl_add|add3|cvt|fma)", op) is not None),
    ("v_other", lambda op: op.startswith("v_")),
    ("global/buffer", lambda op: op.startswith("global_") or op.startswith("buffer_") or op.startswith("flat_")),
    ("ds", lambda op: op.startswith("ds_")),
    ("s_waitcnt", lambda op: op.startswith("s_waitcnt")),
    ("s_other", lambda op: op.startswith("s_")),
])


def kernels(path):
    cur, body = None, []
    for line in open(path):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            if cur:
                yield cur, body
            cur, body = m.group(1), []
            continue
        if cur and line.startswith("\t.size") and cur in line:
            yield cur, body
            cur, body = None, []
            continue
        if cur:
            s = line.strip()
            if s and not s.startswith((".", ";")) and not s.endswith(":"):
                body.append(s.split()[0])


def classify(ops):
    c = Counter()
    for op in ops:
        for name, f in CLASSES.items():
            if f(op):
                c[name] += 1
                break
        else:
            c["other"] += 1
    return c


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    rows = []
    for name, ops in kernels(path):
        if any(s in name for s in subs):
            rows.append((name, classify(ops), len(ops)))
    cols = list(CLASSES) + ["other"]
    print("kernel".ljust(44) + "".join(c[:9].rjust(10) for c in cols) + "total".rjust(8) + "VALU".rjust(7))
    for name, c, tot in rows:
        short = re.sub(r"^_ZN4rsmi\d+", "", name)[:44]
        valu = sum(v for k, v in c.items() if k.startswith("v_") and k != "v_mfma")
        print(short.ljust(44) + "".join(str(c.get(k, 0)).rjust(10) for k in cols) + str(tot).rjust(8) + str(valu).rjust(7))


if __name__ == "__main__":
    main()
