#!/usr/bin/env python3
"""Generate the committed golden fixtures from the CPU oracle (oracle/rs_oracle.c).

Provenance: "restatement-derived, KAT-anchored" (SURVEY.md 8(c)).  The oracle must pass
rs_oracle_selftest() (upstream klauspost v1.11.0 KATs + the reference's RS(2,1)
"123456" fixture) before anything is written.  Inputs are splitmix64 bytes with seed
0xF11EDA6 ^ index.  Run from the repo root:  python tests/golden/gen_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as orc  # noqa: E402

CONFIGS = [(2, 1), (4, 2), (10, 4), (16, 4), (5, 5)]
SIZES = [1, 6, 4099]


def main():
    assert orc.lib().rs_oracle_selftest() == 0, "oracle failed its known-answer tests"
    mats = {f"{k},{m}": orc.build_matrix(k, m).tolist() for k, m in CONFIGS}
    with open(os.path.join(HERE, "matrices.json"), "w") as f:
        json.dump({"provenance": "rs_oracle_build_matrix (KAT-anchored restatement of klauspost v1.11.0)",
                   "matrices": mats}, f, indent=0)
    for k, m in CONFIGS:
        n = k + m
        arrays = {}
        for B in SIZES:
            block = orc.splitmix64_bytes(0xF11EDA6 ^ (1000 * k + B), B)
            sh = orc.split(k, m, block.tobytes())
            sh[k:] = orc.encode(k, m, sh[:k])
            arrays[f"block_{B}"] = block
            arrays[f"shards_{B}"] = sh
            # reconstruct vectors: first data shard lost (ReconstructData) and the
            # last min(m,2) shards + first data shard lost (Reconstruct)
            lost = [0] + list(range(n - min(m, 2) + 1, n)) if m >= 2 else [0]
            present = np.array([i not in lost for i in range(n)], dtype=np.uint8)
            er = sh.copy()
            er[lost] = 0
            rc, rec = orc.reconstruct(k, m, er, present, False)
            assert rc == 0 and np.array_equal(rec, sh)
            arrays[f"present_{B}"] = present
        if (k, m) == (2, 1):
            sh = orc.split(2, 1, b"123456")
            sh[2:] = orc.encode(2, 1, sh[:2])
            arrays["shards_123456"] = sh
        np.savez(os.path.join(HERE, f"vectors_k{k}_m{m}.npz"), **arrays)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
