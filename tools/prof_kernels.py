#!/usr/bin/env python3
"""Launch exactly the bench's dominant kernels a few times (for rocprofv3 kernel-trace / PMC
passes).  Same workload as bench.py.  Usage: prof_kernels.py [iters] [pitched|split|fused]
(split: rows back to back at pitch S, the UA kernels; fused: the encode with the CRC-16 fused
in, then the combine, on the pitched layout)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))
import rsmi  # noqa: E402


def main():
    k, m, nb, B = 10, 4, 4096, 256 * 1024
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    mode = sys.argv[2] if len(sys.argv) > 2 else "pitched"
    n = k + m
    S = (B + k - 1) // k
    rs = S if mode == "split" else rsmi.recommended_pitch(S)
    buf = torch.randint(0, 256, (nb, n, rs), dtype=torch.uint8, device="cuda")
    raw = torch.empty((nb, n), dtype=torch.int32, device="cuda")
    base = buf.data_ptr()
    c = rsmi.Codec(k, m)
    st = torch.cuda.current_stream().cuda_stream
    present = [i != 0 for i in range(n)]
    for _ in range(iters):
        if mode == "fused":
            c.encode_batch_dev_crc(base, rs, n * rs, base + k * rs, rs, n * rs, S, nb, raw.data_ptr(), st)
        else:
            c.encode_batch_dev(base, rs, n * rs, base + k * rs, rs, n * rs, S, nb, st)
        c.reconstruct_batch_dev(base, rs, n * rs, S, nb, present, True, st)
    torch.cuda.synchronize()
    print("kernels:", c.last_kernel(), "S", S, "pitch", rs, "alg bytes enc", nb * n * S, "rec", nb * (k + 1) * S)


if __name__ == "__main__":
    main()
