#!/usr/bin/env python3
"""Launch the fused encode + CRC-16 (bench layout: RS(10,4) 256 KiB x 4096, 32 KiB pitch) a few
times, for rocprofv3 kernel-trace / PMC passes.  RSMI_LIB selects a library variant."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))
import rsmi  # noqa: E402


def main():
    k, m, nb, B = 10, 4, 4096, 262144
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    n, S = k + m, (B + k - 1) // k
    rs = rsmi.recommended_pitch(S)
    buf = torch.randint(0, 256, (nb * n * rs,), dtype=torch.uint8, device="cuda")
    raw = torch.empty((nb, n), dtype=torch.int32, device="cuda")
    b = buf.data_ptr()
    c = rsmi.Codec(k, m)
    sh = torch.cuda.current_stream().cuda_stream
    for _ in range(iters):
        c.encode_batch_dev_crc(b, rs, n * rs, b + k * rs, rs, n * rs, S, nb, raw.data_ptr(), sh)
        c.encode_batch_dev(b, rs, n * rs, b + k * rs, rs, n * rs, S, nb, sh)
    torch.cuda.synchronize()
    print("kernels:", c.last_kernel())


if __name__ == "__main__":
    main()
