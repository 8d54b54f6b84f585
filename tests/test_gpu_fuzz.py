"""Seeded random-shape parity sweep on the GPU: random (k, m), shard sizes, batch sizes,
layouts (aligned pitches, padded strides, unaligned offsets) and erasure patterns, every
result compared byte for byte with the CPU oracle.  Complements the fixed grids of
test_gpu_parity.py with shapes nobody picked by hand."""
import numpy as np
import pytest

import oracle_lib as orc
import rsmi

CASES = 60


def _case(seed):
    r = np.random.default_rng(1000 + seed)
    k = int(r.choice([1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 16, 17, 20]))
    m = int(r.integers(1, min(8, 256 - k) + 1))
    S = int(r.choice([1, 2, 15, 16, 17, int(r.integers(1, 5000)), int(r.integers(5000, 70000))]))
    nb = int(r.integers(1, 9))
    layout = r.choice(["pitched", "padded", "unaligned"])
    nlost = int(r.integers(1, m + 1))
    lost = sorted(int(x) for x in r.choice(k + m, size=nlost, replace=False))
    data_only = bool(r.integers(0, 2))
    return k, m, S, nb, str(layout), lost, data_only, r


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(CASES))
def test_random_shape_encode_reconstruct(seed):
    import torch

    k, m, S, nb, layout, lost, data_only, r = _case(seed)
    n = k + m
    if layout == "pitched":
        rs, off = rsmi.recommended_pitch(S), 0
    elif layout == "padded":
        rs, off = (S + 15) // 16 * 16 + 48, 0
    else:
        rs, off = S + 3, 7
    bs = n * rs + (16 if layout == "padded" else 0)
    host = np.zeros(off + nb * bs + 64, dtype=np.uint8)
    data = r.integers(0, 256, size=(nb, k, S), dtype=np.uint8)
    for b in range(nb):
        for c in range(k):
            host[off + b * bs + c * rs:][:S] = data[b, c]
    d = torch.from_numpy(host).cuda()
    base = d.data_ptr() + off
    st = torch.cuda.current_stream().cuda_stream
    with rsmi.Codec(k, m) as c:
        c.encode_batch_dev(base, rs, bs, base + k * rs, rs, bs, S, nb, st)
        torch.cuda.synchronize()
        got = d.cpu().numpy()
        want = orc.encode_fast(k, m, data, threads=4)
        full = np.zeros((nb, n, S), dtype=np.uint8)
        full[:, :k] = data
        full[:, k:] = want
        for b in range(nb):
            for j in range(m):
                assert np.array_equal(got[off + b * bs + (k + j) * rs:][:S], want[b, j]), (b, j)
        # erase and rebuild
        for b in range(nb):
            for i in lost:
                d[off + b * bs + i * rs: off + b * bs + i * rs + S] = 0
        present = [i not in lost for i in range(n)]
        c.reconstruct_batch_dev(base, rs, bs, S, nb, present, data_only, st)
        torch.cuda.synchronize()
        got = d.cpu().numpy()
    for b in range(nb):
        for i in range(n):
            row = got[off + b * bs + i * rs:][:S]
            if i not in lost or i < k or not data_only:
                assert np.array_equal(row, full[b, i]), (k, m, S, layout, lost, data_only, b, i)
            else:
                assert not row.any()
