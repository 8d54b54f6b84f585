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


GROUP_CASES = 16


def _group_case(seed):
    r = np.random.default_rng(5000 + seed)
    k, m = [(2, 1), (4, 2), (10, 4), (16, 4), (3, 2), (10, 4)][int(r.integers(0, 6))]
    B = int(r.choice([int(r.integers(1, 64)), int(r.integers(64, 5000)), int(r.integers(5000, 300000)),
                      262144, 1048576 + 14]))
    T = int(r.choice([2, 3, int(r.integers(4, 20)), int(r.integers(60, 70))]))
    crc = bool(r.integers(0, 2))
    nlost = int(r.integers(1, m + 1))
    lost = sorted(int(x) for x in r.choice(k + m, size=nlost, replace=False))
    data_only = bool(r.integers(0, 2))
    return k, m, B, T, crc, lost, data_only, r


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(GROUP_CASES))
def test_random_coalesced_groups(seed):
    """Seeded random coalesced groups (DagNode.Put / degraded Get from T goroutines at once,
    node.go:358-408 / :220-326) over page-locked buffers: random (k, m) among the table shapes and
    one without, block sizes from 1 byte to 1 MiB + 14 (rows under 16 bytes, aligned and odd
    shard sizes), 2..69 requests in one deterministic batch (one lane, coalesce_us; more than 64
    take two table launches), with and without CRC-16, then a random loss pattern rebuilt the same
    way.  Every shard, R(shard) and rebuilt row equals the oracle's; rows not asked for stay
    untouched."""
    import ctypes
    import threading

    k, m, B, T, crc, lost, data_only, r = _group_case(seed)
    n = k + m
    S = (B + k - 1) // k
    L = rsmi.lib()
    blocks = [bytes(r.integers(0, 256, size=B, dtype=np.uint8)) for _ in range(T)]
    want = []
    for b in blocks:
        w = orc.split(k, m, b)
        w[k:] = orc.encode(k, m, w[:k])
        want.append(w)
    ptrs = [L.rsmi_host_alloc(n * S) for _ in range(T)]
    assert all(ptrs)
    try:
        views = [np.ctypeslib.as_array((ctypes.c_uint8 * (n * S)).from_address(p)).reshape(n, S) for p in ptrs]
        raws = [(ctypes.c_uint32 * n)() for _ in range(T)]
        with rsmi.Codec(k, m) as c:
            c.set_option("coalesce_lanes", 1)
            c.set_option("coalesce_us", 100000)
            c.set_option("coalesce_max", T)
            for t in range(T):
                flat = views[t].reshape(-1)
                flat[:] = 0x5A
                flat[:B] = np.frombuffer(blocks[t], dtype=np.uint8)
            rcs = [None] * T

            def enc(t):
                rcs[t] = L.rsmi_encode_block_coalesced(c._h, ptrs[t], B, ptrs[t], raws[t] if crc else None)

            th = [threading.Thread(target=enc, args=(t,)) for t in range(T)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            assert rcs == [0] * T, c.last_kernel()
            for t in range(T):
                assert np.array_equal(views[t], want[t]), (t, c.last_kernel())
                for i in range(n if crc else 0):
                    assert rsmi.crc16_entry(b"", raws[t][i], S) == orc.crc16_ibm(want[t][i].tobytes()), (t, i)
            present = (ctypes.c_uint8 * n)(*[0 if i in lost else 1 for i in range(n)])
            for t in range(T):
                views[t][lost] = 0xEE

            def rec(t):
                rcs[t] = L.rsmi_reconstruct_coalesced(c._h, ptrs[t], S, present, 1 if data_only else 0)

            th = [threading.Thread(target=rec, args=(t,)) for t in range(T)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            assert rcs == [0] * T
            for t in range(T):
                for i in range(n):
                    if i in lost and data_only and i >= k:
                        assert (views[t][i] == 0xEE).all(), (t, i)
                    else:
                        assert np.array_equal(views[t][i], want[t][i]), (t, i, c.last_kernel())
    finally:
        for p in ptrs:
            L.rsmi_host_free(p)


LONE_CASES = 24


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(LONE_CASES))
def test_random_lone_in_place_calls(seed):
    """Seeded random one-block in-place host calls on page-locked memory -- a lone DagNode.Put,
    repair, degraded and verified read (node.go:358-408, :220-326, data_recovery.go:16-112) --
    which take the one-base table launches with completion flags where the shape has them and
    the plain launches and stream synchronisation where it does not (rows under 16 bytes, shapes
    without table kernels, 5+ lost rows): random (k, m), block sizes from 1 byte to 1 MiB + 14,
    random loss patterns, the option coalesce_flag on and off.  Shards, R(shard), rebuilt rows and
    the survivors' R(row) against the oracle."""
    import ctypes

    r = np.random.default_rng(9000 + seed)
    k, m = [(2, 1), (4, 2), (10, 4), (16, 4), (3, 2), (5, 5), (10, 4)][int(r.integers(0, 7))]
    B = int(r.choice([int(r.integers(1, 64)), int(r.integers(64, 5000)), int(r.integers(5000, 300000)),
                      262144, 1048576 + 14]))
    flag = int(r.integers(0, 2))
    n = k + m
    S = (B + k - 1) // k
    L = rsmi.lib()
    p = L.rsmi_host_alloc(n * S)
    assert p
    try:
        sh = np.ctypeslib.as_array((ctypes.c_uint8 * (n * S)).from_address(p)).reshape(n, S)
        block = r.integers(0, 256, size=B, dtype=np.uint8)
        full = orc.split(k, m, block.tobytes())
        full[k:] = orc.encode(k, m, full[:k])
        r16 = [orc.crc16_ibm(full[i].tobytes()) for i in range(n)]
        with rsmi.Codec(k, m) as c:
            c.set_option("coalesce_flag", flag)
            for rep in range(3):  # the flag slots reused
                sh[:] = 0x5A
                sh[:k] = full[:k]
                raw = np.zeros(n, dtype=np.uint32)
                c.encode_batch_host_crcs_ptr(p, n * S, p + k * S, n * S, S, 1, raw.ctypes.data, None)
                assert np.array_equal(sh, full), (k, m, B, rep)
                assert [rsmi.crc16_entry(b"", int(x), S) for x in raw] == r16, (k, m, B, rep)
                nlost = int(r.integers(1, m + 1))
                lost = sorted(int(x) for x in r.choice(n, size=nlost, replace=False))
                present = [i not in lost for i in range(n)]
                sh[lost] = 0xEE
                c.reconstruct_rows_batch_host_ptr(p, n * S, S, 1, present, [i in lost for i in range(n)])
                assert np.array_equal(sh, full), (k, m, B, lost)
                if any(i < k for i in lost):
                    sh[lost] = 0xEE
                    v16 = np.zeros(k, dtype=np.uint32)
                    c.reconstruct_batch_host_verify_ptr(p, n * S, S, 1, present, True, v16.ctypes.data)
                    for i in range(n):
                        if i < k or i not in lost:
                            assert np.array_equal(sh[i], full[i]), (k, m, B, lost, i)
                    used = [i for i in range(n) if present[i]][:k]
                    assert [rsmi.crc16_entry(b"", int(v16[j]), S) for j in range(k)] == [r16[i] for i in used]
    finally:
        L.rsmi_host_free(p)
