"""Datanode entry checksum (dag/node/datanode/server.go:58-75, howeyc/crc16 IBMTable) and
its GPU split (include/rsmi.h "datanode CRC-16").

CPU tests pin the byte-serial oracle (crc16_oracle.c) to the CRC-16/USB check value and
prove the host half of the split -- rsmi_crc16_entry folding a 12-byte entry header onto
R(data) -- against the oracle's whole-entry checksum, with R(data) computed here in pure
Python.  GPU tests check the device R(row) kernel and the encode+CRC host batches against
the oracle byte for byte.  The CRC variant itself is parity-unpinned (no reference test
holds a value)."""
import ctypes
import random

import numpy as np
import pytest

import oracle_lib as orc
import rsmi
from rsmi import multi

_T = []


def _table():
    if not _T:
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ 0xA001 if c & 1 else c >> 1
            _T.append(c)
    return _T


def raw_crc(data: bytes, s: int = 0) -> int:
    """R(D): the register after D from s (no complement) -- pure-Python byte loop."""
    T = _table()
    for b in data:
        s = T[(s ^ b) & 0xFF] ^ (s >> 8)
    return s


def test_oracle_check_value():
    assert orc.crc16_ibm(b"123456789") == 0xB4C8  # CRC-16/USB catalogue check
    assert orc.crc16_ibm(b"") == 0x0000  # ~(~0) with no bytes
    assert orc.crc16_ibm(b"123456789") == multi.crc16_ibm(b"123456789")


def test_library_checksum_matches_oracle():
    r = random.Random(11)
    for n in [0, 1, 2, 15, 16, 17, 255, 256, 257, 272, 1024, 4099, 26215, 26227, 104858]:
        b = bytes(r.randrange(256) for _ in range(n))
        assert rsmi.crc16_ibm(b) == orc.crc16_ibm(b), n


def test_oracle_entry_crc_is_checksum_of_framed_entry():
    meta = (262144).to_bytes(4, "little")
    data = bytes(range(200))
    framed = orc.entry_head(meta, len(data)) + data
    assert orc.datanode_entry_crc(meta, data) == orc.crc16_ibm(framed)


@pytest.mark.parametrize("n", [0, 1, 3, 16, 1023, 1024, 1025, 26215, 40000])
def test_entry_from_raw_matches_oracle(n):
    """rsmi_crc16_entry(head, R(D), |D|) == Checksum(head || D): the host half of the split,
    including shifts past the 32767-byte order of the zero-byte map."""
    r = random.Random(n)
    data = bytes(r.randrange(256) for _ in range(n))
    meta = (n * 10 + 3).to_bytes(4, "little")
    head = orc.entry_head(meta, n)
    assert rsmi.crc16_entry(head, raw_crc(data), n) == orc.datanode_entry_crc(meta, data)
    assert rsmi.crc16_entry(b"", raw_crc(data), n) == orc.crc16_ibm(data)


def test_raw_crc_is_linear():
    """R(D1 || D2) = A^|D2|(R(D1)) ^ R(D2): the identity the GPU combine rests on."""
    r = random.Random(3)
    d1 = bytes(r.randrange(256) for _ in range(37))
    d2 = bytes(r.randrange(256) for _ in range(91))
    shifted = raw_crc(b"\0" * len(d2), raw_crc(d1))
    assert raw_crc(d1 + d2) == shifted ^ raw_crc(d2)


def _device_rows(nb, nrows, S, pitch, offset, seed):
    import torch

    g = torch.Generator().manual_seed(seed)
    bs = nrows * pitch
    host = torch.randint(0, 256, (offset + nb * bs + 64,), dtype=torch.uint8, generator=g)
    return host, host.to("cuda")


@pytest.mark.gpu
@pytest.mark.parametrize("S", [1, 7, 15, 16, 17, 1000, 1024, 1025, 4095, 4097, 8191, 8192, 8193, 26215, 32767, 32768,
                               32769, 36865, 65536, 104858, 262144, 1048579])
@pytest.mark.parametrize("layout", ["aligned", "unaligned"])
@pytest.mark.parametrize("wpc", [0, 1])
@pytest.mark.parametrize("fold", [1, 0])
def test_rows_dev_matches_oracle(S, layout, wpc, fold):
    """Fold 1 (the default) runs the matrix-core pass -- on unaligned rows with aligned loads
    funnel-shifted by the row's misalignment --, fold 0 the nibble passes (pipelined on aligned
    rows); waves_per_cu=1 makes each wave walk many items (the pipelined pass's two register sets
    alternate).  Row sizes cover half-group, group (8 KiB) and item (32 KiB) boundaries on both
    sides; unaligned rows sit at pitch S + 3 from offset 5, so their misalignments vary."""
    import torch

    nrows, nb = 3, 5
    if layout == "aligned":
        pitch, off = (S + 15) // 16 * 16 + 16, 0
    else:
        pitch, off = S + 3, 5
    host, dev = _device_rows(nb, nrows, S, pitch, off, S)
    out = torch.full((nb, nrows + 1), 0xDEAD, dtype=torch.int32, device="cuda")
    with rsmi.Codec(4, 2) as c:
        c.set_option("waves_per_cu", wpc)
        c.set_option("crc16_fold", fold)
        c.crc16_rows_dev(dev.data_ptr() + off, pitch, nrows * pitch, nrows, S, nb, out.data_ptr(), nrows + 1)
        torch.cuda.synchronize()
    got = out.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
    h = host.numpy()
    for b in range(nb):
        assert got[b, nrows] == 0xDEAD  # slots past nrows untouched
        for r in range(nrows):
            row = h[off + b * nrows * pitch + r * pitch:][:S].tobytes()
            assert got[b, r] < 0x10000
            assert rsmi.crc16_entry(b"", int(got[b, r]), S) == orc.crc16_ibm(row), (b, r)


@pytest.mark.gpu
@pytest.mark.parametrize("S", [1, 15, 16, 17, 1023, 1024, 1040, 8191, 8193, 26215, 32761, 32768, 104858])
def test_rows_dev_split_layout_every_misalignment(S):
    """The Split layout (rows back to back at pitch S) from each of the 16 byte offsets of an
    aligned base: every row misalignment (0..15) of the matrix-core pass's memory-grid fold
    (leading bytes masked, rows reaching one tile, group or item further on the memory grid, the
    end shift by the misalignment), against the oracle."""
    import torch

    nrows, nb = 4, 3
    for off in range(16):
        host, dev = _device_rows(nb, nrows, S, S, off, S * 7 + off)
        out = torch.zeros((nb, nrows), dtype=torch.int32, device="cuda")
        with rsmi.Codec(4, 2) as c:
            c.crc16_rows_dev(dev.data_ptr() + off, S, nrows * S, nrows, S, nb, out.data_ptr(), nrows)
            torch.cuda.synchronize()
            assert c.last_kernel() == ("rs_crc16_rows_kernel,MFMA" if (off % 16 == 0 and S % 16 == 0) else
                                       "rs_crc16_rows_kernel,MFMA,UA"), c.last_kernel()
        got = out.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
        h = host.numpy()
        for b in range(nb):
            for r in range(nrows):
                row = h[off + (b * nrows + r) * S:][:S].tobytes()
                assert rsmi.crc16_entry(b"", int(got[b, r]), S) == orc.crc16_ibm(row), (off, b, r)


@pytest.mark.gpu
def test_rows_dev_random_shapes_both_folds():
    """40 random aligned geometries (row length, rows per block, blocks, pitch and block stride
    with random 16-byte padding): the matrix-core and the nibble folds give the oracle's R(row)
    on every row."""
    import torch

    rng = random.Random(2026)
    for _ in range(40):
        S = rng.choice([rng.randrange(1, 2048), rng.randrange(2048, 70000), rng.randrange(70000, 300000)])
        nrows, nb = rng.randrange(1, 6), rng.randrange(1, 7)
        pitch = (S + 15) // 16 * 16 + 16 * rng.randrange(0, 4)
        bstride = nrows * pitch + 16 * rng.randrange(0, 3)
        g = torch.Generator().manual_seed(S)
        host = torch.randint(0, 256, (nb * bstride + 64,), dtype=torch.uint8, generator=g)
        dev = host.to("cuda")
        h = host.numpy()
        for fold in (1, 0):
            out = torch.zeros((nb, nrows), dtype=torch.int32, device="cuda")
            with rsmi.Codec(4, 2) as c:
                c.set_option("crc16_fold", fold)
                c.crc16_rows_dev(dev.data_ptr(), pitch, bstride, nrows, S, nb, out.data_ptr(), nrows)
                torch.cuda.synchronize()
            got = out.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
            for b in range(nb):
                for r in range(nrows):
                    row = h[b * bstride + r * pitch:][:S].tobytes()
                    assert rsmi.crc16_entry(b"", int(got[b, r]), S) == orc.crc16_ibm(row), (S, nrows, nb, fold, b, r)


@pytest.mark.gpu
def test_rows_dev_random_unaligned_shapes_both_folds():
    """40 random unaligned geometries (any base offset, pitch >= S and block stride at any byte
    granularity, so rows of one launch take many misalignments): the matrix-core pass's
    memory-grid fold and the nibble pass give the oracle's R(row) on every row."""
    import torch

    rng = random.Random(2027)
    for _ in range(40):
        S = rng.choice([rng.randrange(16, 2048), rng.randrange(2048, 70000), rng.randrange(70000, 200000)])
        nrows, nb = rng.randrange(1, 6), rng.randrange(1, 6)
        off = rng.randrange(0, 16)
        pitch = S + rng.randrange(0, 40)
        bstride = nrows * pitch + rng.randrange(0, 40)
        g = torch.Generator().manual_seed(S + off)
        host = torch.randint(0, 256, (off + nb * bstride + 64,), dtype=torch.uint8, generator=g)
        dev = host.to("cuda")
        h = host.numpy()
        for fold in (1, 0):
            out = torch.zeros((nb, nrows), dtype=torch.int32, device="cuda")
            with rsmi.Codec(4, 2) as c:
                c.set_option("crc16_fold", fold)
                c.crc16_rows_dev(dev.data_ptr() + off, pitch, bstride, nrows, S, nb, out.data_ptr(), nrows)
                torch.cuda.synchronize()
            got = out.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
            for b in range(nb):
                for r in range(nrows):
                    row = h[off + b * bstride + r * pitch:][:S].tobytes()
                    assert rsmi.crc16_entry(b"", int(got[b, r]), S) == orc.crc16_ibm(row), (S, off, pitch, bstride, fold, b, r)


@pytest.mark.gpu
@pytest.mark.parametrize("fold", [1, 0])
def test_rows_dev_full_size_batch(fold):
    """RS(10,4) 256 KiB geometry, 4096 blocks x 14 rows: a checksum of checksums against the
    oracle on a sample of rows, plus every row nonzero-tested against its own recompute."""
    import torch

    k, m, nb = 10, 4, 4096
    n, S = k + m, 26215
    pitch = rsmi.recommended_pitch(S)
    g = torch.Generator(device="cuda").manual_seed(9)
    dev = torch.randint(0, 256, (nb, n, pitch), dtype=torch.uint8, device="cuda", generator=g)
    out = torch.empty((nb, n), dtype=torch.int32, device="cuda")
    with rsmi.Codec(k, m) as c:
        c.set_option("crc16_fold", fold)
        c.crc16_rows_dev(dev.data_ptr(), pitch, n * pitch, n, S, nb, out.data_ptr(), n)
        torch.cuda.synchronize()
        assert c.last_kernel() == ("rs_crc16_rows_kernel,MFMA" if fold else "rs_crc16_rows_kernel")
    got = out.cpu().numpy()
    rng = random.Random(1)
    for _ in range(64):
        b, r = rng.randrange(nb), rng.randrange(n)
        row = dev[b, r, :S].cpu().numpy().tobytes()
        assert rsmi.crc16_entry(b"", int(got[b, r]) & 0xFFFF, S) == orc.crc16_ibm(row)


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,B", [(2, 1, 6), (4, 2, 262144), (10, 4, 262144), (10, 4, 1048576), (16, 4, 65536 + 7)])
@pytest.mark.parametrize("small", [0, 1 << 30])
def test_encode_batch_host_crc_entries_match_oracle(k, m, B, small):
    """Every shard's datanode entry checksum from the GPU split equals server.go:70 on the
    oracle's shards."""
    n = k + m
    S = (B + k - 1) // k
    nb = 6
    r = np.random.default_rng(B + k)
    data = np.zeros((nb, k * S), dtype=np.uint8)
    data[:, :B] = r.integers(0, 256, size=(nb, B), dtype=np.uint8)
    par = np.zeros((nb, m * S), dtype=np.uint8)
    raw = np.zeros((nb, n), dtype=np.uint32)
    with rsmi.Codec(k, m) as c:
        c.set_option("small_call_bytes", small)  # copy-engine pipeline / zero-copy single kernel
        c.encode_batch_host_crc_ptr(data.ctypes.data, k * S, par.ctypes.data, m * S, S, nb, raw.ctypes.data)
    meta = B.to_bytes(4, "little")
    head = orc.entry_head(meta, S)
    for b in range(nb):
        want_par = orc.encode(k, m, data[b].reshape(k, S))
        assert np.array_equal(par[b].reshape(m, S), want_par)
        rows = list(data[b].reshape(k, S)) + list(want_par)
        for i in range(n):
            assert rsmi.crc16_entry(head, int(raw[b, i]), S) == orc.datanode_entry_crc(meta, rows[i].tobytes()), (b, i)


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 6, 4099, 262144])
def test_encode_block_crc(B):
    k, m = 10, 4
    block = bytes(np.random.default_rng(B).integers(0, 256, size=B, dtype=np.uint8))
    with rsmi.Codec(k, m) as c:
        shards, raw = c.encode_block_crc(block)
    S = len(shards) // (k + m)
    for i in range(k + m):
        row = shards[i * S:(i + 1) * S]
        assert rsmi.crc16_entry(b"", raw[i], S) == orc.crc16_ibm(row)
    assert shards[:B] == block


@pytest.mark.gpu
def test_coalesced_encode_concurrent_callers():
    """rsmi_encode_block_coalesced from 16 threads at once (DagNode.Put's shape): every block's
    shards and raw CRCs equal the oracle's, mixed block sizes batch by shard size, and the
    calls were coalesced into fewer GPU batches than calls."""
    import threading

    k, m = 10, 4
    n = k + m
    rng = np.random.default_rng(21)
    sizes = [262144] * 40 + [262143] * 8 + [6, 1, 4099, 1048576]
    blocks = [bytes(rng.integers(0, 256, size=B, dtype=np.uint8)) for B in sizes]
    out = [None] * len(blocks)
    with rsmi.Codec(k, m) as c:
        c.set_option("coalesce_us", 200)
        nxt = [0]
        lock = threading.Lock()

        def worker():
            while True:
                with lock:
                    i = nxt[0]
                    nxt[0] += 1
                if i >= len(blocks):
                    return
                out[i] = c.encode_block_coalesced(blocks[i], want_raw=(i % 2 == 0))

        th = [threading.Thread(target=worker) for _ in range(16)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        calls, batches = c.stat("coalesced_calls"), c.stat("coalesced_batches")
    assert calls == len(blocks)
    assert 1 <= batches < calls
    for i, B in enumerate(sizes):
        S = (B + k - 1) // k
        got = out[i][0] if i % 2 == 0 else out[i]
        want = orc.split(k, m, blocks[i])
        want[k:] = orc.encode(k, m, want[:k])
        assert got == want.tobytes(), i
        if i % 2 == 0:
            for r in range(n):
                assert rsmi.crc16_entry(b"", out[i][1][r], S) == orc.crc16_ibm(want[r].tobytes())


@pytest.mark.gpu
def test_coalesced_encode_lone_caller_and_errors():
    with rsmi.Codec(4, 2) as c:
        assert c.encode_block_coalesced(b"123456") == c.encode_block(b"123456")
        with pytest.raises(rsmi.RsmiError) as e:
            c.encode_block_coalesced(b"")
        assert e.value.code == rsmi.ErrShortData
        assert c.stat("coalesced_batches") == 1


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,B", [(10, 4, 262144), (2, 1, 262144), (16, 4, 4194304), (4, 2, 6), (10, 4, 4099)])
def test_coalesced_lone_call_in_place_on_page_locked_buffer(k, m, B):
    """A lone coalesced encode or reconstruct whose shard buffer is page-locked (the host
    mirror's block scratch, DagNode.Put / a degraded Get, node.go:358-408 / :277-326) is coded
    in place by one zero-copy kernel instead of through the engine's staging: shards, raw
    CRC-16s and the rebuilt rows equal the oracle's, rows not asked for stay untouched."""
    import ctypes

    n = k + m
    S = (B + k - 1) // k
    L = rsmi.lib()
    block = bytes(np.random.default_rng(B + k).integers(0, 256, size=B, dtype=np.uint8))
    want = orc.split(k, m, block)
    want[k:] = orc.encode(k, m, want[:k])
    p = L.rsmi_host_alloc(n * S)
    assert p
    try:
        out = np.ctypeslib.as_array((ctypes.c_uint8 * (n * S)).from_address(p))
        out[:] = 0xA5  # stale bytes: the padding and parity must be written, not assumed zero
        raw = (ctypes.c_uint32 * n)()
        with rsmi.Codec(k, m) as c:
            src = bytearray(block)
            assert L.rsmi_encode_block_coalesced(c._h, ctypes.addressof((ctypes.c_char * B).from_buffer(src)), B, p,
                                                 raw) == 0
            assert np.array_equal(out.reshape(n, S), want)
            for r in range(n):
                assert rsmi.crc16_entry(b"", raw[r], S) == orc.crc16_ibm(want[r].tobytes())
            assert c.stat("coalesced_batches") == 1
            for lost, data_only in (([0], True), ([1, n - 1] if m >= 2 else [n - 1], False)):
                sh = out.reshape(n, S)
                sh[:] = want
                for r in lost:
                    sh[r] = 0xEE
                present = (ctypes.c_uint8 * n)(*[0 if r in lost else 1 for r in range(n)])
                assert L.rsmi_reconstruct_coalesced(c._h, p, S, present, 1 if data_only else 0) == 0
                for r in range(n):
                    if r in lost and (r < k or not data_only):
                        assert np.array_equal(sh[r], want[r]), (lost, r)
                    elif r in lost:
                        assert (sh[r] == 0xEE).all()
                    else:
                        assert np.array_equal(sh[r], want[r])
    finally:
        L.rsmi_host_free(p)


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["coalesced", "one_block", "reconstruct"])
@pytest.mark.parametrize("k,m,B", [(10, 4, 262144), (2, 1, 262144), (10, 4, 4099)])
def test_wait_hook_runs_once_inside_the_call(path, k, m, B):
    """rsmi_set_wait_hook (DagNode.Put's data-shard writes beside the encode, node.go:376-399):
    the next coalesced encode or one-block host encode on this thread runs the hook exactly once,
    on this thread, while the kernel codes the block in place; the hook reads the final data rows
    meanwhile, and shards and R(shard) still equal the oracle's.  A call that fails before
    launching leaves the hook to rsmi_run_wait_hook.  "reconstruct": the one-block in-place
    ReconstructData of a lone degraded DagNode.Get (node.go:277-326), data row 0 lost; the hook
    reads the survivors while the kernel rebuilds row 0."""
    import threading

    n = k + m
    S = (B + k - 1) // k
    L = rsmi.lib()
    block = bytes(np.random.default_rng(B + 7 * k).integers(0, 256, size=B, dtype=np.uint8))
    want = orc.split(k, m, block)
    want[k:] = orc.encode(k, m, want[:k])
    p = L.rsmi_host_alloc(n * S)
    assert p
    try:
        out = np.ctypeslib.as_array((ctypes.c_uint8 * (n * S)).from_address(p))
        seen = []
        me = threading.get_ident()

        def hook(arg):
            seen.append((threading.get_ident(), bytes(out[: (B // S) * S])))

        cb = ctypes.CFUNCTYPE(None, ctypes.c_void_p)(hook)
        raw = (ctypes.c_uint32 * n)()
        with rsmi.Codec(k, m) as c:
            for rep in range(3):
                out[:] = 0xA5
                out[:B] = np.frombuffer(block, dtype=np.uint8)  # Split's copy, by the caller
                L.rsmi_set_wait_hook(cb, None)
                if path == "coalesced":
                    rc = L.rsmi_encode_block_coalesced_crcs(c._h, p, B, p, raw, None)
                elif path == "one_block":
                    out[B:k * S] = 0
                    rc = L.rsmi_encode_batch_host_crcs(c._h, p, n * S, p + k * S, n * S, S, 1, raw, None)
                else:
                    out.reshape(n, S)[:] = want
                    out[:S] = 0xEE  # data row 0 lost
                    present = (ctypes.c_uint8 * n)(*[0] + [1] * (n - 1))
                    rc = L.rsmi_reconstruct_batch_host(c._h, p, n * S, S, 1, present, 1)
                assert rc == 0
                assert L.rsmi_run_wait_hook() == 0  # the call took it
                assert len(seen) == rep + 1 and seen[-1][0] == me
                if path == "reconstruct":  # the survivors were as given (row 0 is the kernel's)
                    assert seen[-1][1][S:] == bytes(want[1: B // S].reshape(-1))
                else:
                    assert seen[-1][1] == bytes(want[: B // S].reshape(-1))  # the data rows were final
                assert np.array_equal(out.reshape(n, S), want)
                for r in range(n):
                    if path != "reconstruct":
                        assert rsmi.crc16_entry(b"", raw[r], S) == orc.crc16_ibm(want[r].tobytes())
            L.rsmi_set_wait_hook(cb, None)
            assert L.rsmi_encode_block_coalesced_crcs(c._h, p, 0, p, raw, None) == rsmi.ErrShortData
            assert len(seen) == 3
            assert L.rsmi_run_wait_hook() == 1 and len(seen) == 4
    finally:
        L.rsmi_host_free(p)


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,B", [(10, 4, 262144), (4, 2, 4099), (16, 4, 4194304)])
def test_coalesced_encode_split_by_caller_pageable(k, m, B):
    """rsmi_encode_block_coalesced with block == shards_out on pageable memory (the staging path
    of a coalesced group): the block at the start of the buffer is zero-padded and encoded, over
    stale bytes, with R(shard) of every shard, equal to the oracle."""
    import ctypes

    n = k + m
    S = (B + k - 1) // k
    L = rsmi.lib()
    block = np.random.default_rng(B + 3).integers(0, 256, size=B, dtype=np.uint8)
    want = orc.split(k, m, bytes(block))
    want[k:] = orc.encode(k, m, want[:k])
    buf = np.full(n * S, 0xA5, dtype=np.uint8)
    buf[:B] = block
    raw = (ctypes.c_uint32 * n)()
    with rsmi.Codec(k, m) as c:
        assert L.rsmi_encode_block_coalesced(c._h, buf.ctypes.data, B, buf.ctypes.data, raw) == 0
    assert np.array_equal(buf.reshape(n, S), want)
    for r in range(n):
        assert rsmi.crc16_entry(b"", raw[r], S) == orc.crc16_ibm(want[r].tobytes()), r


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,B", [(10, 4, 262144), (16, 4, 1048576 + 14), (2, 1, 4099), (4, 2, 262144)])
@pytest.mark.parametrize("split_by_caller", [False, True])
def test_coalesced_group_in_place_on_page_locked_buffers(k, m, B, split_by_caller):
    """Concurrent coalesced encodes and degraded reconstructs (DagNode.Put / Get from many
    goroutines, node.go:358-408, :277-326) whose shard buffers are each page-locked: the group is
    coded where the buffers lie, one zero-copy launch per request and one synchronisation, with
    no staging (an encode group with CRC-16s: one launch over a table of the blocks' bases,
    aligned for RS(4,2) 256 KiB, unaligned windows otherwise).  split_by_caller: each caller has
    copied its block to the start of its buffer
    and passes the buffer as the block too (include/rsmi.h: block == shards_out), as the host
    mirror does, over stale bytes in the padding and parity.  Every shard, raw CRC-16 and
    rebuilt row equals the oracle's, and the calls did coalesce."""
    import ctypes
    import threading

    n = k + m
    S = (B + k - 1) // k
    L = rsmi.lib()
    T = 12
    rng = np.random.default_rng(B)
    blocks = [bytes(rng.integers(0, 256, size=B, dtype=np.uint8)) for _ in range(T)]
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
            c.set_option("coalesce_us", 3000)
            c.set_option("coalesce_max", T)
            srcs = [bytearray(b) for b in blocks]
            rcs = [None] * T
            if split_by_caller:
                for t in range(T):
                    flat = views[t].reshape(-1)
                    flat[:] = 0xA5
                    flat[:B] = np.frombuffer(blocks[t], dtype=np.uint8)

            def enc(t):
                src = ptrs[t] if split_by_caller else ctypes.addressof((ctypes.c_char * B).from_buffer(srcs[t]))
                rcs[t] = L.rsmi_encode_block_coalesced(c._h, src, B, ptrs[t], raws[t])

            th = [threading.Thread(target=enc, args=(t,)) for t in range(T)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            assert rcs == [0] * T
            assert c.stat("coalesced_batches") < c.stat("coalesced_calls") == T
            for t in range(T):
                assert np.array_equal(views[t], want[t]), t
                for r in range(n):
                    assert rsmi.crc16_entry(b"", raws[t][r], S) == orc.crc16_ibm(want[t][r].tobytes()), (t, r)
            lost = [0, k] if m >= 2 else [0]
            present = (ctypes.c_uint8 * n)(*[0 if r in lost else 1 for r in range(n)])
            for t in range(T):
                views[t][lost] = 0xEE

            def rec(t):
                rcs[t] = L.rsmi_reconstruct_coalesced(c._h, ptrs[t], S, present, 0)

            th = [threading.Thread(target=rec, args=(t,)) for t in range(T)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            assert rcs == [0] * T
            for t in range(T):
                assert np.array_equal(views[t], want[t]), t
    finally:
        for p in ptrs:
            L.rsmi_host_free(p)


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,B,T,crc", [
    (10, 4, 262144, 12, True),      # unaligned windows (S = 26215), the fused kernel + its combine launch
    (10, 4, 262144, 4, True),       # 28 units: the fused kernel with the combine inside
    (10, 4, 262144, 1, True),       # a lone caller: one block through the table kernel too
    (16, 4, 4194304, 1, True),      # a lone 4 MiB block (the combine launch)
    (10, 4, 262144, 1, False),
    (10, 4, 262144, 12, False),     # the plain encode over the table
    (2, 1, 262144, 6, True),        # aligned rows (S = 131072)
    (4, 2, 4099, 80, True),         # more blocks than one table holds: two table launches
    (16, 4, 1048576 + 14, 5, True),
    (2, 1, 6, 8, True),             # S = 3: no table kernel (rows under 16 bytes), a launch per block
    (5, 3, 70000, 7, True),         # a shape without table kernels: a launch per block
])
def test_coalesced_table_launch(k, m, B, T, crc):
    """A coalesced group of T requests whose shard buffers are each page-locked (DagNode.Put and
    degraded Gets from many goroutines, node.go:358-408 / :220-326) is coded by one launch over a
    table of the blocks' bases (rs_fast_kernel / rs_fused_mfma_kernel TB, up to 64 blocks per
    launch): one lane and coalesce_us make the T calls one deterministic batch.  Every shard, raw
    CRC-16 and rebuilt row equals the oracle's, rows not asked for stay untouched, and the
    BASELINE shapes' batches ran the table kernels."""
    import ctypes
    import threading

    n = k + m
    S = (B + k - 1) // k
    L = rsmi.lib()
    rng = np.random.default_rng(B + T)
    blocks = [bytes(rng.integers(0, 256, size=B, dtype=np.uint8)) for _ in range(T)]
    want = []
    for b in blocks:
        w = orc.split(k, m, b)
        w[k:] = orc.encode(k, m, w[:k])
        want.append(w)
    ptrs = [L.rsmi_host_alloc(n * S) for _ in range(T)]
    assert all(ptrs)
    table = S >= 16 and (k, m) in ((2, 1), (4, 2), (10, 4), (16, 4))
    try:
        views = [np.ctypeslib.as_array((ctypes.c_uint8 * (n * S)).from_address(p)).reshape(n, S) for p in ptrs]
        raws = [(ctypes.c_uint32 * n)() for _ in range(T)]
        with rsmi.Codec(k, m) as c:
            c.set_option("coalesce_lanes", 1)
            c.set_option("coalesce_us", 100000)
            c.set_option("coalesce_max", T)
            c.warm()
            b0 = c.stat("coalesced_batches")
            rcs = [None] * T
            for t in range(T):
                flat = views[t].reshape(-1)
                flat[:] = 0xA5  # stale bytes: padding and parity must be written
                flat[:B] = np.frombuffer(blocks[t], dtype=np.uint8)

            def enc(t):
                rcs[t] = L.rsmi_encode_block_coalesced(c._h, ptrs[t], B, ptrs[t], raws[t] if crc else None)

            th = [threading.Thread(target=enc, args=(t,)) for t in range(T)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            assert rcs == [0] * T
            assert c.stat("coalesced_batches") - b0 == 1
            assert (",TB" in c.last_kernel()) == table, c.last_kernel()
            for t in range(T):
                assert np.array_equal(views[t], want[t]), t
                for r in range(n if crc else 0):
                    assert rsmi.crc16_entry(b"", raws[t][r], S) == orc.crc16_ibm(want[t][r].tobytes()), (t, r)
            for lost, data_only in (([0], True), ([1, n - 1] if m >= 2 else [n - 1], False)):
                present = (ctypes.c_uint8 * n)(*[0 if r in lost else 1 for r in range(n)])
                for t in range(T):
                    views[t][:] = want[t]
                    views[t][lost] = 0xEE

                def rec(t):
                    rcs[t] = L.rsmi_reconstruct_coalesced(c._h, ptrs[t], S, present, 1 if data_only else 0)

                b0 = c.stat("coalesced_batches")
                th = [threading.Thread(target=rec, args=(t,)) for t in range(T)]
                for x in th:
                    x.start()
                for x in th:
                    x.join()
                assert rcs == [0] * T
                assert c.stat("coalesced_batches") - b0 == 1
                if any(r < k or not data_only for r in lost):
                    assert (",TB" in c.last_kernel()) == table, c.last_kernel()
                for t in range(T):
                    for r in range(n):
                        if r in lost and (r < k or not data_only):
                            assert np.array_equal(views[t][r], want[t][r]), (t, lost, r)
                        elif r in lost:
                            assert (views[t][r] == 0xEE).all(), (t, r)
                        else:
                            assert np.array_equal(views[t][r], want[t][r]), (t, r)
    finally:
        for p in ptrs:
            L.rsmi_host_free(p)


@pytest.mark.gpu
@pytest.mark.parametrize("lanes", [1, 2, 4])
def test_coalesced_lanes_concurrent_callers(lanes):
    """Concurrent coalesced encodes with CRC-16s and degraded reconstructs from 24 threads over 1,
    2 or 4 coalescing lanes (each lane i > 0 a child context with its own stream and scratch):
    batches on different lanes run at once, and every result equals the oracle's."""
    import ctypes
    import threading

    k, m, B = 10, 4, 65536 + 7
    n = k + m
    S = (B + k - 1) // k
    L = rsmi.lib()
    T, per = 24, 6
    rng = np.random.default_rng(lanes)
    blocks = [bytes(rng.integers(0, 256, size=B, dtype=np.uint8)) for _ in range(T * per)]
    ptrs = [L.rsmi_host_alloc(n * S) for _ in range(T)]
    assert all(ptrs)
    errors = []
    try:
        views = [np.ctypeslib.as_array((ctypes.c_uint8 * (n * S)).from_address(p)).reshape(n, S) for p in ptrs]
        with rsmi.Codec(k, m) as c:
            c.set_option("coalesce_lanes", lanes)
            c.warm()
            present = (ctypes.c_uint8 * n)(*[0 if r == 3 else 1 for r in range(n)])

            def work(t):
                raw = (ctypes.c_uint32 * n)()
                for j in range(per):
                    i = t * per + j
                    w = orc.split(k, m, blocks[i])
                    w[k:] = orc.encode(k, m, w[:k])
                    flat = views[t].reshape(-1)
                    flat[:B] = np.frombuffer(blocks[i], dtype=np.uint8)
                    if L.rsmi_encode_block_coalesced(c._h, ptrs[t], B, ptrs[t], raw):
                        errors.append(("enc", i))
                        return
                    if not np.array_equal(views[t], w):
                        errors.append(("shards", i))
                    for r in range(n):
                        if rsmi.crc16_entry(b"", raw[r], S) != orc.crc16_ibm(w[r].tobytes()):
                            errors.append(("crc", i, r))
                    views[t][3] = 0
                    if L.rsmi_reconstruct_coalesced(c._h, ptrs[t], S, present, 1):
                        errors.append(("rec", i))
                        return
                    if not np.array_equal(views[t], w):
                        errors.append(("rebuilt", i))

            th = [threading.Thread(target=work, args=(t,)) for t in range(T)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            assert c.stat("coalesced_calls") == 2 * T * per  # rsmi_warm codes outside the queue
    finally:
        for p in ptrs:
            L.rsmi_host_free(p)
    assert errors == []


@pytest.mark.gpu
def test_coalesced_host_fault_reports_err_host():
    """A coalesced batch whose executor throws std::bad_alloc (option "inject_host_fault") fails
    its requests with RSMI_ERR_HOST, the status the boundary gives host-resource exceptions
    (include/rsmi.h), not a device error; the queue keeps working afterwards, for encode and
    for reconstruct (the degraded DagNode.Get's coalesced form, node.go:220-326)."""
    k, m = 4, 2
    block = b"123456" * 1000
    with rsmi.Codec(k, m) as c:
        c.set_option("inject_host_fault", 2)
        with pytest.raises(rsmi.RsmiError) as e:
            c.encode_block_coalesced(block)
        assert e.value.code == rsmi.ErrHost
        sh = orc.split(k, m, block)
        sh[k:] = orc.encode(k, m, sh[:k])
        work = bytearray(sh.tobytes())
        S = sh.shape[1]
        work[0:S] = bytes(S)
        present = [r != 0 for r in range(k + m)]
        with pytest.raises(rsmi.RsmiError) as e:
            c.reconstruct_coalesced(work, S, present, True)
        assert e.value.code == rsmi.ErrHost
        assert c.encode_block_coalesced(block) == c.encode_block(block)
        c.reconstruct_coalesced(work, S, present, True)
        assert bytes(work) == sh.tobytes()


@pytest.mark.gpu
def test_set_option_after_failed_lane_open():
    """A coalescing lane whose context fails to open (option "inject_lane_fault") leaves a null
    lane slot; rsmi_set_option must skip it rather than lock through it, and the
    context keeps coding: the lane opens on the next warm-up, every option reaches it, and the
    coalesced encode still equals the plain one."""
    k, m = 4, 2
    block = bytes(range(256)) * 64
    with rsmi.Codec(k, m) as c:
        c.set_option("coalesce_lanes", 3)
        c.set_option("inject_lane_fault", 1)
        with pytest.raises(rsmi.RsmiError) as e:
            c.warm()  # lane 0 is the context itself; lane 1's open fails, so warm stops there
        assert e.value.code == rsmi.ErrDevice
        for key, value in (("waves_per_cu", 0), ("crc16_fold", 1), ("coalesce_flag", 1)):
            c.set_option(key, value)
        c.warm()  # lane 1 opens now, then lane 2
        c.set_option("waves_per_cu", 0)
        assert c.encode_block_coalesced(block) == c.encode_block(block)


@pytest.mark.gpu
def test_coalesced_reconstruct_concurrent_callers():
    """rsmi_reconstruct_coalesced from 16 threads (concurrent degraded DagNode.Gets): two
    erasure patterns, both data_only modes and two shard sizes in flight together; every
    rebuilt row equals the original, present rows are untouched."""
    import threading

    k, m = 10, 4
    n = k + m
    rng = np.random.default_rng(5)
    jobs = []
    for i in range(48):
        B = 262144 if i % 3 else 4099
        block = bytes(rng.integers(0, 256, size=B, dtype=np.uint8))
        sh = orc.split(k, m, block)
        sh[k:] = orc.encode(k, m, sh[:k])
        lost = [0] if i % 2 else [3, 11]
        data_only = i % 4 != 1
        work = sh.copy()
        for r in lost:
            work[r] = 0
        jobs.append((sh, bytearray(work.tobytes()), [r not in lost for r in range(n)], data_only, lost))
    with rsmi.Codec(k, m) as c:
        c.set_option("coalesce_us", 200)
        nxt = [0]
        lock = threading.Lock()

        def worker():
            while True:
                with lock:
                    i = nxt[0]
                    nxt[0] += 1
                if i >= len(jobs):
                    return
                sh, work, present, data_only, _ = jobs[i]
                c.reconstruct_coalesced(work, sh.shape[1], present, data_only)

        th = [threading.Thread(target=worker) for _ in range(16)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert c.stat("coalesced_batches") < c.stat("coalesced_calls") == len(jobs)
    for sh, work, present, data_only, lost in jobs:
        got = np.frombuffer(bytes(work), dtype=np.uint8).reshape(n, -1)
        for r in range(n):
            if present[r]:
                assert np.array_equal(got[r], sh[r])
            elif r < k or not data_only:
                assert np.array_equal(got[r], sh[r]), (lost, data_only, r)
            else:
                assert not got[r].any()  # ReconstructData leaves missing parity alone


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,S,nb,layout", [(10, 4, 26215, 64, "pitched"), (10, 4, 26215, 9, "split"),
                                             (4, 2, 65536, 8, "pitched"), (16, 4, 4097, 5, "split"),
                                             (3, 2, 7, 6, "split"), (20, 4, 333, 3, "split"),
                                             (10, 4, 26215, 700, "pitched"), (10, 4, 104858, 5, "split"),
                                             (16, 4, 262144, 3, "pitched"), (2, 1, 17, 9, "split"),
                                             (2, 1, 16, 9, "split"), (5, 3, 1000, 7, "pitched"),
                                             (6, 6, 5000, 4, "split"), (12, 4, 1, 5, "pitched"),
                                             (1, 1, 33, 5, "split"), (8, 4, 65535, 3, "padded")])
@pytest.mark.parametrize("opts", [[("crc16_fused_fold", 1)], [("crc16_fused_fold", 0)],
                                  [("crc16_fused_fold", 0), ("waves_per_cu", 1)]])
def test_encode_batch_dev_crc_fused(k, m, S, nb, layout, opts):
    """Device-resident encode with the CRC fused into the encode pass: parity and every row's
    R(row) equal the oracle's (k > 16, m > 4, and S < 16 in unaligned layouts take the separate
    CRC pass).  Row padding in pitched layouts holds garbage, which must not reach the CRC.
    crc16_fused_fold 1: aligned layouts and unaligned ones with S >= 16 fold on the matrix cores
    (rs_fused_mfma_kernel, ",UA" on the latter), 0: the nibble-table variants; waves_per_cu=1 makes every nibble-fold wave code many tiles and every
    combine wave many blocks."""
    import torch

    n = k + m
    rs = {"pitched": rsmi.recommended_pitch(S), "split": S, "padded": (S + 15) // 16 * 16 + 32}[layout]
    data = np.random.default_rng(S + k).integers(0, 256, size=(nb, k, S), dtype=np.uint8)
    host = np.random.default_rng(5).integers(0, 256, size=(nb, n, rs), dtype=np.uint8)  # garbage padding
    host[:, :k, :S] = data
    d = torch.from_numpy(host.reshape(-1).copy()).cuda()
    raw = torch.zeros((nb, n), dtype=torch.int32, device="cuda")
    base = d.data_ptr()
    with rsmi.Codec(k, m) as c:
        for opt in opts:
            c.set_option(*opt)
        c.encode_batch_dev_crc(base, rs, n * rs, base + k * rs, rs, n * rs, S, nb, raw.data_ptr(),
                               torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        kern = c.last_kernel()
    got = d.cpu().numpy().reshape(nb, n, rs)
    want = orc.encode_fast(k, m, data)
    assert np.array_equal(got[:, k:, :S], want)
    if k <= 16 and m <= 4 and (S >= 16 or rs % 16 == 0):
        if opts[0][1] == 1:
            assert kern.startswith("rs_fused_mfma_kernel"), kern
            assert (",UA" in kern) == (rs % 16 != 0), kern
        else:
            assert ",CRC" in kern, kern
            assert (",UA" in kern) == (rs % 16 != 0), kern
    r = raw.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
    for b in range(nb):
        rows = list(data[b]) + list(want[b])
        for i in range(n):
            assert r[b, i] < 0x10000
            assert rsmi.crc16_entry(b"", int(r[b, i]), S) == orc.crc16_ibm(rows[i].tobytes()), (b, i)


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,B", [(10, 4, 262144), (2, 1, 262144), (4, 2, 262144), (16, 4, 4194304), (10, 4, 1048576),
                                   (10, 4, 4096), (16, 4, 65536), (10, 4, 65536)])
@pytest.mark.parametrize("layout", ["pitched", "split"])
def test_fused_inline_combine_small_launches(k, m, B, layout):
    """A fused encode + CRC-16 launch of at most kFusedInlineUnits (64) units -- DagNode.Put's
    per-block call, node.go:358-408 with server.go:57-80's checksum -- combines its records in
    the kernel (",INL": the block's last unit, found by a per-block counter that wraps back to
    zero; blocks of one unit, 4 KiB and 64 KiB RS(16,4), skip the counter) instead of a second
    launch.  Repeated launches (the counters must be back at zero), 1..N blocks, and a launch just
    past the limit (the two-launch form) all give the oracle's parity and R(row)."""
    import torch

    n = k + m
    S = (B + k - 1) // k
    tpb = ((S + 15) // 16 + 63) // 64
    upb = (tpb + 3) // 4
    rs = rsmi.recommended_pitch(S) if layout == "pitched" else S
    nb_max = 64 // upb
    for nb in sorted({1, 2, max(1, nb_max), nb_max + 1}):
        data = np.random.default_rng(nb + S).integers(0, 256, size=(nb, k, S), dtype=np.uint8)
        host = np.zeros((nb, n, rs), dtype=np.uint8)
        host[:, :k, :S] = data
        want = orc.encode_fast(k, m, data)
        with rsmi.Codec(k, m) as c:
            for rep in range(3):
                d = torch.from_numpy(host.reshape(-1).copy()).cuda()
                raw = torch.zeros((nb, n), dtype=torch.int32, device="cuda")
                base = d.data_ptr()
                c.encode_batch_dev_crc(base, rs, n * rs, base + k * rs, rs, n * rs, S, nb, raw.data_ptr(),
                                       torch.cuda.current_stream().cuda_stream)
                torch.cuda.synchronize()
                kern = c.last_kernel()
                assert kern.startswith("rs_fused_mfma_kernel"), kern
                assert (",INL" in kern) == (nb * upb <= 64), (nb, kern)
                got = d.cpu().numpy().reshape(nb, n, rs)
                assert np.array_equal(got[:, k:, :S], want), (nb, rep)
                r = raw.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
                for b in range(nb):
                    rows = list(data[b]) + list(want[b])
                    for i in range(n):
                        assert rsmi.crc16_entry(b"", int(r[b, i]), S) == orc.crc16_ibm(rows[i].tobytes()), (nb, rep, b, i)


@pytest.mark.gpu
@pytest.mark.parametrize("pinned", [True, False])
def test_host_calls_crc_readback(pinned):
    """Host calls that read the row CRCs back by kernel into the context's page-locked area (no
    blocking copy after the sync), twice on one context: encode with both CRCs, the rows-CRC
    call, the verified reconstruct and the rows rebuild with CRCs all equal the oracle, over
    page-locked and pageable shards (DagNode.Put / Get / RepairDataNode, node.go:358-408,
    :220-326, data_recovery.go:16-112)."""
    k, m, S, nb = 10, 4, 26215, 3
    n = k + m
    data = np.random.default_rng(7 * pinned).integers(0, 256, size=(nb, k, S), dtype=np.uint8)
    full = np.concatenate([data, orc.encode_fast(k, m, data)], axis=1)
    r16 = [[orc.crc16_ibm(full[b, r].tobytes()) for r in range(n)] for b in range(nb)]
    r32 = [[orc.crc32_ieee(full[b, r].tobytes()) for r in range(n)] for b in range(nb)]
    ptr = rsmi.lib().rsmi_host_alloc(nb * n * S) if pinned else None
    try:
        sh = (np.ctypeslib.as_array((ctypes.c_uint8 * (nb * n * S)).from_address(ptr)).reshape(nb, n, S)
              if pinned else np.empty((nb, n, S), dtype=np.uint8))
        with rsmi.Codec(k, m) as c:
            for rounds in range(2):
                sh[:] = 0
                sh[:, :k] = data
                a16 = np.zeros((nb, n), dtype=np.uint32)
                a32 = np.zeros((nb, n), dtype=np.uint32)
                c.encode_batch_host_crcs_ptr(sh.ctypes.data, n * S, sh.ctypes.data + k * S, n * S, S, nb,
                                             a16.ctypes.data, a32.ctypes.data)
                assert np.array_equal(sh, full)
                for b in range(nb):
                    for r in range(n):
                        assert rsmi.crc16_entry(b"", int(a16[b, r]), S) == r16[b][r], (b, r)
                        assert rsmi.crc32_entry(b"", int(a32[b, r]), S) == r32[b][r], (b, r)
                c16 = np.zeros(nb * n, dtype=np.uint32)
                c32 = np.zeros(nb * n, dtype=np.uint32)
                c.crc_rows_host_ptr(sh.ctypes.data, S, nb * n, S, c16.ctypes.data, c32.ctypes.data)
                for b in range(nb):
                    for r in range(n):
                        assert rsmi.crc16_entry(b"", int(c16[b * n + r]), S) == r16[b][r], (b, r)
                        assert rsmi.crc32_entry(b"", int(c32[b * n + r]), S) == r32[b][r], (b, r)
                lost = [2, 11]
                present = [i not in lost for i in range(n)]
                sh[:, lost] = 0
                v16 = np.zeros((nb, k), dtype=np.uint32)
                c.reconstruct_batch_host_verify_ptr(sh.ctypes.data, n * S, S, nb, present, False, v16.ctypes.data)
                assert np.array_equal(sh, full)
                used = [i for i in range(n) if present[i]][:k]
                for b in range(nb):
                    for j, r in enumerate(used):
                        assert rsmi.crc16_entry(b"", int(v16[b, j]), S) == r16[b][r], (b, j)
                sh[:, lost] = 0
                e16 = np.zeros((nb, n), dtype=np.uint32)
                e32 = np.zeros((nb, n), dtype=np.uint32)
                c.reconstruct_rows_batch_host_crcs_ptr(sh.ctypes.data, n * S, S, nb, present,
                                                       [i in lost for i in range(n)], e16.ctypes.data, e32.ctypes.data)
                assert np.array_equal(sh, full)
                for b in range(nb):
                    for r in lost:
                        assert rsmi.crc16_entry(b"", int(e16[b, r]), S) == r16[b][r], (b, r)
                        assert rsmi.crc32_entry(b"", int(e32[b, r]), S) == r32[b][r], (b, r)
            del sh
    finally:
        if pinned:
            rsmi.lib().rsmi_host_free(ptr)


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,S,nb,lost,pinned", [(10, 4, 26215, 24, [0], True), (10, 4, 26215, 24, [3, 11], False),
                                                  (10, 4, 26215, 9, [2, 5, 7, 9], True), (4, 2, 65536, 8, [1], True),
                                                  (16, 4, 4097, 5, [0, 15], True), (3, 2, 7, 6, [1], True),
                                                  (20, 4, 333, 3, [4], True), (10, 4, 26215, 4, [], True),
                                                  (10, 4, 26215, 4, [12], True), (2, 1, 16, 7, [0], True)])
def test_reconstruct_verify_survivor_crcs(k, m, S, nb, lost, pinned):
    """rsmi_reconstruct_batch_host_verify: the rebuild equals the oracle's and raw16[b*k + c] is
    R of survivor used[c] (the first k present rows), whether one fused kernel read page-locked
    shards (k <= 16, rows >= 16 B) or the separate pass ran (pageable, k > 16, S < 16, nothing
    to rebuild)."""
    n = k + m
    data = np.random.default_rng(S + k + len(lost)).integers(0, 256, size=(nb, k, S), dtype=np.uint8)
    full = np.concatenate([data, orc.encode_fast(k, m, data)], axis=1)
    present = [i not in lost for i in range(n)]
    used = [i for i in range(n) if present[i]][:k]
    with rsmi.Codec(k, m) as c:
        if pinned:
            ptr = rsmi.lib().rsmi_host_alloc(nb * n * S)
            sh = np.ctypeslib.as_array((ctypes.c_uint8 * (nb * n * S)).from_address(ptr)).reshape(nb, n, S)
        else:
            sh = np.empty((nb, n, S), dtype=np.uint8)
        try:
            sh[:] = full
            sh[:, lost] = 0
            raw = np.zeros((nb, k), dtype=np.uint32)
            c.reconstruct_batch_host_verify_ptr(sh.ctypes.data, n * S, S, nb, present, False, raw.ctypes.data)
            kern = c.last_kernel()
            assert np.array_equal(sh, full)
            if pinned and lost and k <= 16 and S >= 16:
                # one fused kernel: the matrix-core fold (",UA" when rows are not on the 16-byte grid)
                assert kern.startswith("rs_fused_mfma_kernel"), kern
                assert (",UA" in kern) == (S % 16 != 0), kern
            for b in range(nb):
                for j, r in enumerate(used):
                    assert rsmi.crc16_entry(b"", int(raw[b, j]), S) == orc.crc16_ibm(full[b, r].tobytes()), (b, j)
        finally:
            if pinned:
                del sh
                rsmi.lib().rsmi_host_free(ptr)


@pytest.mark.gpu
@pytest.mark.parametrize("k,m", [(10, 4), (16, 4), (1, 1), (2, 1), (3, 2), (4, 2), (12, 3), (5, 1)])
@pytest.mark.parametrize("fill", ["ones", "zeros", "random"])
def test_fused_mfma_counts_exact(k, m, fill):
    """rs_fused_mfma_kernel packs two shards into one f32 accumulator (the odd one scaled by
    2^12) and reads both parities once per 4-tile unit: all-0xFF rows drive every count to its
    maximum, so any inexact accumulation shows.  Row sizes cross the unit boundary (4 tiles =
    4 KiB per row), end inside and on a chunk, and leave the last unit 1..4 tiles long."""
    import torch

    n = k + m
    for S in (1, 15, 16, 1023, 1024, 4096, 4097, 5000, 16384, 26215):
        nb = 5
        rs = rsmi.recommended_pitch(S)
        if fill == "ones":
            data = np.full((nb, k, S), 0xFF, dtype=np.uint8)
        elif fill == "zeros":
            data = np.zeros((nb, k, S), dtype=np.uint8)
        else:
            data = np.random.default_rng(S * 31 + k).integers(0, 256, size=(nb, k, S), dtype=np.uint8)
        host = np.full((nb, n, rs), 0xA5, dtype=np.uint8)  # padding that must not reach the CRC
        host[:, :k, :S] = data
        d = torch.from_numpy(host.reshape(-1).copy()).cuda()
        raw = torch.zeros((nb, n), dtype=torch.int32, device="cuda")
        with rsmi.Codec(k, m) as c:
            c.encode_batch_dev_crc(d.data_ptr(), rs, n * rs, d.data_ptr() + k * rs, rs, n * rs, S, nb,
                                   raw.data_ptr(), torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            assert c.last_kernel().startswith("rs_fused_mfma_kernel"), c.last_kernel()
        got = d.cpu().numpy().reshape(nb, n, rs)
        want = orc.encode_fast(k, m, data)
        assert np.array_equal(got[:, k:, :S], want), S
        assert (got[:, k:, S:] == 0xA5).all(), S  # padding past S never written
        r = raw.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
        for b in range(nb):
            rows = list(data[b]) + list(want[b])
            for i in range(n):
                assert rsmi.crc16_entry(b"", int(r[b, i]), S) == orc.crc16_ibm(rows[i].tobytes()), (S, b, i)


@pytest.mark.gpu
@pytest.mark.parametrize("nb", [2, 64])
def test_encode_batch_dev_crc_concurrent_streams(nb):
    """Two threads call rsmi_encode_batch_dev_crc on one context, each on its own stream, over and
    over (the fused kernel's unit records and the inline combine's counters used to be
    one per context, so kernels of the two streams could share them).  Each stream now has its
    own scratch; every parity row and R(shard) equals the oracle's.  nb = 2: small launches, the
    combine inside the kernel (its counters); nb = 64: the separate combine."""
    import threading

    import torch

    k, m, S = 10, 4, 26215
    n = k + m
    rs = rsmi.recommended_pitch(S)
    errors = []
    with rsmi.Codec(k, m) as c:
        def work(seed):
            st = torch.cuda.Stream()
            data = np.random.default_rng(seed).integers(0, 256, size=(nb, k, S), dtype=np.uint8)
            host = np.zeros((nb, n, rs), dtype=np.uint8)
            host[:, :k, :S] = data
            want = orc.encode_fast(k, m, data)
            with torch.cuda.stream(st):
                d = torch.from_numpy(host.reshape(-1).copy()).cuda()
                raw = torch.zeros((nb, n), dtype=torch.int32, device="cuda")
                for _ in range(20):
                    raw.zero_()
                    d.view(nb, n, rs)[:, k:, :] = 0
                    c.encode_batch_dev_crc(d.data_ptr(), rs, n * rs, d.data_ptr() + k * rs, rs, n * rs, S, nb,
                                           raw.data_ptr(), st.cuda_stream)
                    got = d.view(nb, n, rs)[:, k:, :S].cpu().numpy()
                    r = raw.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
                    if not np.array_equal(got, want):
                        errors.append(("parity", seed))
                        return
                    for b in (0, nb - 1):
                        rows = list(data[b]) + list(want[b])
                        for i in range(n):
                            if rsmi.crc16_entry(b"", int(r[b, i]), S) != orc.crc16_ibm(rows[i].tobytes()):
                                errors.append(("crc", seed, b, i))
                                return

        th = [threading.Thread(target=work, args=(s,)) for s in (1, 2)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    assert errors == []


@pytest.mark.gpu
@pytest.mark.parametrize("k,m", [(10, 4), (16, 4), (2, 1), (5, 3)])
@pytest.mark.parametrize("mis", [0, 1, 3])
def test_fused_mfma_split_every_tail(k, m, mis):
    """rs_fused_mfma_kernel on unaligned-window rows (the Split layout at a base misaligned by
    `mis` bytes): the lane holding a row's last, overlapping window corrects its counts to the
    chunk position, for every tail S % 16 (the shift d = 16 - S % 16) and rows that end in the
    first, a middle and the last tile of a 4-tile unit; all-0xFF rows as well, so the correction's
    extra counts show if they ever carried into the other shard's bits."""
    import torch

    n = k + m
    for S in [4096 * 2 + 1024 + r for r in range(16)] + [17, 31, 1040, 4111, 26215]:
        nb = 3
        for fill in ("random", "ones"):
            if fill == "ones":
                data = np.full((nb, k, S), 0xFF, dtype=np.uint8)
            else:
                data = np.random.default_rng(S * 7 + k + mis).integers(0, 256, size=(nb, k, S), dtype=np.uint8)
            buf = torch.zeros(nb * n * S + mis + 64, dtype=torch.uint8, device="cuda")
            view = buf[mis:mis + nb * n * S].view(nb, n, S)
            view[:, :k] = torch.from_numpy(data).cuda()
            raw = torch.zeros((nb, n), dtype=torch.int32, device="cuda")
            base = view.data_ptr()
            with rsmi.Codec(k, m) as c:
                c.encode_batch_dev_crc(base, S, n * S, base + k * S, S, n * S, S, nb, raw.data_ptr(),
                                       torch.cuda.current_stream().cuda_stream)
                torch.cuda.synchronize()
                kern = c.last_kernel()
            assert kern.startswith("rs_fused_mfma_kernel"), kern
            assert (",UA" in kern) == (S % 16 != 0 or mis != 0), kern
            got = view.cpu().numpy()
            want = orc.encode_fast(k, m, data)
            assert np.array_equal(got[:, k:], want), (S, fill)
            r = raw.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
            for b in range(nb):
                rows = list(data[b]) + list(want[b])
                for i in range(n):
                    assert rsmi.crc16_entry(b"", int(r[b, i]), S) == orc.crc16_ibm(rows[i].tobytes()), (S, fill, b, i)


@pytest.mark.gpu
@pytest.mark.parametrize("flag", [1, 0])
@pytest.mark.parametrize("k,m,B", [(10, 4, 262144), (2, 1, 4096), (16, 4, 1 << 20)])
def test_coalesced_lone_calls_completion_flag(k, m, B, flag):
    """A lone caller's coalesced encode + CRC-16, and a one-block in-place host call, is one table
    launch of the fused kernel whose last workgroup releases the context's completion flag (option
    coalesce_flag 1, BlockBases::done_flag; 0: the stream synchronisation).  150 calls back to back
    on fresh data, the two kinds alternating (the two flag slots and their counters reused ~75
    times each), every shard and R(shard) against the oracle; after each encode a lone repair and a
    lone degraded read rebuild lost rows in place through the plain table kernel and its flag."""
    n = k + m
    S = (B + k - 1) // k
    L = rsmi.lib()
    p = L.rsmi_host_alloc(n * S)
    assert p
    try:
        sh = np.ctypeslib.as_array((ctypes.c_uint8 * (n * S)).from_address(p)).reshape(n, S)
        rng = np.random.default_rng(B + flag)
        raw = (ctypes.c_uint32 * n)()
        with rsmi.Codec(k, m) as c:
            c.set_option("coalesce_flag", flag)
            c.warm()
            for it in range(150):
                block = rng.integers(0, 256, size=B, dtype=np.uint8)
                full = orc.split(k, m, block.tobytes())
                full[k:] = orc.encode_fast(k, m, full[None, :k], threads=4)[0]
                flat = sh.reshape(-1)
                flat[:] = 0xA5
                flat[:B] = block
                if it % 2:  # the lone in-place host call (encode_small) takes the same flagged launch
                    flat[B:k * S] = 0  # Split's zero padding (the coalesced call writes it itself)
                    c.encode_batch_host_crcs_ptr(p, n * S, p + k * S, n * S, S, 1, ctypes.addressof(raw), None)
                else:
                    assert L.rsmi_encode_block_coalesced(c._h, p, B, p, raw) == 0
                assert np.array_equal(sh, full), it
                if it % 30 == 0:
                    assert ",TB" in c.last_kernel(), c.last_kernel()
                    for r in range(n):
                        assert rsmi.crc16_entry(b"", raw[r], S) == orc.crc16_ibm(full[r].tobytes()), (it, r)
                # a lone repair (the rows asked for) and a lone degraded read (the data rows) rebuilt
                # in place: the plain table kernel with the flag
                lost = [it % n, (it + 3) % n] if m > 1 else [it % n]
                present = [i not in lost for i in range(n)]
                sh[lost] = 0xEE
                c.reconstruct_rows_batch_host_ptr(p, n * S, S, 1, present, [i in lost for i in range(n)])
                assert np.array_equal(sh, full), (it, lost)
                sh[lost] = 0xEE
                c.reconstruct_batch_host_ptr(p, n * S, S, 1, present, True)
                for r in range(n):
                    if r in lost and r >= k:
                        assert (sh[r] == 0xEE).all(), (it, r)
                    else:
                        assert np.array_equal(sh[r], full[r]), (it, r)
                # a lone verified degraded read: the fused reconstruct with the survivors' R(row)
                # (the in-kernel-combine table form, its R stored straight to page-locked memory)
                if any(r < k for r in lost):
                    sh[lost] = 0xEE
                    v16 = np.zeros(k, dtype=np.uint32)
                    c.reconstruct_batch_host_verify_ptr(p, n * S, S, 1, present, True, v16.ctypes.data)
                    used = [i for i in range(n) if present[i]][:k]
                    for r in range(k):
                        assert np.array_equal(sh[r], full[r]), (it, r)
                    if it % 10 == 0:
                        for j, r in enumerate(used):
                            assert rsmi.crc16_entry(b"", int(v16[j]), S) == orc.crc16_ibm(full[r].tobytes()), (it, r)
    finally:
        L.rsmi_host_free(p)


@pytest.mark.gpu
def test_coalesced_pipelined_host_fault_midrun():
    """Batches failing in their executor (option "inject_host_fault", set by one caller mid-run)
    while other batches of the same lanes are in flight (pipelined, with completion flags): the
    failed batches' callers get RSMI_ERR_HOST, every other call's shards and R(shard) equal the
    oracle's, no caller hangs, and the queue codes correctly afterwards."""
    import threading

    k, m, B = 10, 4, 262144
    n = k + m
    S = (B + k - 1) // k
    L = rsmi.lib()
    T, per = 8, 30
    rng = np.random.default_rng(77)
    blocks = [rng.integers(0, 256, size=B, dtype=np.uint8) for _ in range(T)]
    want = []
    for b in blocks:
        w = orc.split(k, m, b.tobytes())
        w[k:] = orc.encode_fast(k, m, w[None, :k], threads=4)[0]
        want.append((w, [orc.crc16_ibm(w[r].tobytes()) for r in range(n)]))
    ptrs = [L.rsmi_host_alloc(n * S) for _ in range(T)]
    assert all(ptrs)
    rcs = [[] for _ in range(T)]
    bad = []
    try:
        views = [np.ctypeslib.as_array((ctypes.c_uint8 * (n * S)).from_address(p)).reshape(n, S) for p in ptrs]
        with rsmi.Codec(k, m) as c:
            c.warm()

            def run(t):
                raw = (ctypes.c_uint32 * n)()
                for i in range(per):
                    if t == 0 and i == 10:
                        c.set_option("inject_host_fault", 3)
                    flat = views[t].reshape(-1)
                    flat[:] = 0xA5
                    flat[:B] = blocks[t]
                    rc = L.rsmi_encode_block_coalesced(c._h, ptrs[t], B, ptrs[t], raw)
                    rcs[t].append(rc)
                    if rc == 0 and (not np.array_equal(views[t], want[t][0]) or
                                    [rsmi.crc16_entry(b"", raw[r], S) for r in range(n)] != want[t][1]):
                        bad.append((t, i))

            th = [threading.Thread(target=run, args=(t,)) for t in range(T)]
            for x in th:
                x.start()
            for x in th:
                x.join(timeout=60)
            assert not any(x.is_alive() for x in th)
            flat = views[0].reshape(-1)
            flat[:B] = blocks[0]
            raw = (ctypes.c_uint32 * n)()
            assert L.rsmi_encode_block_coalesced(c._h, ptrs[0], B, ptrs[0], raw) == 0
            assert np.array_equal(views[0], want[0][0])
    finally:
        for p in ptrs:
            L.rsmi_host_free(p)
    codes = [rc for r in rcs for rc in r]
    assert set(codes) <= {0, rsmi.ErrHost}, set(codes)
    assert codes.count(rsmi.ErrHost) >= 1
    assert bad == []


@pytest.mark.gpu
def test_mixed_lone_and_coalesced_stress():
    """24 threads on one context mixing, at random, coalesced encodes + CRC-16 and coalesced
    degraded reconstructs (the group commit: pipelined table launches, completion flags, two lanes)
    with direct one-block in-place host calls (encode + CRC-16, repair rows, verified read) that
    hold the context and share lane 0's stream and flags: three block sizes, every result against
    the oracle, no caller left waiting."""
    import threading

    k, m = 10, 4
    n = k + m
    L = rsmi.lib()
    sizes = [4096, 65536 + 7, 262144]
    ref = {}
    rng = np.random.default_rng(4242)
    for B in sizes:
        S = (B + k - 1) // k
        block = rng.integers(0, 256, size=B, dtype=np.uint8)
        full = orc.split(k, m, block.tobytes())
        full[k:] = orc.encode(k, m, full[:k])
        ref[B] = (block, full, [orc.crc16_ibm(full[r].tobytes()) for r in range(n)], S)
    T, per = 24, 40
    bufs = [L.rsmi_host_alloc(n * ((max(sizes) + k - 1) // k)) for _ in range(T)]
    assert all(bufs)
    errors = []
    try:
        with rsmi.Codec(k, m) as c:
            c.warm()

            def run(t):
                r = np.random.default_rng(t)
                raw = (ctypes.c_uint32 * n)()
                for i in range(per):
                    B = sizes[int(r.integers(0, len(sizes)))]
                    block, full, r16, S = ref[B]
                    sh = np.ctypeslib.as_array((ctypes.c_uint8 * (n * S)).from_address(bufs[t])).reshape(n, S)
                    op = int(r.integers(0, 4))
                    sh[:] = 0x5A
                    sh.reshape(-1)[:B] = block
                    if op == 0:
                        rc = L.rsmi_encode_block_coalesced(c._h, bufs[t], B, bufs[t], raw)
                    else:
                        sh.reshape(-1)[B:k * S] = 0
                        c.encode_batch_host_crcs_ptr(bufs[t], n * S, bufs[t] + k * S, n * S, S, 1, ctypes.addressof(raw), None)
                        rc = 0
                    if rc or not np.array_equal(sh, full) or [rsmi.crc16_entry(b"", raw[x], S) for x in range(n)] != r16:
                        errors.append((t, i, "encode", op, rc))
                        continue
                    lost = sorted(int(x) for x in r.choice(n, size=int(r.integers(1, m + 1)), replace=False))
                    present = [x not in lost for x in range(n)]
                    sh[lost] = 0xEE
                    if op == 1:
                        c.reconstruct_rows_batch_host_ptr(bufs[t], n * S, S, 1, present, [x in lost for x in range(n)])
                    elif op == 2 and any(x < k for x in lost):
                        v16 = np.zeros(k, dtype=np.uint32)
                        c.reconstruct_batch_host_verify_ptr(bufs[t], n * S, S, 1, present, False, v16.ctypes.data)
                        used = [x for x in range(n) if present[x]][:k]
                        if [rsmi.crc16_entry(b"", int(v16[j]), S) for j in range(k)] != [r16[x] for x in used]:
                            errors.append((t, i, "verify R"))
                    else:
                        p = (ctypes.c_uint8 * n)(*[1 if x else 0 for x in present])
                        rc = L.rsmi_reconstruct_coalesced(c._h, bufs[t], S, p, 0)
                        if rc:
                            errors.append((t, i, "reconstruct rc", rc))
                            continue
                    if not np.array_equal(sh, full):
                        errors.append((t, i, "rebuilt", op, lost))

            th = [threading.Thread(target=run, args=(t,)) for t in range(T)]
            for x in th:
                x.start()
            for x in th:
                x.join(timeout=120)
            assert not any(x.is_alive() for x in th)
    finally:
        for p in bufs:
            L.rsmi_host_free(p)
    assert errors == []
