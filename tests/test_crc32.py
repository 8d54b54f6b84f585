"""Mutcask value checksum (kv/mutcask/cask.go:73-97: | crc32 (4 B LE) | value |, Go
crc32.ChecksumIEEE) and its GPU split (include/rsmi.h "mutcask CRC-32").

Parity is pinned: Go's crc32.ChecksumIEEE is the zlib CRC-32, so the bit-serial oracle
(crc32_oracle.c), the library's host half and the device R32(row) kernel are all checked
against Python's zlib.crc32 and the catalogue check value 0xCBF43926.  Raw R32(D) (register
after D from zero, no complement) = ~zlib.crc32(D, 0xFFFFFFFF)."""
import ctypes
import random
import zlib

import numpy as np
import pytest

import oracle_lib as orc
import rsmi

M32 = 0xFFFFFFFF


def raw32(data: bytes) -> int:
    """R32(D) from zlib: zlib.crc32(D, v) = ~fold(~v, D), so v = ~0 gives ~fold(0, D)."""
    return ~zlib.crc32(data, M32) & M32


def test_oracle_check_value_and_zlib():
    assert orc.crc32_ieee(b"123456789") == 0xCBF43926  # CRC-32/ISO-HDLC catalogue check
    assert orc.crc32_ieee(b"") == 0
    r = random.Random(5)
    for n in [1, 2, 3, 15, 16, 17, 255, 1024, 4099]:
        b = bytes(r.randrange(256) for _ in range(n))
        assert orc.crc32_ieee(b) == zlib.crc32(b), n


def test_library_checksum_matches_zlib():
    r = np.random.default_rng(12)
    for n in [0, 1, 7, 16, 255, 256, 257, 1023, 1024, 1025, 26215, 262144, 262147]:
        b = r.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        assert rsmi.crc32_ieee(b) == zlib.crc32(b), n


def test_mutcask_value_roundtrip_value():
    """cask_test.go TestValueEncodeDecode's value: EncodeValue prefixes ChecksumIEEE(v) LE."""
    v = b"mutation of bitcask"
    enc = zlib.crc32(v).to_bytes(4, "little") + v
    assert int.from_bytes(enc[:4], "little") == orc.crc32_ieee(v) == rsmi.crc32_ieee(v)


@pytest.mark.parametrize("hl,n", [(0, 0), (0, 5), (12, 0), (16, 1), (16, 1023), (16, 1024), (20, 26215),
                                  (16, 104858), (3, 262144)])
def test_entry_from_raw_matches_zlib(hl, n):
    """The host half of the split: ChecksumIEEE(head || D) from R32(D) and |D| only."""
    r = np.random.default_rng(hl * 7 + n)
    head = r.integers(0, 256, size=hl, dtype=np.uint8).tobytes()
    d = r.integers(0, 256, size=n, dtype=np.uint8).tobytes()
    assert rsmi.crc32_entry(head, raw32(d), n) == zlib.crc32(head + d)


def test_oracle_mutcask_entry_crc_is_checksum_of_framed_entry():
    meta = (262144).to_bytes(4, "little")
    data = bytes(range(256)) * 3
    c16 = orc.datanode_entry_crc(meta, data)
    framed = c16.to_bytes(4, "little") + orc.entry_head(meta, len(data)) + data
    assert orc.mutcask_entry_crc(c16, meta, data) == zlib.crc32(framed)


@pytest.mark.gpu
@pytest.mark.parametrize("S", [1, 7, 15, 16, 17, 1000, 1023, 1024, 1025, 8191, 8192, 8193, 16384, 24577, 26215, 32767,
                               32768, 32769, 40961, 65536, 73729, 104858, 262144, 1048579])
@pytest.mark.parametrize("layout", ["aligned", "unaligned"])
@pytest.mark.parametrize("wpc", [0, 1])
@pytest.mark.parametrize("fold", [1, 0])
def test_rows_dev_matches_zlib(S, layout, wpc, fold):
    import torch

    nrows, nb = 3, 5
    if layout == "aligned":
        pitch, off = (S + 15) // 16 * 16 + 16, 0
    else:
        pitch, off = S + 3, 5
    g = torch.Generator().manual_seed(S)
    host = torch.randint(0, 256, (off + nb * nrows * pitch + 64,), dtype=torch.uint8, generator=g)
    dev = host.to("cuda")
    out = torch.full((nb, nrows + 1), 0xDEAD, dtype=torch.int32, device="cuda")
    with rsmi.Codec(4, 2) as c:
        c.set_option("waves_per_cu", wpc)
        c.set_option("crc32_fold", fold)
        c.crc32_rows_dev(dev.data_ptr() + off, pitch, nrows * pitch, nrows, S, nb, out.data_ptr(), nrows + 1)
        torch.cuda.synchronize()
        assert c.last_kernel() == ("rs_crc32_rows_kernel,MFMA" if fold else "rs_crc32_rows_kernel")
    got = out.cpu().numpy().astype(np.int64) & M32
    h = host.numpy()
    for b in range(nb):
        assert got[b, nrows] == 0xDEAD  # slots past nrows untouched
        for r in range(nrows):
            row = h[off + b * nrows * pitch + r * pitch:][:S].tobytes()
            assert got[b, r] == raw32(row), (b, r)


@pytest.mark.gpu
@pytest.mark.parametrize("S", [17, 1009, 1024, 8177, 8185, 8192, 16383, 26215, 32761, 32768, 73729])
def test_rows_dev_split_layout_every_misalignment(S):
    """The Split layout (rows back to back at pitch S) from each of the 16 byte offsets of an
    aligned base: every row misalignment of the unaligned pass's memory-grid fold (leading bytes
    masked, rows reaching one tile or one 8 KiB group further on the memory grid, the end shift
    by the misalignment), against zlib."""
    import torch

    nrows, nb = 4, 3
    for off in range(16):
        g = torch.Generator().manual_seed(S * 7 + off)
        host = torch.randint(0, 256, (off + nb * nrows * S + 64,), dtype=torch.uint8, generator=g)
        dev = host.to("cuda")
        h = host.numpy()
        for fold in (1, 0):
            out = torch.zeros((nb, nrows), dtype=torch.int32, device="cuda")
            with rsmi.Codec(4, 2) as c:
                c.set_option("crc32_fold", fold)
                c.crc32_rows_dev(dev.data_ptr() + off, S, nrows * S, nrows, S, nb, out.data_ptr(), nrows)
                torch.cuda.synchronize()
            got = out.cpu().numpy().astype(np.int64) & M32
            for b in range(nb):
                for r in range(nrows):
                    row = h[off + (b * nrows + r) * S:][:S].tobytes()
                    assert got[b, r] == raw32(row), (off, fold, b, r)


@pytest.mark.gpu
def test_rows_dev_random_unaligned_shapes():
    """40 random unaligned geometries (any base offset, pitch >= S and block stride at any byte
    granularity): the unaligned pass's memory-grid fold against zlib on every row."""
    import random

    import torch

    rng = random.Random(2028)
    for _ in range(40):
        S = rng.choice([rng.randrange(1, 2048), rng.randrange(2048, 70000), rng.randrange(70000, 200000)])
        nrows, nb = rng.randrange(1, 6), rng.randrange(1, 6)
        off = rng.randrange(1, 16)
        pitch = S + rng.randrange(0, 40)
        bstride = nrows * pitch + rng.randrange(0, 40)
        g = torch.Generator().manual_seed(S + off)
        host = torch.randint(0, 256, (off + nb * bstride + 64,), dtype=torch.uint8, generator=g)
        dev = host.to("cuda")
        h = host.numpy()
        for fold in (1, 0):
            out = torch.zeros((nb, nrows), dtype=torch.int32, device="cuda")
            with rsmi.Codec(4, 2) as c:
                c.set_option("crc32_fold", fold)
                c.crc32_rows_dev(dev.data_ptr() + off, pitch, bstride, nrows, S, nb, out.data_ptr(), nrows)
                torch.cuda.synchronize()
            got = out.cpu().numpy().astype(np.int64) & M32
            for b in range(nb):
                for r in range(nrows):
                    row = h[off + b * bstride + r * pitch:][:S].tobytes()
                    assert got[b, r] == raw32(row), (S, off, pitch, bstride, fold, b, r)


@pytest.mark.gpu
def test_rows_dev_full_size_batch():
    """RS(10,4) 256 KiB geometry, 4096 blocks x 14 rows, against zlib on a sample of rows."""
    import torch

    k, m, nb = 10, 4, 4096
    n, S = k + m, 26215
    pitch = rsmi.recommended_pitch(S)
    g = torch.Generator(device="cuda").manual_seed(10)
    dev = torch.randint(0, 256, (nb, n, pitch), dtype=torch.uint8, device="cuda", generator=g)
    out = torch.empty((nb, n), dtype=torch.int32, device="cuda")
    with rsmi.Codec(k, m) as c:
        c.crc32_rows_dev(dev.data_ptr(), pitch, n * pitch, n, S, nb, out.data_ptr(), n)
        torch.cuda.synchronize()
    got = out.cpu().numpy().astype(np.int64) & M32
    rng = random.Random(2)
    for _ in range(64):
        b, r = rng.randrange(nb), rng.randrange(n)
        assert got[b, r] == raw32(dev[b, r, :S].cpu().numpy().tobytes())


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,B", [(2, 1, 6), (4, 2, 262144), (10, 4, 262144), (10, 4, 1048576), (16, 4, 65536 + 7)])
@pytest.mark.parametrize("small", [0, 1 << 30])
@pytest.mark.parametrize("want16", [True, False])
@pytest.mark.parametrize("pinned", [False, True])
def test_encode_batch_host_crcs_entries(k, m, B, small, want16, pinned):
    """Both raw checksums of every shard from one host batch: the datanode entry CRC-16 and the
    mutcask value CRC-32 of that entry equal the oracle's, on the oracle's shards."""
    n = k + m
    S = (B + k - 1) // k
    nb = 5
    r = np.random.default_rng(B + k + small % 7)
    ptrs = []

    def buf(shape, dtype):
        nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
        if not pinned:
            return np.zeros(shape, dtype=dtype)
        p = rsmi.lib().rsmi_host_alloc(nbytes)
        assert p
        ptrs.append(p)
        a = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p)).view(dtype).reshape(shape)
        a[...] = 0
        return a

    data = buf((nb, k * S), np.uint8)
    data[:, :B] = r.integers(0, 256, size=(nb, B), dtype=np.uint8)
    par = buf((nb, m * S), np.uint8)
    raw16 = buf((nb, n), np.uint32)
    raw32v = buf((nb, n), np.uint32)
    with rsmi.Codec(k, m) as c:
        c.set_option("small_call_bytes", small)  # copy-engine pipeline / zero-copy single kernel
        c.encode_batch_host_crcs_ptr(data.ctypes.data, k * S, par.ctypes.data, m * S, S, nb,
                                     raw16.ctypes.data if want16 else None, raw32v.ctypes.data)
    meta = B.to_bytes(4, "little")
    head = orc.entry_head(meta, S)
    for b in range(nb):
        want_par = orc.encode(k, m, np.ascontiguousarray(data[b]).reshape(k, S))
        assert np.array_equal(par[b].reshape(m, S), want_par)
        rows = list(np.ascontiguousarray(data[b]).reshape(k, S)) + list(want_par)
        for i in range(n):
            row = rows[i].tobytes()
            c16 = orc.datanode_entry_crc(meta, row)
            if want16:
                assert rsmi.crc16_entry(head, int(raw16[b, i]), S) == c16, (b, i)
            assert int(raw32v[b, i]) == raw32(row), (b, i)
            # the mutcask value checksum of the whole entry, from R32(shard) and the header
            h32 = c16.to_bytes(4, "little") + head
            assert rsmi.crc32_entry(h32, int(raw32v[b, i]), S) == orc.mutcask_entry_crc(c16, meta, row), (b, i)
    for p in ptrs:
        rsmi.lib().rsmi_host_free(p)


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,S,nb,lost,required", [(10, 4, 26215, 24, [3], [3]), (10, 4, 26215, 9, [0, 12], [12]),
                                                    (4, 2, 65536, 33, [1, 5], [1, 5]), (16, 4, 4097, 5, [9], [9])])
@pytest.mark.parametrize("small", [0, 1 << 30])
def test_reconstruct_rows_crcs(k, m, S, nb, lost, required, small):
    """rsmi_reconstruct_rows_batch_host_crcs: the rebuilt rows equal the oracle's, and their raw
    CRC-16 / CRC-32 equal the checksums of those rows; rows not rebuilt report 0."""
    n = k + m
    r = np.random.default_rng(S + nb)
    data = r.integers(0, 256, size=(nb, k, S), dtype=np.uint8)
    full = np.concatenate([data, orc.encode_fast(k, m, data)], axis=1)
    shards = full.copy()
    shards[:, lost, :] = 0
    present = [i not in lost for i in range(n)]
    req = [i in required for i in range(n)]
    r16 = np.full((nb, n), 0xDEAD, dtype=np.uint32)
    r32 = np.full((nb, n), 0xDEAD, dtype=np.uint32)
    with rsmi.Codec(k, m) as c:
        c.set_option("small_call_bytes", small)
        c.reconstruct_rows_batch_host_crcs_ptr(shards.ctypes.data, n * S, S, nb, present, req, r16.ctypes.data,
                                               r32.ctypes.data)
    for b in range(nb):
        for i in range(n):
            if i in required:
                row = full[b, i].tobytes()
                assert np.array_equal(shards[b, i], full[b, i]), (b, i)
                assert rsmi.crc16_entry(b"", int(r16[b, i]), S) == orc.crc16_ibm(row), (b, i)
                assert int(r32[b, i]) == raw32(row), (b, i)
            else:
                assert r16[b, i] == 0 and r32[b, i] == 0, (b, i)
