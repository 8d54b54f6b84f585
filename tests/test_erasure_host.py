"""Host logic of the Erasure mirror (dag/node/dagnode/erasure.go) that runs without a GPU:
validation, ShardSize, the EncodeData/DecodeDataBlocks short-circuits and error paths."""
import numpy as np
import pytest

import rsmi
from rsmi import multi


def test_new_erasure_validation():
    with pytest.raises(rsmi.RsmiError) as e:
        rsmi.NewErasure(0, 1, 10)
    assert e.value.code == rsmi.ErrInvShardNum
    with pytest.raises(rsmi.RsmiError) as e:
        rsmi.NewErasure(2, 0, 10)
    assert e.value.code == rsmi.ErrInvShardNum
    with pytest.raises(rsmi.RsmiError) as e:
        rsmi.NewErasure(250, 7, 10)
    assert e.value.code == rsmi.ErrMaxShardNum
    e = rsmi.NewErasure(2, 1, 6)
    assert e.shard_size() == 3


@pytest.mark.parametrize("n,d,want", [(6, 2, 3), (7, 2, 4), (0, 3, 0), (5, 0, 0), (-7, 2, -3), (7, -2, -3),
                                      (262144, 10, 26215), (1048576, 10, 104858)])
def test_ceil_frac(n, d, want):
    """utils.go:6-21 (denominator 0 -> 0; negative denominators flipped; ceil only for n>0)."""
    assert rsmi.ceil_frac(n, d) == want


def test_encode_empty_block_returns_nil_shards():
    """erasure.go:52-54: B == 0 -> k+m nil shards, no codec call."""
    e = rsmi.NewErasure(4, 2, 0)
    assert e.encode_data(b"") == [None] * 6
    assert e._codec is None  # the encoder was never built


def test_decode_nothing_missing_is_noop():
    e = rsmi.NewErasure(2, 1, 6)
    sh = [b"123", b"456", b"\x3b\x3c\x39"]
    e.decode_data_blocks(sh)
    assert sh == [b"123", b"456", b"\x3b\x3c\x39"]
    assert e._codec is None


def test_decode_all_empty_is_shard_no_data():
    """The isZero loop breaks after the first empty shard (erasure.go:72-77), so an all-empty
    set reaches ReconstructData and fails with ErrShardNoData: a 0-byte block can be Put but
    not Get."""
    e = rsmi.NewErasure(2, 1, 0)
    with pytest.raises(rsmi.RsmiError) as ex:
        e.decode_data_blocks([None, None, None])
    assert ex.value.code == rsmi.ErrShardNoData


def test_decode_size_mismatch():
    e = rsmi.NewErasure(2, 1, 6)
    with pytest.raises(rsmi.RsmiError) as ex:
        e.decode_data_blocks([b"123", None, b"\x3b\x3c"])
    assert ex.value.code == rsmi.ErrShardSize


def test_decode_too_few_and_wrong_count():
    e = rsmi.NewErasure(2, 1, 6)
    with pytest.raises(rsmi.RsmiError) as ex:
        e.decode_data_blocks([b"123", None, None])
    assert ex.value.code == rsmi.ErrTooFewShards
    with pytest.raises(rsmi.RsmiError) as ex:
        e.decode_data_and_parity_blocks([b"123", b"456"])
    assert ex.value.code == rsmi.ErrTooFewShards


def test_data_only_with_parity_missing_is_noop():
    """ReconstructData returns early when every data shard is present."""
    e = rsmi.NewErasure(2, 1, 6)
    sh = [b"123", b"456", None]
    e.decode_data_blocks(sh)
    assert sh[2] is None


def test_crc16_ibm_check_value():
    assert multi.crc16_ibm(b"123456789") == 0xB4C8
    assert 0 <= multi.key_hash_slot("QmSomeCid") < 16384


def test_partition_blocks_cover_once():
    for nb in (0, 1, 7, 4096, 8193):
        for world in (1, 2, 3, 8):
            got = [multi.partition_blocks(nb, world, r) for r in range(world)]
            assert sum(c for _, c in got) == nb
            pos = 0
            for s, c in got:
                assert s == pos
                pos += c
            assert max(c for _, c in got) - min(c for _, c in got) <= 1


def test_key_gpu_stable_and_balanced():
    keys = [f"bafkrei{i:08d}" for i in range(4000)]
    counts = [0] * 8
    for k in keys:
        g = multi.key_gpu(k, 8)
        assert g == multi.key_gpu(k, 8)
        counts[g] += 1
    assert min(counts) > 300


_CLMUL_LENGTHS = [0, 1, 7, 8, 9, 15, 16, 17, 100, 255, 256, 257, 271, 272, 511, 512, 513, 1000, 4099, 26215,
                  26227, 104858, 262147]


@pytest.mark.parametrize("tables", [0, 1])
def test_datanode_crc_slice_by_8_matches_byte_serial(tables):
    """The datanode entry CRC (slice-by-8 below 256 bytes, carry-less-multiply folding from 256,
    csrc/host/datanode.cpp + crc_clmul.cpp) equals the byte-serial restatement of
    howeyc/crc16 Checksum(IBMTable) on every length class, from any register start value.
    tables=1 forces slice-by-8 at every length (the path of CPUs without VPCLMULQDQ)."""
    import ctypes

    L = ctypes.CDLL(rsmi.LIB_PATH)
    f = L._ZN4rsmi4host9crc16_ibmEPKhmt
    f.restype = ctypes.c_uint16
    f.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint16]
    rng = np.random.default_rng(5)
    L.rsmi_host_crc_force_tables(tables)
    try:
        for n in _CLMUL_LENGTHS:
            b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            assert f(b, n, 0) == multi.crc16_ibm(b), n
            # a continued checksum (the entry's header first, then the shard) equals the whole one
            h = n // 3
            assert f(b[h:], n - h, f(b[:h], h, 0)) == multi.crc16_ibm(b), n
    finally:
        L.rsmi_host_crc_force_tables(0)


@pytest.mark.parametrize("tables", [0, 1])
def test_datanode_value_crc32_matches_zlib(tables):
    """The mutcask value CRC-32 of the in-process datanode (slice-by-8 / carry-less-multiply
    folding) equals zlib's crc32 (Go crc32.ChecksumIEEE) on every length class, on both paths."""
    import ctypes
    import zlib

    L = ctypes.CDLL(rsmi.LIB_PATH)
    f = L._ZN4rsmi4host10crc32_ieeeEPKhm
    f.restype = ctypes.c_uint32
    f.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    rng = np.random.default_rng(6)
    L.rsmi_host_crc_force_tables(tables)
    try:
        for n in _CLMUL_LENGTHS:
            b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            assert f(b, n) == zlib.crc32(b), n
    finally:
        L.rsmi_host_crc_force_tables(0)
