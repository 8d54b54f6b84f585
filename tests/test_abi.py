"""The C-ABI boundary on CPU: librsmi.so loads, exports every symbol include/rsmi.h
declares, and its host-only logic (argument validation, matrices, decode matrices,
shard checks) matches the oracle.  No compute calls: without a GPU they must fail
loudly with RSMI_ERR_NO_DEVICE (there is no CPU fallback)."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle_lib as orc
import rsmi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rsmi.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rsmi_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_seam():
    syms = declared_symbols()
    for s in ["rsmi_open", "rsmi_close", "rsmi_encode", "rsmi_reconstruct", "rsmi_encode_block",
              "rsmi_encode_batch_dev", "rsmi_reconstruct_batch_dev", "rsmi_encode_batch_host",
              "rsmi_reconstruct_batch_host", "rsmi_shard_size", "rsmi_check_shards"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    L = ctypes.CDLL(rsmi.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing


def test_python_binding_covers_header():
    L = rsmi.lib()
    for s in declared_symbols():
        assert getattr(L, s).restype is not None or s in ("rsmi_close", "rsmi_host_free", "rsmi_group_close", "rsmi_group_host_free",
                                                          "rsmi_set_wait_hook"), s


def test_abi_version_and_status_strings():
    assert rsmi.lib().rsmi_abi_version() == 5
    for code in (0, 1, 2, 3, 4, 5, 6, 7, 8, 100, 101, 102):
        assert rsmi.status_string(code) not in ("", "unknown status")


@pytest.mark.parametrize("k,m,want", [(0, 1, rsmi.ErrInvShardNum), (1, 0, rsmi.ErrInvShardNum),
                                      (-1, 2, rsmi.ErrInvShardNum), (200, 57, rsmi.ErrMaxShardNum),
                                      (255, 1, rsmi.OK), (1, 1, rsmi.OK), (128, 128, rsmi.OK)])
def test_open_validation_matches_new_erasure(k, m, want):
    """erasure.go:18-24"""
    h = ctypes.c_void_p()
    rc = rsmi.lib().rsmi_open(k, m, 0, ctypes.byref(h))
    assert rc == want
    if rc == 0:
        rsmi.lib().rsmi_close(h)


@pytest.mark.parametrize("B,k", [(0, 2), (6, 2), (7, 2), (262144, 10), (1048576, 10), (4194304, 16), (1, 16)])
def test_shard_size(B, k):
    assert rsmi.lib().rsmi_shard_size(B, k) == orc.lib().rs_oracle_shard_size(B, k) == rsmi.ceil_frac(B, k)


def test_recommended_pitch():
    p = rsmi.recommended_pitch
    assert p(26215) == 32768 and p(65536) == 65536 and p(262144) == 262144
    assert p(104858) == 147456  # 11/8 S in 4 KiB granules between 96 and 128 KiB (+7% at 1 MiB blocks)
    assert p(150000) == 151552  # 4 KiB granules above
    assert p(17) == 32 and p(1) == 16
    assert p(40000) == 40960  # next pow2 (65536) would waste > S/2
    assert p(1 << 22) == 1 << 22 and p(3000) == 4096
    for S in (1, 3, 17, 4097, 26215, 40000, 104858, 262145):
        assert p(S) >= S and p(S) % 16 == 0


@pytest.mark.parametrize("k,m", [(2, 1), (4, 2), (10, 4), (16, 4), (5, 5), (1, 1), (20, 4), (100, 28)])
def test_encode_matrix_matches_oracle(k, m):
    with rsmi.Codec(k, m) as c:
        got = np.frombuffer(c.encode_matrix(), dtype=np.uint8).reshape(k + m, k)
    assert np.array_equal(got, orc.build_matrix(k, m))


@pytest.mark.parametrize("k,m,lost", [(10, 4, [0]), (10, 4, [0, 5, 11]), (16, 4, [0, 9]), (4, 2, [2, 3]),
                                      (2, 1, [1]), (5, 5, [0, 1, 2, 3, 4])])
def test_decode_matrix_matches_oracle(k, m, lost):
    n = k + m
    present = [i not in lost for i in range(n)]
    with rsmi.Codec(k, m) as c:
        dec, used = c.decode_matrix(present)
    want_used = [i for i in range(n) if present[i]][:k]
    assert used == want_used
    M = orc.build_matrix(k, m)
    sub = np.ascontiguousarray(M[want_used]).reshape(-1)
    inv = np.zeros(k * k, dtype=np.uint8)
    assert orc.lib().rs_oracle_invert(orc.ptr(sub), orc.ptr(inv), k) == 0
    assert np.frombuffer(dec, dtype=np.uint8).tolist() == inv.tolist()


def test_decode_matrix_too_few():
    with rsmi.Codec(4, 2) as c:
        with pytest.raises(rsmi.RsmiError) as e:
            c.decode_matrix([True, True, True, False, False, False])
    assert e.value.code == rsmi.ErrTooFewShards


@pytest.mark.parametrize("lens,nil_ok", [([3, 3, 3], 0), ([3, 0, 3], 1), ([3, 0, 3], 0), ([0, 0, 0], 1),
                                         ([2, 3, 0], 1), ([0, 5, 5, 5], 1)])
def test_check_shards_matches_oracle(lens, nil_ok):
    rc, S = rsmi.check_shards(lens, bool(nil_ok))
    arr = np.array(lens, dtype=np.uint64)
    So = np.zeros(1, dtype=np.uint64)
    assert rc == orc.lib().rs_oracle_check_shards(len(lens), orc.ptr(arr), nil_ok, orc.ptr(So))
    assert S == int(So[0])


def _no_gpu():
    return rsmi.device_count() == 0


@pytest.mark.skipif(not _no_gpu(), reason="only meaningful on a host without a GPU")
def test_compute_fails_loudly_without_gpu():
    """No CPU fallback: every compute entry point reports RSMI_ERR_NO_DEVICE."""
    with rsmi.Codec(2, 1) as c:
        with pytest.raises(rsmi.RsmiError) as e:
            c.encode_block(b"123456")
        assert e.value.code == rsmi.ErrNoDevice
        with pytest.raises(rsmi.RsmiError) as e:
            c.reconstruct(bytearray(9), 3, [True, False, True], True)
        assert e.value.code == rsmi.ErrNoDevice
        # argument errors are still reported before any device access
        with pytest.raises(rsmi.RsmiError) as e:
            c.encode_block(b"")
        assert e.value.code == rsmi.ErrShortData
        with pytest.raises(rsmi.RsmiError) as e:
            c.reconstruct(bytearray(9), 3, [True, False, False], True)
        assert e.value.code == rsmi.ErrTooFewShards
        # nothing missing: upstream quick return, no device needed
        c.reconstruct(bytearray(9), 3, [True, True, True], False)


def test_null_arguments():
    L = rsmi.lib()
    assert L.rsmi_open(2, 1, 0, None) == rsmi.ErrInvalidArg
    assert L.rsmi_encode(None, None, None, 3) == rsmi.ErrInvalidArg
    assert L.rsmi_encode_matrix(None, None) == rsmi.ErrInvalidArg
    with rsmi.Codec(2, 1) as c:
        assert L.rsmi_set_option(c._h, b"no_such_knob", 1) == rsmi.ErrInvalidArg
        # kernel variants measured slower than the defaults are not in the library
        for gone in (b"chunks_per_lane", b"nontemporal", b"prefetch", b"tables", b"lds_dma", b"store_aux",
                     b"buffer_stores", b"xcd_order", b"crc_fold", b"crc32_pipe"):
            assert L.rsmi_set_option(c._h, gone, 1) == rsmi.ErrInvalidArg, gone
        assert L.rsmi_set_option(c._h, b"zero_copy", 0) == rsmi.OK
        assert L.rsmi_set_option(c._h, b"zero_copy", 2) == rsmi.OK
        assert L.rsmi_set_option(c._h, b"zero_copy", 3) == rsmi.ErrInvalidArg


def test_new_options_and_stats_validate():
    L = rsmi.lib()
    with rsmi.Codec(10, 4) as c:
        for key, good, bad in [(b"waves_per_cu", 8, -1), (b"coalesce_us", 50, -1), (b"coalesce_max", 16, 0),
                               (b"crc16_fold", 0, 2), (b"crc16_fused_fold", 0, 2), (b"coalesce_lanes", 4, 0),
                               (b"coalesce_lanes", 16, 17), (b"coalesce_carry", 0, -1), (b"coalesce_carry", 16, 17),
                               (b"coalesce_pipeline", 0, -1), (b"coalesce_pipeline", 1, 2),
                               (b"coalesce_flag", 0, -1), (b"coalesce_flag", 1, 2)]:
            assert L.rsmi_set_option(c._h, key, good) == rsmi.OK, key
            assert L.rsmi_set_option(c._h, key, bad) == rsmi.ErrInvalidArg, key
        assert c.stat("coalesced_calls") == 0 and c.stat("coalesced_batches") == 0
        assert c.stat("no_such_counter") == -1


def test_warm_fails_loudly_without_gpu():
    """rsmi_warm binds the device and opens the coalescing lanes: on a host without a GPU it
    reports RSMI_ERR_NO_DEVICE (no CPU fallback), and a NULL context is an argument error."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    L = rsmi.lib()
    assert L.rsmi_warm(None) == rsmi.ErrInvalidArg
    with rsmi.Codec(10, 4) as c:
        with pytest.raises(rsmi.RsmiError) as e:
            c.warm()
        assert e.value.code == rsmi.ErrNoDevice


def test_coalesced_calls_fail_loudly_without_gpu():
    """No CPU fallback on the coalesced entry points either; argument errors come first."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with rsmi.Codec(10, 4) as c:
        with pytest.raises(rsmi.RsmiError) as e:
            c.encode_block_coalesced(b"x" * 100)
        assert e.value.code == rsmi.ErrNoDevice
        with pytest.raises(rsmi.RsmiError) as e:
            c.encode_block_coalesced(b"")
        assert e.value.code == rsmi.ErrShortData
        sh = bytearray(14 * 10)
        with pytest.raises(rsmi.RsmiError) as e:
            c.reconstruct_coalesced(sh, 10, [i != 0 for i in range(14)], True)
        assert e.value.code == rsmi.ErrNoDevice
        with pytest.raises(rsmi.RsmiError) as e:
            c.reconstruct_coalesced(sh, 10, [i > 4 for i in range(14)], True)
        assert e.value.code == rsmi.ErrTooFewShards


def test_small_call_option_validates():
    L = rsmi.lib()
    with rsmi.Codec(10, 4) as c:
        assert L.rsmi_set_option(c._h, b"small_call_bytes", 0) == rsmi.OK
        assert L.rsmi_set_option(c._h, b"small_call_bytes", 1 << 30) == rsmi.OK
        assert L.rsmi_set_option(c._h, b"small_call_bytes", -1) == rsmi.ErrInvalidArg


def test_wait_hook_is_per_thread_and_one_shot():
    """rsmi_set_wait_hook / rsmi_run_wait_hook without a device: a pending hook runs once through
    rsmi_run_wait_hook, NULL clears it, a call that fails before launching (no GPU here) leaves it
    pending, and another thread does not see this thread's hook."""
    import threading

    L = rsmi.lib()
    ran = []
    cb = ctypes.CFUNCTYPE(None, ctypes.c_void_p)(lambda arg: ran.append(arg))
    assert L.rsmi_run_wait_hook() == 0
    L.rsmi_set_wait_hook(cb, 7)
    assert L.rsmi_run_wait_hook() == 1 and ran == [7]
    assert L.rsmi_run_wait_hook() == 0 and ran == [7]
    L.rsmi_set_wait_hook(cb, 8)
    L.rsmi_set_wait_hook(None, None)
    assert L.rsmi_run_wait_hook() == 0 and ran == [7]
    L.rsmi_set_wait_hook(cb, 9)
    other = []
    t = threading.Thread(target=lambda: other.append(L.rsmi_run_wait_hook()))
    t.start()
    t.join()
    assert other == [0] and ran == [7]
    with rsmi.Codec(10, 4) as c:
        with pytest.raises(rsmi.RsmiError):
            c.encode_block_coalesced(b"")  # an argument error: nothing launched
    assert ran == [7]
    assert L.rsmi_run_wait_hook() == 1 and ran == [7, 9]
