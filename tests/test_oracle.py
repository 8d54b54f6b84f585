"""The CPU oracle against the upstream known-answer tests, the reference fixture and the
committed golden vectors (CPU only).  SURVEY.md 8(c), Appendix A.4."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle_lib as orc

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_selftest_all_kats():
    assert orc.lib().rs_oracle_selftest() == 0


@pytest.mark.parametrize("a,b,want", [(3, 4, 12), (7, 7, 21), (23, 45, 41), (0, 9, 0), (1, 200, 200)])
def test_gal_multiply_kat(a, b, want):
    assert orc.lib().rs_oracle_gal_mul(a, b) == want


@pytest.mark.parametrize("a,n,want", [(2, 2, 4), (5, 20, 235), (13, 7, 43), (0, 0, 1), (0, 3, 0), (9, 0, 1)])
def test_gal_exp_kat(a, n, want):
    assert orc.lib().rs_oracle_gal_exp(a, n) == want


def test_inverse_kat():
    m = np.array([56, 23, 98, 3, 100, 200, 45, 201, 123], dtype=np.uint8)
    out = np.zeros(9, dtype=np.uint8)
    assert orc.lib().rs_oracle_invert(orc.ptr(m), orc.ptr(out), 3) == 0
    assert out.tolist() == [175, 133, 33, 130, 13, 245, 112, 35, 126]


def test_singular_matrix():
    m = np.array([1, 2, 2, 4], dtype=np.uint8)  # row 2 = 2 * row 1
    out = np.zeros(4, dtype=np.uint8)
    assert orc.lib().rs_oracle_invert(orc.ptr(m), orc.ptr(out), 2) == 7


def test_one_encode_5_5():
    data = np.array([[0, 1], [4, 5], [2, 3], [6, 7], [8, 9]], dtype=np.uint8)
    assert orc.encode(5, 5, data).tolist() == [[12, 13], [10, 11], [14, 15], [90, 91], [94, 95]]


def test_reference_fixture_123456():
    sh = orc.split(2, 1, b"123456")
    sh[2:] = orc.encode(2, 1, sh[:2])
    assert bytes(sh[0]) == b"123" and bytes(sh[1]) == b"456"
    assert sh[2].tolist() == [0x3B, 0x3C, 0x39]


def test_matrix_rows_quoted_in_survey():
    assert orc.build_matrix(2, 1)[2].tolist() == [3, 2]
    assert orc.build_matrix(4, 2)[4:].tolist() == [[27, 28, 18, 20], [28, 27, 20, 18]]
    assert orc.build_matrix(10, 4)[10].tolist() == [129, 150, 175, 184, 210, 196, 254, 232, 3, 2]
    assert orc.build_matrix(16, 4)[16][:4].tolist() == [33, 181, 246, 133]
    for k, m in [(2, 1), (4, 2), (10, 4), (16, 4), (200, 56)]:
        M = orc.build_matrix(k, m)
        assert np.array_equal(M[:k], np.eye(k, dtype=np.uint8)), (k, m)


def test_decode_row_quoted_in_survey():
    """A.3: (10,4), shard 0 lost, survivors 1..10 -> decode row for shard 0."""
    M = orc.build_matrix(10, 4)
    sub = np.ascontiguousarray(M[1:11]).reshape(-1)
    inv = np.zeros(100, dtype=np.uint8)
    assert orc.lib().rs_oracle_invert(orc.ptr(sub), orc.ptr(inv), 10) == 0
    assert inv.reshape(10, 10)[0].tolist() == [153, 44, 180, 112, 188, 245, 57, 252, 168, 84]


def test_error_sentinels():
    L = orc.lib()
    assert L.rs_oracle_build_matrix(0, 1, orc.ptr(np.zeros(1, np.uint8))) == 5
    assert L.rs_oracle_build_matrix(1, 0, orc.ptr(np.zeros(1, np.uint8))) == 5
    assert L.rs_oracle_build_matrix(200, 57, orc.ptr(np.zeros(257 * 200, np.uint8))) == 6
    assert orc.split(2, 1, b"") == 1  # ErrShortData
    rc, _ = orc.reconstruct(4, 2, np.zeros((6, 4), np.uint8), [1, 1, 1, 0, 0, 0], False)
    assert rc == 2  # ErrTooFewShards
    lens = np.array([0, 0, 0], dtype=np.uint64)
    S = np.zeros(1, dtype=np.uint64)
    assert L.rs_oracle_check_shards(3, orc.ptr(lens), 1, orc.ptr(S)) == 3  # ErrShardNoData
    lens = np.array([4, 0, 5], dtype=np.uint64)
    assert L.rs_oracle_check_shards(3, orc.ptr(lens), 1, orc.ptr(S)) == 4  # ErrShardSize
    lens = np.array([4, 0, 4], dtype=np.uint64)
    assert L.rs_oracle_check_shards(3, orc.ptr(lens), 1, orc.ptr(S)) == 0
    assert L.rs_oracle_check_shards(3, orc.ptr(lens), 0, orc.ptr(S)) == 4


def test_golden_matrices():
    d = json.load(open(os.path.join(GOLDEN, "matrices.json")))
    for key, rows in d["matrices"].items():
        k, m = map(int, key.split(","))
        assert orc.build_matrix(k, m).tolist() == rows


@pytest.mark.parametrize("k,m", [(2, 1), (4, 2), (10, 4), (16, 4), (5, 5)])
def test_golden_vectors(k, m):
    z = np.load(os.path.join(GOLDEN, f"vectors_k{k}_m{m}.npz"))
    n = k + m
    for B in (1, 6, 4099):
        block = z[f"block_{B}"]
        want = z[f"shards_{B}"]
        sh = orc.split(k, m, block.tobytes())
        sh[k:] = orc.encode(k, m, sh[:k])
        assert np.array_equal(sh, want)
        present = z[f"present_{B}"].astype(bool)
        er = want.copy()
        er[~present] = 0
        rc, rec = orc.reconstruct(k, m, er, present, False)
        assert rc == 0 and np.array_equal(rec, want)
        rc, rec = orc.reconstruct(k, m, er, present, True)
        assert rc == 0 and np.array_equal(rec[:k], want[:k])
    if (k, m) == (2, 1):
        assert z["shards_123456"][2].tolist() == [0x3B, 0x3C, 0x39]


@pytest.mark.parametrize("k,m,S,nb", [(10, 4, 26215, 6), (4, 2, 65536, 3), (16, 4, 4097, 5), (3, 2, 31, 9)])
def test_fast_simd_matches_scalar(k, m, S, nb):
    data = orc.splitmix64_bytes(0xF11EDA6 ^ S, nb * k * S).reshape(nb, k, S)
    fast = orc.encode_fast(k, m, data, threads=4)
    for b in range(nb):
        assert np.array_equal(fast[b], orc.encode(k, m, data[b])), b
    # batch reconstruct of two lost rows
    full = np.concatenate([data, fast], axis=1).copy()
    sh = full.copy()
    lost = [1, k + m - 1]
    sh[:, lost] = 0
    p = np.array([i not in lost for i in range(k + m)], dtype=np.uint8)
    assert orc.lib().rs_cpu_reconstruct_batch(k, m, orc.ptr(sh), (k + m) * S, S, nb, orc.ptr(p), 0, 4) == 0
    assert np.array_equal(sh, full)


@pytest.mark.parametrize("isa", ["avx2", "scalar"])
def test_fast_isa_paths_agree(isa):
    """Every SIMD path of the baseline gives the scalar oracle's bytes (forced by env)."""
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "import numpy as np, oracle_lib as orc\n"
        "d = orc.splitmix64_bytes(5, 3*10*1000+0).reshape(3,10,1000)\n"
        "f = orc.encode_fast(10, 4, d, threads=2)\n"
        "assert all(np.array_equal(f[b], orc.encode(10, 4, d[b])) for b in range(3))\n"
        "print(orc.lib().rs_cpu_isa().decode())\n" % os.path.dirname(os.path.abspath(__file__))
    )
    env = dict(os.environ, RS_CPU_ISA=isa)
    out = subprocess.check_output([sys.executable, "-c", code], env=env).decode()
    assert out.strip().startswith("avx2" if isa == "avx2" else "scalar")
