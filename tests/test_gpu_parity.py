"""HIP path vs the CPU oracle, bit-exact (GPU tests; call through the C-ABI).

Sizes follow SURVEY.md 8(d) / Appendix B.3: every (k, m) in BASELINE.json's configs plus
a few others, block sizes {1, k-1, k, k+1, 6, 262143, 262144, 262145, ~1 MiB leaf}, and
the loss patterns {each single shard, first two data, last two parity, data+parity}.
Full-size configs are checked through size-independent properties (encode -> erase ->
reconstruct round trips) plus oracle spot checks.
"""
import ctypes
import itertools

import numpy as np
import pytest

import oracle_lib as orc

torch = pytest.importorskip("torch")
rsmi = pytest.importorskip("rsmi")

pytestmark = pytest.mark.gpu

CONFIGS = [(2, 1), (4, 2), (10, 4), (16, 4), (5, 5), (3, 2), (6, 3), (8, 4), (12, 4), (1, 1), (20, 4), (17, 3)]


def _rng_bytes(seed, n):
    return orc.splitmix64_bytes(0xF11EDA6 ^ seed, n)


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available() or rsmi.device_count() == 0:
        pytest.skip("no GPU")


def test_encode_matrix_matches_oracle():
    for k, m in CONFIGS:
        with rsmi.Codec(k, m) as c:
            got = np.frombuffer(c.encode_matrix(), dtype=np.uint8).reshape(k + m, k)
            assert np.array_equal(got, orc.build_matrix(k, m)), (k, m)


@pytest.mark.parametrize("k,m", CONFIGS)
def test_encode_block_grid(k, m):
    # SURVEY.md 8(d)'s correctness grid, with the dag-pb leaf (1 MiB + 14) and 4 MiB blocks
    sizes = sorted({1, max(1, k - 1), k, k + 1, 6, 4095, 65537, 262143, 262144, 262145, 1048576 + 14, 4 << 20})
    with rsmi.Codec(k, m) as c:
        for B in sizes:
            block = _rng_bytes(B, B).tobytes()
            got = np.frombuffer(c.encode_block(block), dtype=np.uint8).reshape(k + m, -1)
            want = orc.split(k, m, block)
            want[k:] = orc.encode(k, m, want[:k])
            assert np.array_equal(got, want), (k, m, B, c.last_kernel())


def test_reference_fixture_123456():
    """node_test.go:33 RS(2,1) "123456": shards "123", "456", parity 3b 3c 39."""
    e = rsmi.NewErasure(2, 1, 6)
    shards = e.encode_data(b"123456")
    assert shards == [b"123", b"456", bytes([0x3B, 0x3C, 0x39])]
    # TestDagNode: Get after losing any one shard returns the block
    for lost in range(3):
        sh = list(shards)
        sh[lost] = None
        e.decode_data_blocks(sh)
        assert b"".join(sh[:2])[:6] == b"123456"


def test_kat_one_encode_5_5():
    """upstream TestOneEncode: RS(5,5) with 2-byte shards."""
    with rsmi.Codec(5, 5) as c:
        data = bytearray([0, 1, 4, 5, 2, 3, 6, 7, 8, 9])
        par = bytearray(10)
        c.encode(data, par, 2)
        assert list(par) == [12, 13, 10, 11, 14, 15, 90, 91, 94, 95]


def _patterns(k, m):
    n = k + m
    pats = [[i] for i in range(n)]
    pats.append([0, 1] if k >= 2 else [0])
    pats.append([n - 2, n - 1] if m >= 2 else [n - 1])
    pats.append([0, n - 1])
    if m >= 2:
        pats.append(list(range(k - 1, k - 1 + m)))  # m losses spanning data and parity
    return [p for p in pats if len(p) <= m]


@pytest.mark.parametrize("k,m", [(2, 1), (4, 2), (10, 4), (16, 4), (5, 5), (6, 3), (20, 4)])
@pytest.mark.parametrize("S", [1, 7, 4099, 26215])
def test_reconstruct_patterns(k, m, S):
    n = k + m
    data = _rng_bytes(k * 1000 + S, k * S).reshape(k, S)
    full = np.zeros((n, S), dtype=np.uint8)
    full[:k] = data
    full[k:] = orc.encode(k, m, data)
    with rsmi.Codec(k, m) as c:
        for lost in _patterns(k, m):
            present = [i not in lost for i in range(n)]
            for data_only in (True, False):
                buf = full.copy()
                buf[lost] = 0xA5  # garbage in the missing rows
                flat = bytearray(buf.tobytes())
                c.reconstruct(flat, S, present, data_only)
                got = np.frombuffer(bytes(flat), dtype=np.uint8).reshape(n, S)
                rc, want = orc.reconstruct(k, m, buf, present, data_only)
                assert rc == 0
                assert np.array_equal(got, want), (k, m, S, lost, data_only)
                if not data_only:
                    assert np.array_equal(got, full)
                else:
                    assert np.array_equal(got[:k], full[:k])


@pytest.mark.parametrize("k,m", [(255, 1), (128, 128), (200, 56), (1, 255), (64, 64)])
@pytest.mark.parametrize("S", [5, 300])
def test_max_shard_counts(k, m, S):
    """k + m at the 256-shard limit (erasure.go:22, klauspost's maximum): the encode of every
    parity row (K > 16: the byte-granular kernel, outputs in launches of 4) and the rebuild of m
    lost rows spread over data and parity, the data rows only, and a single lost row, against the
    oracle."""
    n = k + m
    data = _rng_bytes(k * 7 + m + S, k * S).reshape(k, S)
    full = np.zeros((n, S), dtype=np.uint8)
    full[:k] = data
    full[k:] = orc.encode(k, m, data)
    with rsmi.Codec(k, m) as c:
        par = bytearray(m * S)
        c.encode(bytearray(data.tobytes()), par, S)
        assert np.array_equal(np.frombuffer(bytes(par), dtype=np.uint8).reshape(m, S), full[k:]), (k, m)
        rng = np.random.default_rng(n + S)
        for lost in (sorted(rng.choice(n, size=m, replace=False).tolist()), [0], list(range(min(m, k)))):
            present = [i not in lost for i in range(n)]
            for data_only in (True, False):
                buf = full.copy()
                buf[lost] = 0xA5
                flat = bytearray(buf.tobytes())
                c.reconstruct(flat, S, present, data_only)
                got = np.frombuffer(bytes(flat), dtype=np.uint8).reshape(n, S)
                rc, want = orc.reconstruct(k, m, buf, present, data_only)
                assert rc == 0
                assert np.array_equal(got, want), (k, m, S, lost, data_only)
                assert np.array_equal(got[:k], full[:k]), (k, m, S, lost)


def test_reconstruct_errors():
    with rsmi.Codec(4, 2) as c:
        S = 16
        flat = bytearray(6 * S)
        with pytest.raises(rsmi.RsmiError) as ei:
            c.reconstruct(flat, S, [True, True, True, False, False, False], False)
        assert ei.value.code == rsmi.ErrTooFewShards
        # nothing missing: no-op
        c.reconstruct(flat, S, [True] * 6, False)
        # data_only with all data present: no-op even if parity is missing
        c.reconstruct(flat, S, [True] * 4 + [False, False], True)


def _dev_layout(k, m, S, nblocks, pad):
    rs = (S + pad - 1) // pad * pad
    return rs, k * rs, m * rs


@pytest.mark.parametrize("k,m,S,nblocks", [(4, 2, 65536, 64), (10, 4, 26215, 96), (16, 4, 4097, 33),
                                           (2, 1, 131072, 8), (10, 4, 104858, 9), (3, 2, 17, 129)])
# waves_per_cu caps the grid, so each wave strides over several tiles (the kernels' loop)
@pytest.mark.parametrize("opts", [{}, {"waves_per_cu": 1}, {"waves_per_cu": 3}])
def test_encode_batch_dev_vs_oracle(k, m, S, nblocks, opts):
    rs, dbs, pbs = _dev_layout(k, m, S, nblocks, 256)
    host = np.zeros((nblocks, k, rs), dtype=np.uint8)
    for b in range(nblocks):
        host[b, :, :S] = _rng_bytes(b, k * S).reshape(k, S)
    d_in = torch.from_numpy(host.reshape(-1)).cuda()
    d_out = torch.full((nblocks * pbs,), 0x5A, dtype=torch.uint8, device="cuda")
    with rsmi.Codec(k, m) as c:
        for key, val in opts.items():
            c.set_option(key, val)
        c.encode_batch_dev(d_in.data_ptr(), rs, dbs, d_out.data_ptr(), rs, pbs, S, nblocks,
                           torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert "rs_fast_kernel" in c.last_kernel()
    got = d_out.cpu().numpy().reshape(nblocks, m, rs)
    want = orc.encode_fast(k, m, np.ascontiguousarray(host[:, :, :S]))
    assert np.array_equal(got[:, :, :S], want)
    # bytes at and past S in every parity row are never written
    assert (got[:, :, S:] == 0x5A).all()


@pytest.mark.parametrize("k,m,S,nblocks", [(10, 4, 26215, 5), (4, 2, 1001, 7), (20, 4, 333, 3), (3, 2, 15, 9),
                                           (10, 4, 16, 4), (10, 4, 17, 4), (16, 4, 104858, 3)])
def test_encode_batch_dev_unaligned(k, m, S, nblocks):
    """Contiguous k*S layout with odd S (the Split layout itself): the unaligned-window fast
    kernel for K <= 16 and S >= 16, the byte-granular kernel otherwise."""
    host = _rng_bytes(77, nblocks * k * S).reshape(nblocks, k, S)
    d_in = torch.from_numpy(host.reshape(-1).copy()).cuda()
    d_out = torch.zeros(nblocks * m * S, dtype=torch.uint8, device="cuda")
    with rsmi.Codec(k, m) as c:
        c.encode_batch_dev(d_in.data_ptr(), S, k * S, d_out.data_ptr(), S, m * S, S, nblocks, 0)
        torch.cuda.synchronize()
        if S % 16 == 0:  # contiguous rows of a multiple of 16 bytes are an aligned layout
            assert "rs_fast_kernel" in c.last_kernel() and ",UA" not in c.last_kernel()
        else:
            assert (",UA" if k <= 16 and S >= 16 else "generic") in c.last_kernel()
    got = d_out.cpu().numpy().reshape(nblocks, m, S)
    assert np.array_equal(got, orc.encode_fast(k, m, host))


@pytest.mark.parametrize("S", [16, 17, 31, 33, 1023, 26215])
@pytest.mark.parametrize("offset", [1, 3, 8])
@pytest.mark.parametrize("lost,data_only", [([0], True), ([2, 11], False), ([10, 12], False)])
def test_unaligned_window_kernel_guards_and_reconstruct(S, offset, lost, data_only):
    """UA kernels on rows at an odd base and pitch S + 5: guard bytes between rows stay
    untouched by encode and by the in-place reconstruct, and every row matches the oracle."""
    k, m, nb = 10, 4, 6
    n = k + m
    rs = S + 5
    bs = n * rs + 3
    host = np.full(offset + nb * bs + 32, 0x5A, dtype=np.uint8)
    data = _rng_bytes(S + offset, nb * k * S).reshape(nb, k, S)
    for b in range(nb):
        for c in range(k):
            host[offset + b * bs + c * rs:][:S] = data[b, c]
    d = torch.from_numpy(host.copy()).cuda()
    base = d.data_ptr() + offset
    with rsmi.Codec(k, m) as c:
        c.encode_batch_dev(base, rs, bs, base + k * rs, rs, bs, S, nb, 0)
        torch.cuda.synchronize()
        assert ",UA" in c.last_kernel()
        got = d.cpu().numpy()
        full = np.zeros((nb, n, S), dtype=np.uint8)
        full[:, :k] = data
        full[:, k:] = orc.encode_fast(k, m, data)
        expect = host.copy()
        for b in range(nb):
            for i in range(n):
                expect[offset + b * bs + i * rs:][:S] = full[b, i]
        assert np.array_equal(got, expect)  # rows right, every guard byte still 0x5A
        for b in range(nb):
            for i in lost:
                d[offset + b * bs + i * rs: offset + b * bs + i * rs + S] = 0
        c.reconstruct_batch_dev(base, rs, bs, S, nb, [i not in lost for i in range(n)], data_only, 0)
        torch.cuda.synchronize()
        got = d.cpu().numpy()
    for b in range(nb):
        for i in lost:
            if i >= k and data_only:
                expect[offset + b * bs + i * rs:][:S] = 0
    assert np.array_equal(got, expect)


@pytest.mark.parametrize("k,m,S,nblocks,lost,data_only",
                         [(10, 4, 26215, 64, [0], True), (16, 4, 262144 // 16, 8, [0, 9], False),
                          (4, 2, 65536, 16, [1, 4], False), (10, 4, 26215, 16, [3, 11, 12, 13], False),
                          (2, 1, 131072, 4, [1], False)])
@pytest.mark.parametrize("opts", [{}, {"waves_per_cu": 1}])
def test_reconstruct_batch_dev_vs_oracle(k, m, S, nblocks, lost, data_only, opts):
    n = k + m
    rs = (S + 255) // 256 * 256
    full = np.zeros((nblocks, n, rs), dtype=np.uint8)
    for b in range(nblocks):
        d = _rng_bytes(b + 5, k * S).reshape(k, S)
        full[b, :k, :S] = d
    full[:, k:, :S] = orc.encode_fast(k, m, np.ascontiguousarray(full[:, :k, :S]))
    erased = full.copy()
    erased[:, lost, :] = 0
    d = torch.from_numpy(erased.reshape(-1).copy()).cuda()
    present = [i not in lost for i in range(n)]
    with rsmi.Codec(k, m) as c:
        for key, val in opts.items():
            c.set_option(key, val)
        c.reconstruct_batch_dev(d.data_ptr(), rs, n * rs, S, nblocks, present, data_only,
                                torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    got = d.cpu().numpy().reshape(nblocks, n, rs)
    rows = [i for i in lost if i < k or not data_only]
    assert np.array_equal(got[:, rows, :S], full[:, rows, :S])
    untouched = [i for i in lost if i not in rows]
    assert (got[:, untouched, :] == 0).all()


def test_batch_host_matches_dev():
    k, m, S, nb = 10, 4, 26215, 300
    data = _rng_bytes(9, nb * k * S).reshape(nb, k, S)
    par = np.zeros((nb, m, S), dtype=np.uint8)
    with rsmi.Codec(k, m) as c:
        c.encode_batch_host_ptr(data.ctypes.data, k * S, par.ctypes.data, m * S, S, nb)
        assert np.array_equal(par, orc.encode_fast(k, m, data))
        full = np.concatenate([data, par], axis=1).copy()
        sh = full.copy()
        sh[:, [0, 12]] = 0
        present = [i not in (0, 12) for i in range(k + m)]
        c.reconstruct_batch_host_ptr(sh.ctypes.data, (k + m) * S, S, nb, present, False)
        assert np.array_equal(sh, full)


def test_full_size_roundtrip_rs10_4():
    """BASELINE config 3 at full size: 4096 x 256 KiB, encode, lose data shard 0,
    ReconstructData, compare with the original bytes; oracle spot check on 8 blocks."""
    k, m, nb = 10, 4, 4096
    B = 256 * 1024
    S = (B + k - 1) // k
    rs = (S + 255) // 256 * 256
    n = k + m
    g = torch.Generator(device="cuda")
    g.manual_seed(1234)
    shards = torch.randint(0, 256, (nb, n, rs), dtype=torch.uint8, device="cuda", generator=g)
    shards[:, :, S:] = 0
    # block tail padding (k*S - B = 6 bytes of the last data row) is zero like Split
    shards[:, k - 1, S - (k * S - B):S] = 0
    with rsmi.Codec(k, m) as c:
        stream = torch.cuda.current_stream().cuda_stream
        base = shards.data_ptr()
        c.encode_batch_dev(base, rs, n * rs, base + k * rs, rs, n * rs, S, nb, stream)
        torch.cuda.synchronize()
        orig = shards.clone()
        shards[:, 0, :] = 0
        c.reconstruct_batch_dev(base, rs, n * rs, S, nb, [i != 0 for i in range(n)], True, stream)
        torch.cuda.synchronize()
    assert torch.equal(shards, orig)
    idx = [0, 1, 777, 2048, 4095, 3, 1000, 4000]
    host = orig[idx].cpu().numpy()
    want = orc.encode_fast(k, m, np.ascontiguousarray(host[:, :k, :S]))
    assert np.array_equal(host[:, k:, :S], want)


def test_concurrent_contexts_threads():
    """One context shared by several threads (DagNode goroutines share one Erasure)."""
    import threading

    k, m = 10, 4
    errs = []
    with rsmi.Codec(k, m) as c:
        def worker(seed):
            try:
                for it in range(5):
                    blk = _rng_bytes(seed * 100 + it, 5000 + seed).tobytes()
                    got = np.frombuffer(c.encode_block(blk), dtype=np.uint8).reshape(k + m, -1)
                    want = orc.split(k, m, blk)
                    want[k:] = orc.encode(k, m, want[:k])
                    assert np.array_equal(got, want)
            except Exception as e:  # pragma: no cover
                errs.append(e)

        ts = [threading.Thread(target=worker, args=(i,)) for i in range(6)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    assert not errs, errs


@pytest.mark.parametrize("k,m", [(2, 1), (4, 2), (10, 4), (16, 4), (5, 5)])
def test_golden_vectors_gpu(k, m):
    """HIP path against the committed golden fixtures (tests/golden, oracle-generated)."""
    import os

    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", f"vectors_k{k}_m{m}.npz"))
    n = k + m
    e = rsmi.NewErasure(k, m, 0)
    for B in (1, 6, 4099):
        want = z[f"shards_{B}"]
        got = e.encode_data(z[f"block_{B}"].tobytes())
        assert np.array_equal(np.frombuffer(b"".join(got), dtype=np.uint8).reshape(n, -1), want)
        present = z[f"present_{B}"].astype(bool)
        sh = [bytes(want[i]) if present[i] else None for i in range(n)]
        e.decode_data_and_parity_blocks(sh)
        assert np.array_equal(np.frombuffer(b"".join(sh), dtype=np.uint8).reshape(n, -1), want)
        sh = [bytes(want[i]) if present[i] else None for i in range(n)]
        e.decode_data_blocks(sh)
        assert all(sh[i] == bytes(want[i]) for i in range(k))


class _HostBufs:
    """numpy arrays over pageable memory, or over page-locked rsmi_host_alloc memory (the
    zero-copy write-back path of the host batch calls)."""

    def __init__(self, pinned):
        self.pinned, self.ptrs = pinned, []

    def full(self, n, fill):
        if not self.pinned:
            return np.full(n, fill, dtype=np.uint8)
        p = rsmi.lib().rsmi_host_alloc(n)
        assert p
        self.ptrs.append(p)
        a = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(p))
        a[:] = fill
        return a

    def free(self):
        for p in self.ptrs:
            rsmi.lib().rsmi_host_free(p)
        self.ptrs = []


@pytest.mark.parametrize("S", [26215, 26216, 4096, 1, 104858])
@pytest.mark.parametrize("padded", [False, True])
@pytest.mark.parametrize("memory", ["pageable", "pinned", "pinned-no-zero-copy", "pinned-zero-copy-2"])
def test_batch_host_layouts(S, padded, memory):
    """Host batch entry points over odd/even S and contiguous vs padded host block strides
    (linear-copy + device repitch path for odd S, 2-D DMA path otherwise), from pageable
    and page-locked host memory (results written back by kernel stores over PCIe)."""
    bufs = _HostBufs(memory != "pageable")
    try:
        zc = {"pinned-no-zero-copy": 0, "pinned-zero-copy-2": 2}.get(memory, 1)
        _batch_host_layouts(S, padded, bufs, zc)
    finally:
        bufs.free()


def _batch_host_layouts(S, padded, bufs, zero_copy):
    k, m = 10, 4
    n = k + m
    nb = 7 if S > 50000 else 37
    gap = 13 if padded else 0
    dbs, pbs, sbs = k * S + gap, m * S + gap, n * S + gap
    data = bufs.full(nb * dbs, 0)
    blocks = _rng_bytes(S + 3, nb * k * S).reshape(nb, k, S)
    for b in range(nb):
        data[b * dbs:b * dbs + k * S] = blocks[b].reshape(-1)
    par = bufs.full(nb * pbs, 0x77)
    want = orc.encode_fast(k, m, blocks)
    with rsmi.Codec(k, m) as c:
        c.set_option("zero_copy", zero_copy)
        c.encode_batch_host_ptr(data.ctypes.data, dbs, par.ctypes.data, pbs, S, nb)
        for b in range(nb):
            assert np.array_equal(par[b * pbs:b * pbs + m * S].reshape(m, S), want[b]), b
            assert (par[b * pbs + m * S:(b + 1) * pbs] == 0x77).all()  # gaps untouched
        sh = bufs.full(nb * sbs, 0x33)
        for b in range(nb):
            sh[b * sbs:b * sbs + k * S] = blocks[b].reshape(-1)
            sh[b * sbs + k * S:b * sbs + n * S] = want[b].reshape(-1)
        full = sh.copy()
        lost = [2, 11]
        for b in range(nb):
            for r in lost:
                sh[b * sbs + r * S:b * sbs + (r + 1) * S] = 0
        c.reconstruct_batch_host_ptr(sh.ctypes.data, sbs, S, nb, [i not in lost for i in range(n)], False)
        assert np.array_equal(sh, full)


@pytest.mark.parametrize("case", ["reconstruct-rs44", "encode-rs164"])
def test_ua4_page_exact_host_buffer(case):
    """The read-heavy unaligned kernel (UA4 loads: a 4-byte-aligned dwordx4 plus the dword
    holding the window's last byte) on page-locked host memory coded in place, where the last
    row of the last block ends exactly at the end of a page-exact rsmi_group_host_alloc mapping
    and its last window is 4-aligned: no load may touch the dword at S (verdict r3 item 1: it
    used to read [S, S+4), past the mapping).  Results against the oracle.
    reconstruct-rs44: RS(4,4), S = 17, 512 blocks = 69 632 B = 17 pages; lose [0, 4, 5, 6] with
    data_only: survivors 1, 2, 3, 7 (row 7 ends the buffer), one output row -> K=4, MT=1, NT=2.
    encode-rs164: RS(16,4), S = 20, 64 blocks of data rows = 20 480 B = 5 pages (data row 15 of
    the last block ends the buffer), parity in a second mapping -> K=16, MT=4, NT=2.
    Reference: data_recovery.go:115-167 (the repair's reconstruct), erasure.go:55-60."""
    import mmap

    page = mmap.PAGESIZE
    if case == "reconstruct-rs44":
        k, m, S, nb = 4, 4, 17, 512
        n = k + m
        assert (nb * n * S) % page == 0
        blocks = _rng_bytes(44, nb * k * S).reshape(nb, k, S)
        full = np.concatenate([blocks, orc.encode_fast(k, m, blocks)], axis=1)
        lost = [0, 4, 5, 6]
        with rsmi.DeviceGroup(k, m, [0]) as g:
            p = g.host_alloc(n * S, nb)
            try:
                sh = np.ctypeslib.as_array((ctypes.c_uint8 * (nb * n * S)).from_address(p)).reshape(nb, n, S)
                sh[:] = full
                sh[:, lost] = 0xEE
                g.reconstruct_batch_host_ptr(p, n * S, S, nb, [i not in lost for i in range(n)], True)
                kern = rsmi.lib().rsmi_last_kernel(rsmi.lib().rsmi_group_context(g._h, 0)).decode()
                assert kern == "rs_fast_kernel<K=4,MT=1,NT=2>,UA", kern
                assert np.array_equal(sh[:, 0], full[:, 0])
                assert (sh[:, 4:7] == 0xEE).all()  # data_only: parity rows not rebuilt
                assert np.array_equal(sh[:, [1, 2, 3, 7]], full[:, [1, 2, 3, 7]])
            finally:
                g.host_free(p)
    else:
        k, m, S, nb = 16, 4, 20, 64
        assert (nb * k * S) % page == 0
        blocks = _rng_bytes(164, nb * k * S).reshape(nb, k, S)
        want = orc.encode_fast(k, m, blocks)
        with rsmi.DeviceGroup(k, m, [0]) as g:
            pd = g.host_alloc(k * S, nb)
            pp = g.host_alloc(m * S, nb)
            try:
                d = np.ctypeslib.as_array((ctypes.c_uint8 * (nb * k * S)).from_address(pd)).reshape(nb, k, S)
                par = np.ctypeslib.as_array((ctypes.c_uint8 * (nb * m * S)).from_address(pp)).reshape(nb, m, S)
                d[:] = blocks
                g.encode_batch_host_ptr(pd, k * S, pp, m * S, S, nb)
                kern = rsmi.lib().rsmi_last_kernel(rsmi.lib().rsmi_group_context(g._h, 0)).decode()
                assert kern == "rs_fast_kernel<K=16,MT=4,NT=2>,UA", kern
                assert np.array_equal(par, want)
            finally:
                g.host_free(pd)
                g.host_free(pp)


@pytest.mark.parametrize("small", [0, 1 << 30])
@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("k,m,B,nb", [(10, 4, 262144, 3), (10, 4, 4099, 5), (4, 2, 6, 2), (2, 1, 131072, 2),
                                      (16, 4, 1048576 + 14, 1)])
def test_host_small_call_path_matches_pipeline(small, pinned, k, m, B, nb):
    """Host batch calls through the zero-copy single-kernel path (small_call_bytes large) and
    through the copy-engine pipeline (small_call_bytes 0) give the oracle's bytes, from
    pageable and page-locked buffers, for encode and for both reconstruct modes."""
    import ctypes

    n = k + m
    S = (B + k - 1) // k
    L = rsmi.lib()
    nbytes = nb * n * S
    if pinned:
        ptr = L.rsmi_host_alloc(nbytes)
        arr = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(ptr))
    else:
        arr = np.zeros(nbytes, dtype=np.uint8)
        ptr = arr.ctypes.data
    try:
        sh = arr.reshape(nb, n, S)
        sh[:] = 0
        rng = np.random.default_rng(B + nb)
        data = rng.integers(0, 256, size=(nb, k * S), dtype=np.uint8)
        data[:, B:] = 0
        sh[:, :k] = data.reshape(nb, k, S)
        want = orc.encode_fast(k, m, np.ascontiguousarray(sh[:, :k]))
        with rsmi.Codec(k, m) as c:
            c.set_option("small_call_bytes", small)
            c.encode_batch_host_ptr(ptr, n * S, ptr + k * S, n * S, S, nb)
            assert np.array_equal(sh[:, k:], want)
            full = sh.copy()
            pats = [([0], True), ([k], True)] + ([([1, n - 1], False)] if m >= 2 else [([n - 1], False)])
            for lost, data_only in pats:
                sh[:, lost] = 0xEE
                present = [i not in lost for i in range(n)]
                c.reconstruct_batch_host_ptr(ptr, n * S, S, nb, present, data_only)
                for i in lost:
                    if i < k or not data_only:
                        assert np.array_equal(sh[:, i], full[:, i]), (lost, data_only, i)
                    else:
                        assert (sh[:, i] == 0xEE).all()
                sh[:] = full
    finally:
        if pinned:
            L.rsmi_host_free(ptr)
