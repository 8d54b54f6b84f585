"""Device groups: one process driving several GPUs (include/rsmi.h; the reference's Dag Pool runs
every DagNode in one process, dag/pool/poolservice/cluster.go:28-41).

CPU tests check the partition and key-routing logic against rsmi.multi (the bench's own
partition) and the reference's keyHashSlot restated there, and that a group opens and fails
loudly without a GPU.  GPU tests run groups of one and several contexts on cuda:0 (members may
repeat a device; the 8-GPU node belongs to the driver) and compare every byte with the oracle.
"""
import ctypes

import numpy as np
import pytest

import oracle_lib as orc
import rsmi
from rsmi import multi


@pytest.mark.parametrize("nblocks", [0, 1, 2, 7, 8, 9, 4095, 4096, 8192, 10001])
@pytest.mark.parametrize("parts", [1, 2, 3, 4, 7, 8])
def test_partition_matches_bench_partition(nblocks, parts):
    got = [rsmi.partition(nblocks, parts, i) for i in range(parts)]
    assert got == [multi.partition_blocks(nblocks, parts, i) for i in range(parts)]
    # contiguous, ordered, covering, balanced
    assert got[0][0] == 0 and sum(c for _, c in got) == nblocks
    for (s0, c0), (s1, _) in zip(got, got[1:]):
        assert s1 == s0 + c0
    assert max(c for _, c in got) - min(c for _, c in got) <= 1


def test_partition_rejects_bad_arguments():
    L = rsmi.lib()
    st, cnt = ctypes.c_size_t(), ctypes.c_size_t()
    assert L.rsmi_partition(10, 0, 0, ctypes.byref(st), ctypes.byref(cnt)) == rsmi.ErrInvalidArg
    assert L.rsmi_partition(10, 2, 2, ctypes.byref(st), ctypes.byref(cnt)) == rsmi.ErrInvalidArg
    assert L.rsmi_partition(10, 2, 0, None, ctypes.byref(cnt)) == rsmi.ErrInvalidArg


@pytest.mark.parametrize("key", [b"", b"a", b"bafkreigh2akiscaildcqabsyg3dfr6chu3fgpregiymsck7e7aqa4s52zy",
                                 b"QmYwAPJzv5CZsnA625s3Xf2nemtYgPpHdWEz79ojWnPbdG", bytes(range(256))])
def test_key_slot_is_reference_hash_slot(key):
    assert rsmi.key_slot(key) == multi.crc16_ibm(key) & 0x3FFF
    if key.isascii():
        assert rsmi.key_slot(key) == multi.key_hash_slot(key.decode())


def test_member_of_key_matches_slot_ranges():
    with rsmi.DeviceGroup(10, 4, [0, 0, 0, 0, 0, 0, 0, 0]) as s:
        assert s.size() == 8
        seen = set()
        for i in range(2000):
            key = f"bafy{i:05d}".encode()
            mbr = s.member_of_key(key)
            assert mbr == multi.key_gpu(key.decode(), 8)
            seen.add(mbr)
        assert seen == set(range(8))  # every GPU owns some keys


def test_group_open_validates_like_open():
    L = rsmi.lib()
    h = ctypes.c_void_p()
    devs = (ctypes.c_int * 2)(0, 0)
    assert L.rsmi_group_open(0, 4, devs, 2, ctypes.byref(h)) == rsmi.ErrInvShardNum
    assert L.rsmi_group_open(250, 7, devs, 2, ctypes.byref(h)) == rsmi.ErrMaxShardNum
    assert L.rsmi_group_open(10, 4, devs, 0, ctypes.byref(h)) == rsmi.ErrInvalidArg
    assert L.rsmi_group_open(10, 4, None, 2, ctypes.byref(h)) == rsmi.ErrInvalidArg


def test_group_calls_fail_loudly_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    k, m, S, nb = 4, 2, 1000, 5
    data = np.zeros((nb, k * S), dtype=np.uint8)
    par = np.zeros((nb, m * S), dtype=np.uint8)
    with rsmi.DeviceGroup(k, m, [0, 0]) as s:
        with pytest.raises(rsmi.RsmiError) as e:
            s.encode_batch_host_ptr(data.ctypes.data, k * S, par.ctypes.data, m * S, S, nb)
        assert e.value.code == rsmi.ErrNoDevice
        s.encode_batch_host_ptr(data.ctypes.data, k * S, par.ctypes.data, m * S, S, 0)  # nothing to do
        with pytest.raises(rsmi.RsmiError) as e:
            s.encode_batch_host_ptr(data.ctypes.data, k * S, par.ctypes.data, m * S, 0, nb)
        assert e.value.code == rsmi.ErrShardNoData


@pytest.mark.gpu
@pytest.mark.parametrize("members", [[0], [0, 0], [0, 0, 0]])
@pytest.mark.parametrize("k,m,B,nb", [(10, 4, 262144, 7), (16, 4, 4 << 20, 5), (4, 2, 65536 + 5, 9)])
def test_group_batches_match_oracle(members, k, m, B, nb):
    """One process, one GPU, one or several member contexts: encode (+ both CRCs) and
    reconstruct over the group equal the oracle byte for byte."""
    n = k + m
    S = (B + k - 1) // k
    data = np.zeros((nb, k * S), dtype=np.uint8)
    for b in range(nb):
        data[b, :B] = orc.splitmix64_bytes(0xF11EDA6 ^ b, B)
    par = np.zeros((nb, m * S), dtype=np.uint8)
    raw16 = np.zeros((nb, n), dtype=np.uint32)
    raw32 = np.zeros((nb, n), dtype=np.uint32)
    want = orc.encode_fast(k, m, data.reshape(nb, k, S))
    with rsmi.DeviceGroup(k, m, members) as s:
        s.encode_batch_host_crcs_ptr(data.ctypes.data, k * S, par.ctypes.data, m * S, S, nb, raw16.ctypes.data,
                                     raw32.ctypes.data)
        assert np.array_equal(par.reshape(nb, m, S), want)
        rows = np.concatenate([data.reshape(nb, k, S), want], axis=1)
        for b in (0, nb // 2, nb - 1):
            for r in range(n):
                assert rsmi.crc16_entry(b"", int(raw16[b, r]), S) == orc.crc16_ibm(rows[b, r].tobytes())
                assert rsmi.crc32_entry(b"", int(raw32[b, r]), S) == orc.crc32_ieee(rows[b, r].tobytes())
        par2 = np.zeros_like(par)
        s.encode_batch_host_ptr(data.ctypes.data, k * S, par2.ctypes.data, m * S, S, nb)
        assert np.array_equal(par2, par)
        shards = np.ascontiguousarray(rows.reshape(nb, n * S))
        lost = [0, k]
        erased = shards.copy().reshape(nb, n, S)
        erased[:, lost] = 0
        erased = np.ascontiguousarray(erased.reshape(nb, n * S))
        s.reconstruct_batch_host_ptr(erased.ctypes.data, n * S, S, nb, [i not in lost for i in range(n)], False)
        assert np.array_equal(erased, shards)


def _fake_sysfs(root):
    """A sysfs tree with two GPUs on two sockets (the MI355X node shape) and a device whose
    firmware reports no node."""
    import os

    for bus, node in (("0000:05:00.0", "0\n"), ("0000:75:00.0", "1\n"), ("0000:f5:00.0", "-1\n")):
        d = os.path.join(root, "bus", "pci", "devices", bus)
        os.makedirs(d)
        with open(os.path.join(d, "numa_node"), "w") as f:
            f.write(node)
    for node, cpus in ((0, "0-3,8-11\n"), (1, "4-7,12-15\n"), (2, "16\n"), (3, "9-5\n")):
        d = os.path.join(root, "devices", "system", "node", f"node{node}")
        os.makedirs(d)
        with open(os.path.join(d, "cpulist"), "w") as f:
            f.write(cpus)
    return str(root)


def test_sysfs_device_to_numa_map(tmp_path):
    """rsmi_device_numa_node's sysfs half (bus/pci/devices/<id>/numa_node, the id in any case)
    and the node CPU lists the member threads bind to, against an injected sysfs root."""
    root = _fake_sysfs(tmp_path)
    assert rsmi.sysfs_numa_node(root, "0000:05:00.0") == 0
    assert rsmi.sysfs_numa_node(root, "0000:75:00.0") == 1
    assert rsmi.sysfs_numa_node(root, "0000:F5:00.0") == -1  # firmware without affinity
    assert rsmi.sysfs_numa_node(root, "0000:99:00.0") == -1  # no such device
    assert rsmi.sysfs_node_cpus(root, 0) == [0, 1, 2, 3, 8, 9, 10, 11]
    assert rsmi.sysfs_node_cpus(root, 1) == [4, 5, 6, 7, 12, 13, 14, 15]
    assert rsmi.sysfs_node_cpus(root, 2) == [16]
    assert rsmi.sysfs_node_cpus(root, 3) is None  # malformed range
    assert rsmi.sysfs_node_cpus(root, 7) is None  # no such node


def test_bind_thread_to_numa_node():
    """A member thread binds itself to its node: CPUs of the node the process may use, and a
    preferred-node memory policy.  Run on a thread of its own (the binding is per thread)."""
    import os
    import threading

    L = rsmi.lib()
    assert L.rsmi_bind_thread_to_numa_node(-1) == rsmi.ErrInvalidArg
    cpus0 = rsmi.sysfs_node_cpus("/sys", 0)
    if not cpus0:
        pytest.skip("no NUMA information in this container's sysfs")
    out = {}

    def run():
        out["rc"] = L.rsmi_bind_thread_to_numa_node(0)
        out["aff"] = os.sched_getaffinity(0)

    allowed = os.sched_getaffinity(0)
    t = threading.Thread(target=run)
    t.start()
    t.join()
    assert out["rc"] == rsmi.OK
    want = set(cpus0) & allowed
    assert out["aff"] == (want or allowed)
    assert os.sched_getaffinity(0) == allowed  # the calling thread is untouched


def test_group_zero_blocks_validates_like_member():
    """nblocks == 0 still validates the arguments: the group returns exactly what
    member 0's single-context call returns for the same arguments, and every member reports
    its NUMA node (-1 without a GPU)."""
    L = rsmi.lib()
    k, m, S = 4, 2, 1000
    n = k + m
    buf = np.zeros(n * S * 2, dtype=np.uint8)
    none_present = bytearray(n)
    all_present = bytearray([1] * n)
    req = bytearray([1] + [0] * (n - 1))
    with rsmi.DeviceGroup(k, m, [0, 0]) as s:
        ctx = L.rsmi_group_context(s._h, 0)
        assert s.member_numa_node(0) == s.member_numa_node(1)
        assert s.member_numa_node(2) == -1
        cases = [
            (lambda h, f: f(h, buf.ctypes.data, n * S, S, 0, (ctypes.c_uint8 * n).from_buffer(none_present), 1),
             L.rsmi_group_reconstruct_batch_host, L.rsmi_reconstruct_batch_host),
            (lambda h, f: f(h, buf.ctypes.data, S, S, 0, (ctypes.c_uint8 * n).from_buffer(all_present), 0),
             L.rsmi_group_reconstruct_batch_host, L.rsmi_reconstruct_batch_host),
            (lambda h, f: f(h, buf.ctypes.data, n * S, S, 0, (ctypes.c_uint8 * n).from_buffer(none_present),
                            (ctypes.c_uint8 * n).from_buffer(req)),
             L.rsmi_group_reconstruct_rows_batch_host, L.rsmi_reconstruct_rows_batch_host),
            (lambda h, f: f(h, buf.ctypes.data, 1, buf.ctypes.data, m * S, S, 0),
             L.rsmi_group_encode_batch_host, L.rsmi_encode_batch_host),
        ]
        for call, gfn, cfn in cases:
            assert call(s._h, gfn) == call(ctx, cfn)


@pytest.mark.gpu
def test_group_host_alloc_places_member_ranges():
    """rsmi_group_host_alloc: one page-locked buffer, zeroed, whose member ranges sit on the
    members' NUMA nodes (checked page by page with get_mempolicy(MPOL_F_NODE | MPOL_F_ADDR) where
    the box reports a node), coded in place by the group's zero-copy path against the oracle."""
    import ctypes.util

    k, m, S, nb = 10, 4, 26215, 16
    data = np.stack([orc.splitmix64_bytes(0xF11EDA6 ^ b, k * S) for b in range(nb)])
    want = orc.encode_fast(k, m, data.reshape(nb, k, S))
    libc = ctypes.CDLL(ctypes.util.find_library("c"), use_errno=True)
    with rsmi.DeviceGroup(k, m, [0, 0]) as g:
        node = g.member_numa_node(0)
        assert node == rsmi.device_numa_node(0)
        pd = g.host_alloc(k * S, nb)
        pp = g.host_alloc(m * S, nb)
        try:
            d = np.ctypeslib.as_array((ctypes.c_uint8 * (nb * k * S)).from_address(pd))
            p = np.ctypeslib.as_array((ctypes.c_uint8 * (nb * m * S)).from_address(pp))
            assert not d.any() and not p.any()
            d[:] = data.reshape(-1)
            g.encode_batch_host_ptr(pd, k * S, pp, m * S, S, nb)
            assert np.array_equal(p.reshape(nb, m, S), want)
            if node >= 0:
                mode = ctypes.c_int(-1)
                for off in range(0, nb * k * S, 1 << 16):  # MPOL_F_NODE | MPOL_F_ADDR: the page's node
                    rc = libc.syscall(239, ctypes.byref(mode), None, ctypes.c_ulong(0), ctypes.c_void_p(pd + off),
                                      ctypes.c_ulong(3))
                    assert rc == 0 and mode.value == node, (off, rc, mode.value, node)
        finally:
            g.host_free(pd)
            g.host_free(pp)
