"""ctypes loader for the CPU oracle (oracle/build/liboracle_rs.so) -- test infrastructure.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "build", "liboracle_rs.so")

_L = None


def lib():
    global _L
    if _L is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = ctypes.CDLL(ORACLE_SO)
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        L.rs_oracle_gal_mul.restype = ctypes.c_uint8
        L.rs_oracle_gal_mul.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.rs_oracle_gal_exp.restype = ctypes.c_uint8
        L.rs_oracle_gal_exp.argtypes = [ctypes.c_uint8, i]
        L.rs_oracle_invert.argtypes = [vp, vp, i]
        L.rs_oracle_build_matrix.argtypes = [i, i, vp]
        L.rs_oracle_shard_size.restype = sz
        L.rs_oracle_shard_size.argtypes = [sz, i]
        L.rs_oracle_split.argtypes = [i, i, vp, sz, vp]
        L.rs_oracle_encode.argtypes = [i, i, vp, sz]
        L.rs_oracle_reconstruct.argtypes = [i, i, vp, sz, vp, i]
        L.rs_oracle_check_shards.argtypes = [i, vp, i, vp]
        L.rs_cpu_encode_batch.argtypes = [i, i, vp, sz, vp, sz, sz, sz, i]
        L.rs_cpu_reconstruct_batch.argtypes = [i, i, vp, sz, sz, sz, vp, i, i]
        L.rs_cpu_isa.restype = ctypes.c_char_p
        L.rs_oracle_crc16_ibm.restype = ctypes.c_uint16
        L.rs_oracle_crc16_ibm.argtypes = [vp, sz]
        L.rs_oracle_datanode_entry_crc.restype = ctypes.c_uint32
        L.rs_oracle_datanode_entry_crc.argtypes = [vp, sz, vp, sz]
        L.rs_oracle_crc32_ieee.restype = ctypes.c_uint32
        L.rs_oracle_crc32_ieee.argtypes = [vp, sz]
        L.rs_oracle_mutcask_entry_crc.restype = ctypes.c_uint32
        L.rs_oracle_mutcask_entry_crc.argtypes = [ctypes.c_uint32, vp, sz, vp, sz]
        _L = L
    return _L


def ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def build_matrix(k, m) -> np.ndarray:
    out = np.zeros((k + m) * k, dtype=np.uint8)
    rc = lib().rs_oracle_build_matrix(k, m, ptr(out))
    assert rc == 0, rc
    return out.reshape(k + m, k)


def encode(k, m, data: np.ndarray) -> np.ndarray:
    """data: (k, S) uint8 -> parity (m, S) via the scalar oracle."""
    S = data.shape[1]
    sh = np.zeros((k + m, S), dtype=np.uint8)
    sh[:k] = data
    rc = lib().rs_oracle_encode(k, m, ptr(sh), S)
    assert rc == 0, rc
    return sh[k:].copy()


def encode_fast(k, m, data: np.ndarray, threads=8) -> np.ndarray:
    """data: (nblocks, k, S) -> parity (nblocks, m, S) via the multi-threaded SIMD oracle."""
    nb, kk, S = data.shape
    data = np.ascontiguousarray(data)
    par = np.zeros((nb, m, S), dtype=np.uint8)
    rc = lib().rs_cpu_encode_batch(k, m, ptr(data), k * S, ptr(par), m * S, S, nb, threads)
    assert rc == 0, rc
    return par


def split(k, m, block: bytes) -> np.ndarray:
    S = lib().rs_oracle_shard_size(len(block), k)
    sh = np.zeros((k + m) * S, dtype=np.uint8)
    src = np.frombuffer(block, dtype=np.uint8).copy()
    rc = lib().rs_oracle_split(k, m, ptr(src), len(block), ptr(sh))
    if rc:
        return rc
    return sh.reshape(k + m, S)


def reconstruct(k, m, shards: np.ndarray, present, data_only: bool):
    """shards: (k+m, S); rows with present[i]==False are overwritten."""
    sh = np.ascontiguousarray(shards).copy()
    p = np.array([1 if x else 0 for x in present], dtype=np.uint8)
    rc = lib().rs_oracle_reconstruct(k, m, ptr(sh), sh.shape[1], ptr(p), 1 if data_only else 0)
    return rc, sh


def splitmix64_bytes(seed: int, nbytes: int) -> np.ndarray:
    """Deterministic input bytes (splitmix64, seed 0xF11EDA6 ^ block index)."""
    n = (nbytes + 7) // 8
    with np.errstate(over="ignore"):
        x = (np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)) + np.uint64(seed)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    return x.view(np.uint8)[:nbytes].copy()


def crc16_ibm(data) -> int:
    """howeyc Checksum(data, IBMTable) via the byte-serial oracle (crc16_oracle.c)."""
    a = np.frombuffer(bytes(data), dtype=np.uint8).copy()
    return int(lib().rs_oracle_crc16_ibm(ptr(a) if a.size else None, a.size))


def datanode_entry_crc(meta, data) -> int:
    """The checksum dag/node/datanode/server.go:70 stores for an entry (meta, data)."""
    m = np.frombuffer(bytes(meta), dtype=np.uint8).copy()
    d = np.frombuffer(bytes(data), dtype=np.uint8).copy()
    return int(lib().rs_oracle_datanode_entry_crc(ptr(m) if m.size else None, m.size,
                                                  ptr(d) if d.size else None, d.size))


def crc32_ieee(data) -> int:
    """Go crc32.ChecksumIEEE(data) via the bit-serial oracle (crc32_oracle.c)."""
    a = np.frombuffer(bytes(data), dtype=np.uint8).copy()
    return int(lib().rs_oracle_crc32_ieee(ptr(a) if a.size else None, a.size))


def mutcask_entry_crc(entry_crc16: int, meta, data) -> int:
    """The value checksum kv/mutcask/cask.go:73-79 stores for a datanode entry (meta, data)."""
    m = np.frombuffer(bytes(meta), dtype=np.uint8).copy()
    d = np.frombuffer(bytes(data), dtype=np.uint8).copy()
    return int(lib().rs_oracle_mutcask_entry_crc(entry_crc16, ptr(m) if m.size else None, m.size,
                                                 ptr(d) if d.size else None, d.size))


def entry_head(meta, data_len: int) -> bytes:
    """|meta size (4 LE)|data size (4 LE)|meta| -- the checksummed bytes before the data."""
    return len(meta).to_bytes(4, "little") + data_len.to_bytes(4, "little") + bytes(meta)
