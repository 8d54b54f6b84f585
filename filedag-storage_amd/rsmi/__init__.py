"""Python host mirror of filedag-storage's Dag Node erasure seam over librsmi.so.

`Erasure` mirrors dag/node/dagnode/erasure.go method for method (NewErasure,
EncodeData, DecodeDataBlocks, DecodeDataAndParityBlocks, ShardSize) with the same
argument meaning and error behaviour; every byte it produces comes out of the gfx950
HIP kernels behind the C-ABI in include/rsmi.h.  There is no CPU fallback: if the
library or a GPU is missing the calls raise.

`Codec` exposes the batched device-resident and host entry points used by bench.py.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
# RSMI_LIB: a diagnostic build of the library (tools/Makefile variants) for A/B runs
LIB_PATH = os.environ.get("RSMI_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "librsmi.so")

# status codes (include/rsmi.h) -- names follow the upstream sentinels
OK = 0
ErrShortData = 1
ErrTooFewShards = 2
ErrShardNoData = 3
ErrShardSize = 4
ErrInvShardNum = 5
ErrMaxShardNum = 6
ErrSingular = 7
ErrInvalidArg = 8
ErrDevice = 100
ErrNoDevice = 101
ErrHost = 102


class RsmiError(Exception):
    def __init__(self, code: int, msg: str = ""):
        self.code = code
        super().__init__(f"rsmi error {code}: {msg or status_string(code)}")


_lib = None


def lib() -> ctypes.CDLL:
    """Load librsmi.so (fails loudly when it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"librsmi.so not built at {LIB_PATH}: run `python __graft_entry__.py build`")
    # One HIP runtime per process: torch ships its own libamdhip64 (soname libamdhip64.so.7).
    # Loaded first, it also satisfies librsmi's dependency; loaded after librsmi, a second
    # runtime (ROCm's) would already own the device and torch would report no GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    c_size = ctypes.c_size_t
    u8p = ctypes.c_void_p
    sig = {
        "rsmi_open": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
        "rsmi_close": (None, [ctypes.c_void_p]),
        "rsmi_warm": (ctypes.c_int, [ctypes.c_void_p]),
        "rsmi_device_count": (ctypes.c_int, []),
        "rsmi_status_string": (ctypes.c_char_p, [ctypes.c_int]),
        "rsmi_abi_version": (ctypes.c_int, []),
        "rsmi_shard_size": (c_size, [c_size, ctypes.c_int]),
        "rsmi_recommended_pitch": (c_size, [c_size]),
        "rsmi_encode_matrix": (ctypes.c_int, [ctypes.c_void_p, u8p]),
        "rsmi_check_shards": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(c_size), ctypes.c_int, ctypes.POINTER(c_size)]),
        "rsmi_decode_matrix": (ctypes.c_int, [ctypes.c_void_p, u8p, u8p, ctypes.POINTER(ctypes.c_int)]),
        "rsmi_encode_block": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, u8p]),
        "rsmi_encode": (ctypes.c_int, [ctypes.c_void_p, u8p, u8p, c_size]),
        "rsmi_reconstruct": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, u8p, ctypes.c_int]),
        "rsmi_encode_batch_host": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, u8p, c_size, c_size, c_size]),
        "rsmi_reconstruct_batch_host": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, c_size, c_size, u8p, ctypes.c_int]),
        "rsmi_reconstruct_rows_batch_host": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, c_size, c_size, u8p, u8p]),
        "rsmi_reconstruct_rows_batch_dev": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, c_size, c_size, c_size, u8p, u8p, ctypes.c_void_p]),
        "rsmi_host_alloc": (ctypes.c_void_p, [c_size]),
        "rsmi_host_free": (None, [ctypes.c_void_p]),
        "rsmi_encode_batch_dev": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, c_size, u8p, c_size, c_size, c_size, c_size, ctypes.c_void_p]),
        "rsmi_reconstruct_batch_dev": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, c_size, c_size, c_size, u8p, ctypes.c_int, ctypes.c_void_p]),
        "rsmi_encode_block_coalesced": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, u8p, ctypes.c_void_p]),
        "rsmi_encode_block_coalesced_crcs": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, u8p, ctypes.c_void_p,
                                                            ctypes.c_void_p]),
        "rsmi_reconstruct_coalesced": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, u8p, ctypes.c_int]),
        "rsmi_get_stat": (ctypes.c_long, [ctypes.c_void_p, ctypes.c_char_p]),
        "rsmi_crc16_ibm": (ctypes.c_uint16, [u8p, c_size]),
        "rsmi_crc16_entry": (ctypes.c_uint16, [u8p, c_size, ctypes.c_uint32, c_size]),
        "rsmi_crc16_rows_dev": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, c_size, ctypes.c_int, c_size, c_size,
                                               ctypes.c_void_p, c_size, ctypes.c_void_p]),
        "rsmi_encode_batch_host_crc": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, u8p, c_size, c_size, c_size,
                                                      ctypes.c_void_p]),
        "rsmi_encode_block_crc": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, u8p, ctypes.c_void_p]),
        "rsmi_encode_batch_dev_crc": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, c_size, u8p, c_size, c_size, c_size,
                                                     c_size, ctypes.c_void_p, ctypes.c_void_p]),
        "rsmi_crc_rows_host": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, c_size, c_size, ctypes.c_void_p,
                                              ctypes.c_void_p]),
        "rsmi_crc32_ieee": (ctypes.c_uint32, [u8p, c_size]),
        "rsmi_crc32_entry": (ctypes.c_uint32, [u8p, c_size, ctypes.c_uint32, c_size]),
        "rsmi_crc32_rows_dev": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, c_size, ctypes.c_int, c_size, c_size,
                                               ctypes.c_void_p, c_size, ctypes.c_void_p]),
        "rsmi_encode_batch_host_crcs": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, u8p, c_size, c_size, c_size,
                                                       ctypes.c_void_p, ctypes.c_void_p]),
        "rsmi_reconstruct_batch_host_verify": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, c_size, c_size, u8p,
                                                              ctypes.c_int, ctypes.c_void_p]),
        "rsmi_reconstruct_rows_batch_host_crcs": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, c_size, c_size, u8p,
                                                                 u8p, ctypes.c_void_p, ctypes.c_void_p]),
        "rsmi_set_option": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_long]),
        "rsmi_group_open": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_void_p)]),
        "rsmi_group_close": (None, [ctypes.c_void_p]),
        "rsmi_group_size": (ctypes.c_int, [ctypes.c_void_p]),
        "rsmi_group_context": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_int]),
        "rsmi_partition": (ctypes.c_int, [c_size, ctypes.c_int, ctypes.c_int, ctypes.POINTER(c_size),
                                          ctypes.POINTER(c_size)]),
        "rsmi_key_slot": (ctypes.c_int, [u8p, c_size]),
        "rsmi_group_member_of_key": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size]),
        "rsmi_group_member_numa_node": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
        "rsmi_group_host_alloc": (ctypes.c_void_p, [ctypes.c_void_p, c_size, c_size]),
        "rsmi_group_host_free": (None, [ctypes.c_void_p, ctypes.c_void_p]),
        "rsmi_device_numa_node": (ctypes.c_int, [ctypes.c_int]),
        "rsmi_sysfs_numa_node": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p]),
        "rsmi_sysfs_node_cpus": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                                ctypes.c_int]),
        "rsmi_bind_thread_to_numa_node": (ctypes.c_int, [ctypes.c_int]),
        "rsmi_group_encode_batch_host": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, u8p, c_size, c_size, c_size]),
        "rsmi_group_encode_batch_host_crcs": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, u8p, c_size, c_size, c_size,
                                                           ctypes.c_void_p, ctypes.c_void_p]),
        "rsmi_group_reconstruct_batch_host": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, c_size, c_size, u8p,
                                                           ctypes.c_int]),
        "rsmi_group_reconstruct_rows_batch_host": (ctypes.c_int, [ctypes.c_void_p, u8p, c_size, c_size, c_size, u8p,
                                                                u8p]),
        "rsmi_last_kernel": (ctypes.c_char_p, [ctypes.c_void_p]),
        "rsmi_set_wait_hook": (None, [ctypes.c_void_p, ctypes.c_void_p]),
        "rsmi_run_wait_hook": (ctypes.c_int, []),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def status_string(code: int) -> str:
    try:
        return lib().rsmi_status_string(code).decode()
    except Exception:  # pragma: no cover - only when the library is absent
        return "unknown"


def _check(rc: int) -> None:
    if rc != OK:
        raise RsmiError(rc)


def ceil_frac(numerator: int, denominator: int) -> int:
    """utils.go:6-21 ceilFrac."""
    if denominator == 0:
        return 0
    if denominator < 0:
        numerator, denominator = -numerator, -denominator
    q = abs(numerator) // denominator * (1 if numerator >= 0 else -1)
    if numerator > 0 and numerator % denominator != 0:
        q += 1
    return q


def _buf(b) -> ctypes.Array:
    return (ctypes.c_uint8 * len(b)).from_buffer(b)


class Codec:
    """One RS(k, m) context on one device (rsmi_open)."""

    def __init__(self, k: int, m: int, device: int = 0):
        h = ctypes.c_void_p()
        _check(lib().rsmi_open(k, m, device, ctypes.byref(h)))
        self.k, self.m, self.n, self.device = k, m, k + m, device
        self._h = h

    def close(self) -> None:
        if self._h:
            lib().rsmi_close(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- host-only helpers
    def encode_matrix(self) -> bytes:
        out = bytearray(self.n * self.k)
        _check(lib().rsmi_encode_matrix(self._h, ctypes.addressof(_buf(out))))
        return bytes(out)

    def decode_matrix(self, present: Sequence[bool]):
        p = bytearray(1 if x else 0 for x in present)
        out = bytearray(self.k * self.k)
        used = (ctypes.c_int * self.k)()
        _check(lib().rsmi_decode_matrix(self._h, ctypes.addressof(_buf(p)), ctypes.addressof(_buf(out)), used))
        return bytes(out), list(used)

    def set_option(self, key: str, value: int) -> None:
        _check(lib().rsmi_set_option(self._h, key.encode(), int(value)))

    def warm(self) -> None:
        """rsmi_warm: bind the device and bring up every coalescing lane now."""
        _check(lib().rsmi_warm(self._h))

    def last_kernel(self) -> str:
        return lib().rsmi_last_kernel(self._h).decode()

    # -- host memory
    def encode_block(self, block: bytes) -> bytes:
        S = lib().rsmi_shard_size(len(block), self.k)
        out = bytearray(self.n * S)
        src = bytearray(block)
        _check(lib().rsmi_encode_block(self._h, ctypes.addressof(_buf(src)) if src else None, len(block),
                                       ctypes.addressof(_buf(out)) if out else None))
        return bytes(out)

    def encode(self, data: bytearray, parity: bytearray, S: int) -> None:
        _check(lib().rsmi_encode(self._h, ctypes.addressof(_buf(data)), ctypes.addressof(_buf(parity)), S))

    def reconstruct(self, shards: bytearray, S: int, present: Sequence[bool], data_only: bool) -> None:
        p = bytearray(1 if x else 0 for x in present)
        _check(lib().rsmi_reconstruct(self._h, ctypes.addressof(_buf(shards)), S, ctypes.addressof(_buf(p)),
                                      1 if data_only else 0))

    def encode_batch_host_ptr(self, data_ptr: int, data_bs: int, parity_ptr: int, parity_bs: int, S: int,
                              nblocks: int) -> None:
        _check(lib().rsmi_encode_batch_host(self._h, data_ptr, data_bs, parity_ptr, parity_bs, S, nblocks))

    def reconstruct_batch_host_ptr(self, ptr: int, bs: int, S: int, nblocks: int, present: Sequence[bool],
                                   data_only: bool) -> None:
        p = bytearray(1 if x else 0 for x in present)
        _check(lib().rsmi_reconstruct_batch_host(self._h, ptr, bs, S, nblocks, ctypes.addressof(_buf(p)),
                                                 1 if data_only else 0))

    def reconstruct_rows_batch_host_ptr(self, ptr: int, bs: int, S: int, nblocks: int, present: Sequence[bool],
                                        required: Sequence[bool]) -> None:
        p = bytearray(1 if x else 0 for x in present)
        q = bytearray(1 if x else 0 for x in required)
        _check(lib().rsmi_reconstruct_rows_batch_host(self._h, ptr, bs, S, nblocks, ctypes.addressof(_buf(p)),
                                                      ctypes.addressof(_buf(q))))

    def encode_block_crc(self, block: bytes):
        """encode_block plus R(shard) of every shard (GPU CRC-16, include/rsmi.h)."""
        S = lib().rsmi_shard_size(len(block), self.k)
        out = bytearray(self.n * S)
        src = bytearray(block)
        raw = (ctypes.c_uint32 * self.n)()
        _check(lib().rsmi_encode_block_crc(self._h, ctypes.addressof(_buf(src)) if src else None, len(block),
                                           ctypes.addressof(_buf(out)) if out else None, raw))
        return bytes(out), list(raw)

    def encode_block_coalesced(self, block: bytes, want_raw: bool = False):
        """encode_block, batched with concurrent callers on this context (group commit)."""
        S = lib().rsmi_shard_size(len(block), self.k)
        out = bytearray(self.n * S)
        src = bytearray(block)
        raw = (ctypes.c_uint32 * self.n)() if want_raw else None
        _check(lib().rsmi_encode_block_coalesced(self._h, ctypes.addressof(_buf(src)) if src else None, len(block),
                                                 ctypes.addressof(_buf(out)) if out else None, raw))
        return (bytes(out), list(raw)) if want_raw else bytes(out)

    def reconstruct_coalesced(self, shards: bytearray, S: int, present: Sequence[bool], data_only: bool) -> None:
        """reconstruct, batched with concurrent callers on this context (group commit)."""
        p = bytearray(1 if x else 0 for x in present)
        _check(lib().rsmi_reconstruct_coalesced(self._h, ctypes.addressof(_buf(shards)), S,
                                                ctypes.addressof(_buf(p)), 1 if data_only else 0))

    def stat(self, key: str) -> int:
        return lib().rsmi_get_stat(self._h, key.encode())

    def encode_batch_host_crc_ptr(self, data_ptr: int, data_bs: int, parity_ptr: int, parity_bs: int, S: int,
                                  nblocks: int, raw_ptr: int) -> None:
        _check(lib().rsmi_encode_batch_host_crc(self._h, data_ptr, data_bs, parity_ptr, parity_bs, S, nblocks,
                                                raw_ptr))

    def encode_batch_dev_crc(self, d_data: int, data_rs: int, data_bs: int, d_parity: int, parity_rs: int,
                             parity_bs: int, S: int, nblocks: int, d_raw: int, stream: int = 0) -> None:
        _check(lib().rsmi_encode_batch_dev_crc(self._h, d_data, data_rs, data_bs, d_parity, parity_rs, parity_bs, S,
                                               nblocks, d_raw, stream or None))

    def crc16_rows_dev(self, d_rows: int, rs: int, bs: int, nrows: int, S: int, nblocks: int, d_out: int,
                       out_bs: int, stream: int = 0) -> None:
        _check(lib().rsmi_crc16_rows_dev(self._h, d_rows, rs, bs, nrows, S, nblocks, d_out, out_bs,
                                         stream or None))

    def crc_rows_host_ptr(self, rows_ptr: int, row_stride: int, nrows: int, S: int, raw16_ptr: Optional[int],
                          raw32_ptr: Optional[int]) -> None:
        _check(lib().rsmi_crc_rows_host(self._h, rows_ptr, row_stride, nrows, S, raw16_ptr or None,
                                        raw32_ptr or None))

    def crc32_rows_dev(self, d_rows: int, rs: int, bs: int, nrows: int, S: int, nblocks: int, d_out: int,
                       out_bs: int, stream: int = 0) -> None:
        """R32(row) of the mutcask value checksum (CRC-32 IEEE, raw) for every row, on the device."""
        _check(lib().rsmi_crc32_rows_dev(self._h, d_rows, rs, bs, nrows, S, nblocks, d_out, out_bs,
                                         stream or None))

    def reconstruct_batch_host_verify_ptr(self, ptr: int, bs: int, S: int, nblocks: int, present: Sequence[bool],
                                          data_only: bool, raw16_ptr: int) -> None:
        """reconstruct_batch_host_ptr that also writes R(row) of the k survivor rows it read into
        raw16_ptr[b*k + c] (uint32; survivors = the first k present shards)."""
        p = bytearray(1 if x else 0 for x in present)
        _check(lib().rsmi_reconstruct_batch_host_verify(self._h, ptr, bs, S, nblocks, ctypes.addressof(_buf(p)),
                                                        1 if data_only else 0, raw16_ptr))

    def reconstruct_rows_batch_host_crcs_ptr(self, shards_ptr: int, block_stride: int, S: int, nblocks: int,
                                             present: Sequence[bool], required: Sequence[bool],
                                             raw16_ptr: Optional[int], raw32_ptr: Optional[int]) -> None:
        p = bytearray(1 if x else 0 for x in present)
        q = bytearray(1 if x else 0 for x in required)
        _check(lib().rsmi_reconstruct_rows_batch_host_crcs(self._h, shards_ptr, block_stride, S, nblocks,
                                                           ctypes.addressof(_buf(p)), ctypes.addressof(_buf(q)),
                                                           raw16_ptr or None, raw32_ptr or None))

    def encode_batch_host_crcs_ptr(self, data_ptr: int, data_bs: int, parity_ptr: int, parity_bs: int, S: int,
                                   nblocks: int, raw16_ptr: Optional[int], raw32_ptr: Optional[int]) -> None:
        _check(lib().rsmi_encode_batch_host_crcs(self._h, data_ptr, data_bs, parity_ptr, parity_bs, S, nblocks,
                                                 raw16_ptr or None, raw32_ptr or None))

    # -- device memory (raw pointers, e.g. torch tensor.data_ptr()); stream = hipStream_t
    def encode_batch_dev(self, d_data: int, data_rs: int, data_bs: int, d_parity: int, parity_rs: int,
                         parity_bs: int, S: int, nblocks: int, stream: int = 0) -> None:
        _check(lib().rsmi_encode_batch_dev(self._h, d_data, data_rs, data_bs, d_parity, parity_rs, parity_bs, S,
                                           nblocks, stream or None))

    def reconstruct_rows_batch_dev(self, d_shards: int, rs: int, bs: int, S: int, nblocks: int,
                                   present: Sequence[bool], required: Sequence[bool], stream: int = 0) -> None:
        p = bytearray(1 if x else 0 for x in present)
        q = bytearray(1 if x else 0 for x in required)
        _check(lib().rsmi_reconstruct_rows_batch_dev(self._h, d_shards, rs, bs, S, nblocks, ctypes.addressof(_buf(p)),
                                                     ctypes.addressof(_buf(q)), stream or None))

    def reconstruct_batch_dev(self, d_shards: int, rs: int, bs: int, S: int, nblocks: int,
                              present: Sequence[bool], data_only: bool, stream: int = 0) -> None:
        p = bytearray(1 if x else 0 for x in present)
        _check(lib().rsmi_reconstruct_batch_dev(self._h, d_shards, rs, bs, S, nblocks, ctypes.addressof(_buf(p)),
                                                1 if data_only else 0, stream or None))


class DeviceGroup:
    """Several GPUs from one process (rsmi_group_open): batches split into contiguous block
    ranges, one per member context, run concurrently (include/rsmi.h "device groups").  The
    reference's Dag Pool runs all its DagNodes in one process (dag/pool/poolservice/cluster.go:
    28-41); members may repeat a device."""

    def __init__(self, k: int, m: int, devices: Sequence[int]):
        arr = (ctypes.c_int * len(devices))(*devices)
        h = ctypes.c_void_p()
        _check(lib().rsmi_group_open(k, m, arr, len(devices), ctypes.byref(h)))
        self.k, self.m, self.n, self.devices = k, m, k + m, list(devices)
        self._h = h

    def close(self) -> None:
        if self._h:
            lib().rsmi_group_close(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def size(self) -> int:
        return lib().rsmi_group_size(self._h)

    def member_of_key(self, key: bytes) -> int:
        b = bytearray(key)
        return lib().rsmi_group_member_of_key(self._h, ctypes.addressof(_buf(b)) if b else None, len(b))

    def member_numa_node(self, i: int) -> int:
        return lib().rsmi_group_member_numa_node(self._h, i)

    def host_alloc(self, block_bytes: int, nblocks: int) -> int:
        """Page-locked buffer whose member block ranges sit on the members' NUMA nodes."""
        p = lib().rsmi_group_host_alloc(self._h, block_bytes, nblocks)
        if not p:  # mmap, NUMA placement or page-locking the host range failed
            raise RsmiError(ErrHost, "rsmi_group_host_alloc failed")
        return p

    def host_free(self, p: int) -> None:
        lib().rsmi_group_host_free(self._h, p)

    def encode_batch_host_ptr(self, data_ptr: int, data_bs: int, parity_ptr: int, parity_bs: int, S: int,
                              nblocks: int) -> None:
        _check(lib().rsmi_group_encode_batch_host(self._h, data_ptr, data_bs, parity_ptr, parity_bs, S, nblocks))

    def encode_batch_host_crcs_ptr(self, data_ptr: int, data_bs: int, parity_ptr: int, parity_bs: int, S: int,
                                   nblocks: int, raw16_ptr: Optional[int], raw32_ptr: Optional[int]) -> None:
        _check(lib().rsmi_group_encode_batch_host_crcs(self._h, data_ptr, data_bs, parity_ptr, parity_bs, S, nblocks,
                                                     raw16_ptr or None, raw32_ptr or None))

    def reconstruct_batch_host_ptr(self, ptr: int, bs: int, S: int, nblocks: int, present: Sequence[bool],
                                   data_only: bool) -> None:
        p = bytearray(1 if x else 0 for x in present)
        _check(lib().rsmi_group_reconstruct_batch_host(self._h, ptr, bs, S, nblocks, ctypes.addressof(_buf(p)),
                                                     1 if data_only else 0))

    def reconstruct_rows_batch_host_ptr(self, ptr: int, bs: int, S: int, nblocks: int, present: Sequence[bool],
                                        required: Sequence[bool]) -> None:
        p = bytearray(1 if x else 0 for x in present)
        q = bytearray(1 if x else 0 for x in required)
        _check(lib().rsmi_group_reconstruct_rows_batch_host(self._h, ptr, bs, S, nblocks, ctypes.addressof(_buf(p)),
                                                          ctypes.addressof(_buf(q))))


def device_numa_node(device: int) -> int:
    return lib().rsmi_device_numa_node(device)


def sysfs_numa_node(sysfs_root: str, pci_bus_id: str) -> int:
    return lib().rsmi_sysfs_numa_node(sysfs_root.encode(), pci_bus_id.encode())


def sysfs_node_cpus(sysfs_root: str, node: int) -> Optional[list]:
    """CPU ids of a NUMA node from <sysfs_root>/devices/system/node/node<N>/cpulist (None if absent)."""
    L = lib()
    n = L.rsmi_sysfs_node_cpus(sysfs_root.encode(), node, None, 0)
    if n < 0:
        return None
    arr = (ctypes.c_int * max(n, 1))()
    L.rsmi_sysfs_node_cpus(sysfs_root.encode(), node, arr, n)
    return list(arr[:n])


def partition(nblocks: int, parts: int, i: int):
    """rsmi_partition: (start, count) of member i's contiguous range."""
    st, cnt = ctypes.c_size_t(), ctypes.c_size_t()
    _check(lib().rsmi_partition(nblocks, parts, i, ctypes.byref(st), ctypes.byref(cnt)))
    return st.value, cnt.value


def key_slot(key: bytes) -> int:
    """keyHashSlot (dag/pool/poolservice/hash_slot.go:20-22) in the library."""
    b = bytearray(key)
    return lib().rsmi_key_slot(ctypes.addressof(_buf(b)) if b else None, len(b))


def check_shards(lens: Sequence[int], nil_ok: bool):
    arr = (ctypes.c_size_t * len(lens))(*lens)
    S = ctypes.c_size_t()
    rc = lib().rsmi_check_shards(len(lens), arr, 1 if nil_ok else 0, ctypes.byref(S))
    return rc, S.value


class Erasure:
    """dag/node/dagnode/erasure.go:9-13 Erasure{encoder, dataBlocks, parityBlocks, blockSize}."""

    def __init__(self, data_blocks: int, parity_blocks: int, block_size: int, device: int = 0):
        # erasure.go:18-24
        if data_blocks <= 0 or parity_blocks <= 0:
            raise RsmiError(ErrInvShardNum)
        if data_blocks + parity_blocks > 256:
            raise RsmiError(ErrMaxShardNum)
        self.data_blocks = data_blocks
        self.parity_blocks = parity_blocks
        self.block_size = block_size
        self._device = device
        self._codec: Optional[Codec] = None

    def encoder(self) -> Codec:
        """erasure.go:31-45: the codec is built lazily, once."""
        if self._codec is None:
            self._codec = Codec(self.data_blocks, self.parity_blocks, self._device)
        return self._codec

    def shard_size(self) -> int:
        """erasure.go:96-98"""
        return ceil_frac(self.block_size, self.data_blocks)

    def encode_data(self, data: bytes) -> List[Optional[bytes]]:
        """erasure.go:51-65 EncodeData: Split + Encode."""
        n = self.data_blocks + self.parity_blocks
        if len(data) == 0:
            return [None] * n
        flat = self.encoder().encode_block(data)
        S = len(flat) // n
        return [flat[i * S:(i + 1) * S] for i in range(n)]

    def _reconstruct(self, shards: List[Optional[bytes]], data_only: bool) -> None:
        n = self.data_blocks + self.parity_blocks
        if len(shards) != n:
            raise RsmiError(ErrTooFewShards)  # upstream: len(shards) != totalShards
        lens = [len(s) if s else 0 for s in shards]
        rc, S = check_shards(lens, nil_ok=True)
        _check(rc)
        present = [bool(x) for x in lens]
        np_ = sum(present)
        dp = sum(present[: self.data_blocks])
        if np_ == n or (data_only and dp == self.data_blocks):
            return
        flat = bytearray(n * S)
        for i, s in enumerate(shards):
            if s:
                flat[i * S:(i + 1) * S] = s
        self.encoder().reconstruct(flat, S, present, data_only)
        for i in range(n):
            if not present[i] and (i < self.data_blocks or not data_only):
                shards[i] = bytes(flat[i * S:(i + 1) * S])

    def decode_data_blocks(self, data: List[Optional[bytes]]) -> None:
        """erasure.go:70-83 DecodeDataBlocks (the isZero loop breaks after the first empty
        shard, so only 'nothing missing' short-circuits; then ReconstructData)."""
        is_zero = 0
        for b in data:
            if not b:
                is_zero += 1
                break
        if is_zero == 0 or is_zero == len(data):
            return
        self._reconstruct(data, data_only=True)

    def decode_data_and_parity_blocks(self, data: List[Optional[bytes]]) -> None:
        """erasure.go:87-93 DecodeDataAndParityBlocks -> Reconstruct."""
        self._reconstruct(data, data_only=False)


def NewErasure(data_blocks: int, parity_blocks: int, block_size: int, device: int = 0) -> Erasure:
    return Erasure(data_blocks, parity_blocks, block_size, device)


def crc16_ibm(data: bytes) -> int:
    """howeyc/crc16 Checksum(data, IBMTable) (dag/node/datanode/server.go:70), host side."""
    b = bytearray(data)
    return lib().rsmi_crc16_ibm(ctypes.addressof(_buf(b)) if b else None, len(b))


def crc16_entry(head: bytes, raw: int, data_len: int) -> int:
    """Checksum(head || D) from R(D) = raw and |D| (include/rsmi.h rsmi_crc16_entry)."""
    h = bytearray(head)
    return lib().rsmi_crc16_entry(ctypes.addressof(_buf(h)) if h else None, len(h), raw, data_len)


def crc32_ieee(data: bytes) -> int:
    """Go crc32.ChecksumIEEE(data) (the mutcask value checksum, kv/mutcask/cask.go:75), host side."""
    b = bytearray(data)
    return lib().rsmi_crc32_ieee(ctypes.addressof(_buf(b)) if b else None, len(b))


def crc32_entry(head: bytes, raw: int, data_len: int) -> int:
    """ChecksumIEEE(head || D) from R32(D) = raw and |D| (include/rsmi.h rsmi_crc32_entry)."""
    h = bytearray(head)
    return lib().rsmi_crc32_entry(ctypes.addressof(_buf(h)) if h else None, len(h), raw, data_len)


def recommended_pitch(S: int) -> int:
    return lib().rsmi_recommended_pitch(S)


def device_count() -> int:
    return lib().rsmi_device_count()
