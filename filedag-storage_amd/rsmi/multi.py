"""Block partitioning across GPUs (one process per GPU, no collective on the data path).

Every block is coded independently (dag/node/dagnode/node.go:358-408), so a batch splits
into per-rank ranges; SURVEY.md 8(e).  Two mappings:
  * partition_blocks: contiguous, balanced ranges (bench.py's weak-scaling layout);
  * key_gpu: a stable key -> GPU map built on the reference's own routing hash,
    keyHashSlot = crc16(key) & 0x3FFF over 16384 slots (dag/pool/poolservice/hash_slot.go:20-22),
    then slot -> GPU by contiguous slot ranges.
"""
from typing import Tuple

CLUSTER_SLOTS = 16384  # dag/slotsmgr/slots_mgr.go:8


def partition_blocks(nblocks: int, world: int, rank: int) -> Tuple[int, int]:
    """(start, count) of rank's contiguous share; shares differ by at most one block."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(nblocks, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def _crc16_table():
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ 0xA001 if c & 1 else c >> 1
        t.append(c)
    return t


_T = _crc16_table()


def crc16_ibm(data: bytes) -> int:
    """howeyc/crc16 Checksum(data, IBMTable) as restated in SURVEY.md 8(a) a10: reflected
    polynomial 0xA001, init 0xFFFF, final xor 0xFFFF (CRC-16/USB; check("123456789") =
    0xB4C8).  The upstream source is not in the container: this variant is unpinned."""
    crc = 0xFFFF
    for b in data:
        crc = _T[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFF


def key_hash_slot(key: str) -> int:
    return crc16_ibm(key.encode()) & 0x3FFF


def key_gpu(key: str, world: int) -> int:
    """Slot ranges of equal size per GPU, like DagNodes owning contiguous SlotPairs."""
    return key_hash_slot(key) * world // CLUSTER_SLOTS
