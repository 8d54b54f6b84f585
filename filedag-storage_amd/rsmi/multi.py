"""Block partitioning across GPUs (one process per GPU, no collective on the data path).

Every block is coded independently (dag/node/dagnode/node.go:358-408), so a batch splits
into per-rank ranges; SURVEY.md 8(e).  Two mappings:
  * partition_blocks: contiguous, balanced ranges (bench.py's weak-scaling layout);
  * key_gpu: a stable key -> GPU map built on the reference's own routing hash,
    keyHashSlot = crc16(key) & 0x3FFF over 16384 slots (dag/pool/poolservice/hash_slot.go:20-22),
    then slot -> GPU by contiguous slot ranges.
"""
import os
from typing import Mapping, Optional, Tuple

CLUSTER_SLOTS = 16384  # dag/slotsmgr/slots_mgr.go:8
KFD_NODES = "class/kfd/kfd/topology/nodes"  # under the sysfs root


def sysfs_gpu_count(sysfs_root: str = "/sys") -> Optional[int]:
    """GPUs the kernel driver lists, read from sysfs without touching the HIP runtime: KFD
    topology nodes whose `properties` carry a non-zero gfx_target_version (CPU nodes carry 0).
    None when the topology is absent (no amdgpu driver, or sysfs not mounted)."""
    base = os.path.join(sysfs_root, KFD_NODES)
    try:
        nodes = os.listdir(base)
    except OSError:
        return None
    n = 0
    for d in nodes:
        try:
            with open(os.path.join(base, d, "properties")) as f:
                for line in f:
                    key, _, val = line.partition(" ")
                    if key == "gfx_target_version":
                        n += int(val.strip() or "0") != 0
                        break
        except (OSError, ValueError):
            continue
    return n


def _visible(spec: str, have: int, uuids: bool) -> int:
    """Devices a *_VISIBLE_DEVICES list leaves out of `have`: the runtime takes entries in
    order and stops at the first it cannot use (an index out of range, or garbage); ROCr also
    takes GPU UUIDs ("GPU-<hex>")."""
    n = 0
    for e in spec.split(","):
        e = e.strip()
        if uuids and e.startswith("GPU-"):
            n += 1
            continue
        if not e.isdigit() or int(e) >= have:
            break
        n += 1
    return min(n, have)


def visible_gpu_count(sysfs_root: str = "/sys", env: Optional[Mapping[str, str]] = None) -> Optional[int]:
    """GPUs a child process will see, counted without initialising HIP in this process (the
    launcher must stay GPU-free before it spawns one process per GPU: bench.py --gpus N).
    sysfs gives the physical count; ROCR_VISIBLE_DEVICES filters it first, then
    HIP_VISIBLE_DEVICES (or CUDA_VISIBLE_DEVICES) indexes the ROCr-visible list.  None when
    sysfs has no KFD topology."""
    env = os.environ if env is None else env
    have = sysfs_gpu_count(sysfs_root)
    if have is None:
        return None
    rocr = env.get("ROCR_VISIBLE_DEVICES")
    if rocr is not None:
        have = _visible(rocr, have, uuids=True)
    hip = env.get("HIP_VISIBLE_DEVICES", env.get("CUDA_VISIBLE_DEVICES"))
    if hip is not None:
        have = _visible(hip, have, uuids=False)
    return have


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
