/*
 * rsmi.h -- C-ABI of the MI355X Reed-Solomon engine (librsmi.so).
 *
 * This is the drop-in seam under filedag-storage's Dag Node: every entry point replaces
 * one call that dag/node/dagnode makes into github.com/klauspost/reedsolomon v1.11.0
 * (go.mod:31).  Plain pointers and sizes only -- no Go, torch or HIP types -- so a cgo
 * file binds it directly.  All functions are thread-safe; one context
 * may be shared by every goroutine of a DagNode (node.go:358 Put, :220 Get, the repair
 * worker at :159 and data_recovery.go:16 RepairDataNode all run concurrently).
 *
 * Buffer ownership: the caller owns every buffer; the library never retains a caller
 * pointer after a call returns (cgo pointer rules).  The *_dev entry points take device
 * pointers and a hipStream_t passed as void*; they are stream-ordered and do not sync.
 *
 * Status codes map 1:1 onto the upstream sentinels (erasure.go:19,23 return two of them
 * directly; the rest surface through Split/Encode/Reconstruct at erasure.go:55,60,82,88).
 * There is no CPU fallback: a device failure is RSMI_ERR_DEVICE / RSMI_ERR_NO_DEVICE.
 */
#ifndef RSMI_H
#define RSMI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: rsmi_set_option lost the keys of kernel variants measured slower than the defaults (they
 * return RSMI_ERR_INVALID_ARG); device groups, NUMA placement, the key slot hash and
 * rsmi_reconstruct_batch_host_verify were added; "crc16_fused_fold" is new.
 * 3: no C++ exception crosses the boundary: every status-returning entry point that can allocate
 * on the host returns RSMI_ERR_HOST instead (new status).
 * 4: coalesced calls run on up to "coalesce_lanes" batches at once (new option, default 2);
 * rsmi_warm is new; the device-resident CRC entry points may run concurrently on different streams
 * of one context; rsmi_last_kernel returns a per-thread copy.
 * 5: the per-thread wait hook (rsmi_set_wait_hook, rsmi_run_wait_hook). */
#define RSMI_ABI_VERSION 5

typedef struct rsmi_ctx rsmi_ctx;

enum rsmi_status {
    RSMI_OK = 0,
    RSMI_ERR_SHORT_DATA = 1,     /* reedsolomon.ErrShortData    (Split of 0 bytes)          */
    RSMI_ERR_TOO_FEW_SHARDS = 2, /* reedsolomon.ErrTooFewShards (< k shards present)        */
    RSMI_ERR_SHARD_NO_DATA = 3,  /* reedsolomon.ErrShardNoData  (every shard empty)         */
    RSMI_ERR_SHARD_SIZE = 4,     /* reedsolomon.ErrShardSize    (unequal non-empty shards)  */
    RSMI_ERR_INV_SHARD_NUM = 5,  /* reedsolomon.ErrInvShardNum  (k<=0 || m<=0), erasure.go:19 */
    RSMI_ERR_MAX_SHARD_NUM = 6,  /* reedsolomon.ErrMaxShardNum  (k+m>256),     erasure.go:23 */
    RSMI_ERR_SINGULAR = 7,       /* matrix not invertible (cannot happen for valid patterns) */
    RSMI_ERR_INVALID_ARG = 8,    /* NULL pointer, stride smaller than a shard, ...          */
    RSMI_ERR_DEVICE = 100,       /* a HIP call failed                                       */
    RSMI_ERR_NO_DEVICE = 101,    /* no usable gfx950 device / kernels not loadable          */
    RSMI_ERR_HOST = 102          /* host resources exhausted (memory, threads): a C++
                                  * exception caught at the boundary, never propagated     */
};

/* ------------------------------------------------------------------ lifecycle */

/* Replaces reedsolomon.New(k, m, WithAutoGoroutines(S)) inside NewErasure
 * (dag/node/dagnode/erasure.go:16-47).  Validates like erasure.go:18-24, builds and caches
 * the n x k systematic matrix.  Device resources are created lazily on first compute call,
 * so opening a context works (and reports argument errors) on a host without a GPU. */
int rsmi_open(int k, int m, int device, rsmi_ctx** out);
void rsmi_close(rsmi_ctx* ctx);

/* Bring up the context's device resources before the first real call (a Dag Node does this when
 * it starts): streams, the encode plan, the CRC tables and every coalescing lane (one tiny fused
 * encode + CRC-16 each), so the first concurrent callers do not pay for them. */
int rsmi_warm(rsmi_ctx* ctx);

int rsmi_device_count(void);
const char* rsmi_status_string(int status);
int rsmi_abi_version(void);

/* ------------------------------------------------------------------ host-only helpers */

/* Erasure.ShardSize (erasure.go:96-98) = ceilFrac(B, k) (utils.go:6-21). */
size_t rsmi_shard_size(size_t block_size, int k);

/* Device row pitch for shards of S bytes that the fast kernels stream best on MI355X:
 * the next power of two for shards up to 64 KiB (when it wastes at most half a shard) and
 * for exact powers of two, 11/8 S in 4 KiB granules for 96 KiB < S < 128 KiB (1 MiB RS(10,4)
 * blocks), otherwise S rounded up to 4 KiB (measured, DESIGN.md "Layout").  The
 * host-staged entry points use it internally. */
size_t rsmi_recommended_pitch(size_t S);

/* The cached (k+m) x k encode matrix, row-major. */
int rsmi_encode_matrix(const rsmi_ctx* ctx, uint8_t* out);

/* Upstream checkShards/shardSize: lens[i]==0 marks shard i missing.  nil_ok=0 is the
 * Encode check, nil_ok=1 the Reconstruct check.  *S_out receives the common size. */
int rsmi_check_shards(int n, const size_t* lens, int nil_ok, size_t* S_out);

/* The k x k data-decode matrix the reconstruct path uses for this erasure pattern
 * (inverse of the rows of the first k present shards, upstream reconstruct()); the k
 * survivor indices are written to used_rows.  present: n flags. */
int rsmi_decode_matrix(const rsmi_ctx* ctx, const uint8_t* present, uint8_t* out, int* used_rows);

/* ------------------------------------------------------------------ one block, host memory */

/* Erasure.EncodeData (erasure.go:51-65): Split + Encode of one raw block of B bytes into
 * (k+m)*S contiguous bytes, S = rsmi_shard_size(B, k); data rows zero-padded like Split.
 * B == 0 -> RSMI_ERR_SHORT_DATA (the Go wrapper short-circuits it before calling). */
int rsmi_encode_block(rsmi_ctx* ctx, const uint8_t* block, size_t B, uint8_t* shards_out);

/* Encoder.Encode on pre-split shards: data = k*S contiguous, parity = m*S contiguous. */
int rsmi_encode(rsmi_ctx* ctx, const uint8_t* data, uint8_t* parity, size_t S);

/* Encoder.ReconstructData (data_only=1, erasure.go:82) / Encoder.Reconstruct (data_only=0,
 * erasure.go:88) on n*S contiguous bytes.  present: n flags; missing rows are overwritten,
 * present rows are only read.  Nothing missing -> RSMI_OK without touching the device. */
int rsmi_reconstruct(rsmi_ctx* ctx, uint8_t* shards, size_t S, const uint8_t* present, int data_only);

/* ------------------------------------------------------------------ batches, host memory */

/* nblocks independent blocks: data block b at data + b*data_block_stride (k rows of S
 * bytes), parity block b at parity + b*parity_block_stride (m rows of S bytes).
 * Copies are overlapped with compute over several HIP streams; pass memory from
 * rsmi_host_alloc for full PCIe rate. */
int rsmi_encode_batch_host(rsmi_ctx* ctx, const uint8_t* data, size_t data_block_stride, uint8_t* parity,
                           size_t parity_block_stride, size_t S, size_t nblocks);

/* One erasure pattern for every block (RepairDataNode shape, data_recovery.go:16-112):
 * block b at shards + b*block_stride holds n rows of S bytes. */
int rsmi_reconstruct_batch_host(rsmi_ctx* ctx, uint8_t* shards, size_t block_stride, size_t S, size_t nblocks,
                                const uint8_t* present, int data_only);

/* Rebuild only the rows flagged in required[] (n flags; rows that are present are left
 * alone) -- RepairDataNode needs one row per key (data_recovery.go:88,102-106), not every
 * missing one.  Same layout and errors as rsmi_reconstruct_batch_host. */
int rsmi_reconstruct_rows_batch_host(rsmi_ctx* ctx, uint8_t* shards, size_t block_stride, size_t S, size_t nblocks,
                                     const uint8_t* present, const uint8_t* required);

/* Page-locked host memory: portable (mapped for every device, so device-group members read and
 * write one buffer in place) and placed by the calling thread's NUMA memory policy. */
void* rsmi_host_alloc(size_t bytes);
void rsmi_host_free(void* p);

/* ------------------------------------------------------------------ batches, device memory */

/* Device-resident encode.  Row c of data block b is at
 *   d_data + b*data_block_stride + c*data_shard_stride
 * and parity row j at d_parity + b*parity_block_stride + j*parity_shard_stride.
 * Fast path: every base/stride a multiple of 16 and each shard stride >= S rounded up to
 * 16 (the rows' padding bytes may be read, are never written).  Any other layout runs a
 * byte-granular kernel.  stream: hipStream_t (NULL = default stream). */
int rsmi_encode_batch_dev(rsmi_ctx* ctx, const uint8_t* d_data, size_t data_shard_stride,
                          size_t data_block_stride, uint8_t* d_parity, size_t parity_shard_stride,
                          size_t parity_block_stride, size_t S, size_t nblocks, void* stream);

/* Device-resident in-place reconstruct, one erasure pattern for all blocks.  Row i of
 * block b at d_shards + b*block_stride + i*shard_stride. */
int rsmi_reconstruct_batch_dev(rsmi_ctx* ctx, uint8_t* d_shards, size_t shard_stride, size_t block_stride,
                               size_t S, size_t nblocks, const uint8_t* present, int data_only, void* stream);

/* Device-resident form of rsmi_reconstruct_rows_batch_host. */
int rsmi_reconstruct_rows_batch_dev(rsmi_ctx* ctx, uint8_t* d_shards, size_t shard_stride, size_t block_stride,
                                    size_t S, size_t nblocks, const uint8_t* present, const uint8_t* required,
                                    void* stream);

/* Erasure.EncodeData for one block (same output as rsmi_encode_block, plus R(shard) in
 * raw_out[0..k+m) when raw_out is not NULL), coalesced with concurrent callers on the same
 * context: DagNode.Put runs once per block from many goroutines (node.go:358-408), and
 * group commit turns those calls into GPU batches.  A caller whose block is still queued and
 * that finds one of the context's "coalesce_lanes" lanes free (default 2) executes every block
 * queued so far (waiting up to option "coalesce_us" for more, default 0; at most
 * "coalesce_max" blocks, default 256) and wakes the others; blocks arriving while every lane
 * codes a batch form the next one.  Lane i > 0 codes on a child context of its own (streams and
 * scratch), so one batch is launched while the one before it runs.  A batch whose blocks lie in
 * page-locked memory (rsmi_host_alloc) is coded in place, up to 64 blocks per launch.  A lone
 * caller never waits on anyone.  block may be
 * shards_out itself: the caller has already copied the block to the start of shards_out
 * (Split's copy, done on the caller's own thread), and the engine zero-pads and encodes it in
 * place; any other overlap of block and shards_out is not allowed. */
int rsmi_encode_block_coalesced(rsmi_ctx* ctx, const uint8_t* block, size_t B, uint8_t* shards_out,
                                uint32_t* raw_out);

/* rsmi_encode_block_coalesced with the mutcask CRC-32 as well: raw32_out[0..k+m) = R32(shard)
 * when not NULL (see "mutcask CRC-32" below); raw16_out as raw_out above. */
int rsmi_encode_block_coalesced_crcs(rsmi_ctx* ctx, const uint8_t* block, size_t B, uint8_t* shards_out,
                                     uint32_t* raw16_out, uint32_t* raw32_out);

/* rsmi_reconstruct (same arguments, results and errors), coalesced the same way.  When a
 * datanode is down every concurrent DagNode.Get misses the same shard (node.go:277-282), so
 * concurrent degraded reads share one erasure pattern and batch into one launch; requests
 * with different shard sizes or patterns run as separate groups of the same batch. */
int rsmi_reconstruct_coalesced(rsmi_ctx* ctx, uint8_t* shards, size_t S, const uint8_t* present, int data_only);

/* Counters: "coalesced_calls", "coalesced_batches" (both coalesced entry points); diagnostic:
 * "coalesced_wakes", the wake-ups of callers that slept, and "coalesced_wake_ns", the summed time
 * from each wake-up call to the caller running again.  -1 for an unknown key. */
long rsmi_get_stat(const rsmi_ctx* ctx, const char* key);

/* A host task for the calling thread to run while its next codec call's device work is in
 * flight.  DagNode.Put (node.go:376-399) encodes and then writes every shard; the data shards
 * that hold only block bytes are final once Split, so the host mirror writes them to their
 * datanodes while the GPU encodes the parity, on the calling thread, without a hand-off.  The
 * hook is per thread and one-shot: the next rsmi_encode_block_coalesced(_crcs),
 * rsmi_reconstruct_coalesced, or one-block host call of rsmi_encode_batch_host(_crcs),
 * rsmi_reconstruct_batch_host or rsmi_reconstruct_rows_batch_host(_crcs) that runs as one
 * in-place kernel (page-locked rows, or a small call) on this thread
 * takes it and runs fn(arg) once on this thread -- after its device work is launched and before
 * it waits for it, or, when the call has no work of its own in flight at that point (a caller whose
 * block another thread's batch codes), before it blocks.  A call may hold the context's lock while
 * fn runs, so fn must make no codec call (host-only helpers such as the CRC folds are fine) and
 * must not throw.  Other entry points, calls that take the copy-engine pipeline and calls that
 * fail before launching leave the hook pending.  fn == NULL clears it.  A lone DagNode.Get uses it
 * too: it copies the block's present data rows while the GPU rebuilds the missing ones. */
void rsmi_set_wait_hook(void (*fn)(void*), void* arg);

/* Run the calling thread's hook if it is still pending (no call took it) and clear it: 1 if it
 * ran, 0 if there was none.  Setting a hook, making the call and then calling this runs the
 * task exactly once whatever path the call took. */
int rsmi_run_wait_hook(void);

/* ------------------------------------------------------------------ datanode CRC-16 */

/* The datanode stores every shard as |crc (4 LE)|meta size|data size|meta|data| with
 * crc = howeyc/crc16 Checksum(entry[4:], IBMTable) (dag/node/datanode/server.go:58-75),
 * and re-checks it on Get / GetMeta (server.go:93-97, :115-119).  These entry points move
 * the byte-serial CRC over the shard bytes onto the GPU; the host
 * only folds in the 12-byte header.  "Raw" CRC R(D) = the CRC-16 register after D from a
 * zero register, no complement (reflected polynomial 0xA001), held in a uint32. */

/* howeyc Checksum(p, IBMTable) on the host (carry-less-multiply folding from 256 bytes where the
 * CPU has VPCLMULQDQ, ~30 GiB/s per core; slice-by-8 otherwise).  Replaces the datanode's
 * crc16.Checksum(entry[4:], IBMTable) (dag/node/datanode/server.go:70, :93-97). */
uint16_t rsmi_crc16_ibm(const uint8_t* p, size_t n);

/* Checksum(head || D) from R(D) and |D|: with head = |meta size (4 LE)|data size (4 LE)|meta|
 * this is the entry checksum server.go:70 computes for a shard D.  head may be empty. */
uint16_t rsmi_crc16_entry(const uint8_t* head, size_t head_len, uint32_t raw, size_t data_len);

/* R(row) for nrows rows of S bytes per block on the device: row r of block b at
 * d_rows + b*block_stride + r*shard_stride; d_raw_out[b*out_block_stride + r] is zeroed and
 * then receives R(row).  Any alignment (16-byte aligned rows take the fast path).
 * Stream-ordered. */
int rsmi_crc16_rows_dev(rsmi_ctx* ctx, const uint8_t* d_rows, size_t shard_stride, size_t block_stride, int nrows,
                        size_t S, size_t nblocks, uint32_t* d_raw_out, size_t out_block_stride, void* stream);

/* rsmi_encode_batch_host plus R(shard) of every shard it touched, computed on the GPU from
 * the rows already resident there: raw_out[b*(k+m) + r] for data rows r < k and parity rows
 * k <= r < k+m.  DagNode.Put / PutMany hand these to the datanodes, which then store the
 * entry without a host CRC pass. */
int rsmi_encode_batch_host_crc(rsmi_ctx* ctx, const uint8_t* data, size_t data_block_stride, uint8_t* parity,
                               size_t parity_block_stride, size_t S, size_t nblocks, uint32_t* raw_out);

/* rsmi_encode_batch_dev with the CRC fused into the encode pass: every row the kernel reads
 * or writes is folded into per-chunk CRC-16 values on the way, and a combine pass writes
 * d_raw_out[b*(k+m) + r] = R(shard r of block b) (device memory).  The SURVEY.md 8(f) rank 2
 * form: no second pass over the shard bytes.  Stream-ordered. */
int rsmi_encode_batch_dev_crc(rsmi_ctx* ctx, const uint8_t* d_data, size_t data_shard_stride,
                              size_t data_block_stride, uint8_t* d_parity, size_t parity_shard_stride,
                              size_t parity_block_stride, size_t S, size_t nblocks, uint32_t* d_raw_out,
                              void* stream);

/* rsmi_encode_block plus raw_out[r] = R(shard r), r < k+m. */
int rsmi_encode_block_crc(rsmi_ctx* ctx, const uint8_t* block, size_t B, uint8_t* shards_out, uint32_t* raw_out);

/* R(row) (raw16_out) and/or R32(row) (raw32_out, mutcask CRC-32) of nrows host rows of S bytes,
 * row r at rows + r*row_stride; page-locked rows (rsmi_host_alloc) are read in place over
 * PCIe.  The Dag Node's GPU-verified reads check fetched shards against the checksums the
 * datanodes stored (server.go:93-97 moved to the reader); either output may be NULL. */
int rsmi_crc_rows_host(rsmi_ctx* ctx, const uint8_t* rows, size_t row_stride, size_t nrows, size_t S,
                       uint32_t* raw16_out, uint32_t* raw32_out);

/* ------------------------------------------------------------------ mutcask CRC-32 */

/* The mutcask KV engine under a datanode (kv/mutcask/cask.go:73-97, selected by
 * server.go:207) stores every value as |crc32 (4 LE)|value| with crc32 = Go
 * crc32.ChecksumIEEE(value) (the zlib CRC-32), and re-checks it on every read (cask.go:250).
 * The value is the datanode's whole entry, so the shard bytes get a second byte-serial pass
 * on every Put and Get.  "Raw" R32(D) = the CRC-32 register after D from a zero register,
 * no complement (reflected polynomial 0xEDB88320). */

/* crc32.ChecksumIEEE(p) on the host (the same folding).  Replaces the mutcask engine's
 * crc32.ChecksumIEEE (kv/mutcask/cask.go:73-79, :250). */
uint32_t rsmi_crc32_ieee(const uint8_t* p, size_t n);

/* ChecksumIEEE(head || D) from R32(D) and |D|: with head = the datanode entry's first 12 + meta
 * bytes (|crc16 (4 LE)|meta size|data size|meta|) this is the mutcask value checksum of a
 * shard D's entry.  head may be empty. */
uint32_t rsmi_crc32_entry(const uint8_t* head, size_t head_len, uint32_t raw, size_t data_len);

/* R32(row) for nrows rows of S bytes per block on the device, laid out as in
 * rsmi_crc16_rows_dev (d_raw_out[b*out_block_stride + r], zeroed first).  Stream-ordered. */
int rsmi_crc32_rows_dev(rsmi_ctx* ctx, const uint8_t* d_rows, size_t shard_stride, size_t block_stride, int nrows,
                        size_t S, size_t nblocks, uint32_t* d_raw_out, size_t out_block_stride, void* stream);

/* rsmi_encode_batch_host with either or both raw checksums of every shard it touched:
 * raw16_out[b*(k+m) + r] = R(shard) (CRC-16, as rsmi_encode_batch_host_crc) and
 * raw32_out[b*(k+m) + r] = R32(shard) (CRC-32), each optional (NULL).  The CRC-32 pass reads
 * the rows where the encode left them (device staging, or page-locked host memory on the
 * zero-copy path).  DagNode.PutMany hands both to mutcask-backed datanodes. */
int rsmi_encode_batch_host_crcs(rsmi_ctx* ctx, const uint8_t* data, size_t data_block_stride, uint8_t* parity,
                                size_t parity_block_stride, size_t S, size_t nblocks, uint32_t* raw16_out,
                                uint32_t* raw32_out);

/* rsmi_reconstruct_batch_host (same arguments, results and errors) that also returns R(row), the
 * datanode CRC-16 of the entry's shard bytes, of the k survivor rows it read: raw16_in[b*k + c] =
 * R(shard used[c]), used = the first k present shards (rsmi_decode_matrix's used_rows).  A
 * reader that fetched shards unchecked (the datanodes' stored checksums, server.go:93-97) checks
 * them for free on a degraded read: with page-locked shards one kernel reads each survivor once
 * for both; otherwise a CRC pass over the survivors follows the rebuild. */
int rsmi_reconstruct_batch_host_verify(rsmi_ctx* ctx, uint8_t* shards, size_t block_stride, size_t S, size_t nblocks,
                                       const uint8_t* present, int data_only, uint32_t* raw16_in);

/* rsmi_reconstruct_rows_batch_host plus the raw checksums of every row it rebuilt, from the
 * GPU where the rows land: raw16_out / raw32_out[b*(k+m) + r] = R(row) / R32(row) for rows r
 * that are required and missing, 0 for the others; either may be NULL.  RepairDataNode's
 * Puts of the rebuilt rows (data_recovery.go:102-106) then carry sender checksums like
 * DagNode.Put's. */
int rsmi_reconstruct_rows_batch_host_crcs(rsmi_ctx* ctx, uint8_t* shards, size_t block_stride, size_t S,
                                          size_t nblocks, const uint8_t* present, const uint8_t* required,
                                          uint32_t* raw16_out, uint32_t* raw32_out);

/* ------------------------------------------------------------------ device groups (several GPUs, one process) */

/* The Dag Pool runs every DagNode of a cluster in one process (dag/pool/poolservice/cluster.go:
 * 28-41).  A device group is one context per entry of devices[] (an entry may repeat: two
 * contexts on one GPU overlap their copies and kernels).  Its batch calls split the blocks
 * into contiguous ranges, one per member, sizes differing by at most one block (rsmi_partition),
 * and run every range on its member's context from its own host thread -- no data crosses
 * devices, no collective runs -- then return the first failing member's status in member
 * order.  Same arguments, layouts, results and errors as the single-context calls (nblocks == 0
 * validates the arguments on member 0 and returns).  Each member's thread is persistent and
 * bound to its GPU's NUMA node (CPUs and preferred memory), so the page-locked staging its
 * context allocates sits on that socket; one batch call runs at a time per group. */
typedef struct rsmi_group rsmi_group;
int rsmi_group_open(int k, int m, const int* devices, int ndev, rsmi_group** out);
void rsmi_group_close(rsmi_group* group);
int rsmi_group_size(const rsmi_group* group);
/* Member i's context (owned by the group), for the single-context calls; NULL if out of range. */
rsmi_ctx* rsmi_group_context(rsmi_group* group, int i);
/* The range of blocks member i of parts codes: contiguous, sizes differ by at most one. */
int rsmi_partition(size_t nblocks, int parts, int i, size_t* start, size_t* count);
/* keyHashSlot (dag/pool/poolservice/hash_slot.go:20-22): howeyc crc16 IBM of the key & 0x3FFF. */
int rsmi_key_slot(const uint8_t* key, size_t len);
/* The member that owns a key: contiguous slot ranges of 16384 / size slots per member, as
 * DagNodes own SlotPairs -- a stable key -> GPU map for per-block callers. */
int rsmi_group_member_of_key(const rsmi_group* group, const uint8_t* key, size_t len);
/* Member i's NUMA node (rsmi_device_numa_node of its device), -1 if unknown. */
int rsmi_group_member_numa_node(const rsmi_group* group, int i);
/* Page-locked (portable, mapped) host memory for nblocks blocks of block_bytes whose member
 * ranges (rsmi_partition over the group's size) sit on the members' NUMA nodes, so on the
 * zero-copy path each member's DMA reads and writes only its own socket's memory.  Zeroed.
 * Freed by rsmi_group_host_free or rsmi_group_close.  NULL on failure. */
void* rsmi_group_host_alloc(rsmi_group* group, size_t block_bytes, size_t nblocks);
void rsmi_group_host_free(rsmi_group* group, void* p);
/* The host NUMA node closest to a device: hipDeviceAttributeHostNumaId, else sysfs
 * bus/pci/devices/<pci bus id>/numa_node; -1 when unknown. */
int rsmi_device_numa_node(int device);
/* Host-only helpers behind it, with the sysfs root injectable ("/sys" in production): the
 * numa_node of a PCI bus id ("0000:75:00.0", any case; -1 if absent), and a node's CPU list
 * (devices/system/node/node<N>/cpulist: returns the number of CPUs, writes at most max_cpus;
 * -1 if absent or malformed). */
int rsmi_sysfs_numa_node(const char* sysfs_root, const char* pci_bus_id);
int rsmi_sysfs_node_cpus(const char* sysfs_root, int node, int* cpus, int max_cpus);
/* Bind the calling thread to a NUMA node: the node's CPUs the process may use, and a
 * preferred-node memory policy (allocations fall back to other nodes, never fail). */
int rsmi_bind_thread_to_numa_node(int node);
int rsmi_group_encode_batch_host(rsmi_group* group, const uint8_t* data, size_t data_block_stride, uint8_t* parity,
                               size_t parity_block_stride, size_t S, size_t nblocks);
int rsmi_group_encode_batch_host_crcs(rsmi_group* group, const uint8_t* data, size_t data_block_stride, uint8_t* parity,
                                    size_t parity_block_stride, size_t S, size_t nblocks, uint32_t* raw16_out,
                                    uint32_t* raw32_out);
int rsmi_group_reconstruct_batch_host(rsmi_group* group, uint8_t* shards, size_t block_stride, size_t S, size_t nblocks,
                                    const uint8_t* present, int data_only);
int rsmi_group_reconstruct_rows_batch_host(rsmi_group* group, uint8_t* shards, size_t block_stride, size_t S,
                                         size_t nblocks, const uint8_t* present, const uint8_t* required);

/* ------------------------------------------------------------------ tuning / introspection */

/* Options: "waves_per_cu" (grid cap; 0 = the default geometry: one tile per wave for the
 * coding kernels, 48/96 waves per CU for the CRC rows passes), "zero_copy" (1 = default: host
 * batch calls whose buffers are page-locked (rsmi_host_alloc) run as one kernel that reads and
 * writes them in place over PCIe, at any size; 2 = the same, also reading inputs in place on
 * the pipeline path; 0 = always the copy-engine pipeline), "small_call_bytes" (host calls moving
 * at most this many shard bytes, default 2 MiB, run as one such kernel -- pageable buffers are
 * staged through a page-locked one by CPU copies; 0 = never), "coalesce_us" / "coalesce_max"
 * (rsmi_encode_block_coalesced), "crc16_fold" (the CRC-16 rows pass on 16-byte-aligned rows:
 * 1 = default, the fold on the matrix cores (fp4 MFMA); 0 = the nibble-table fold; both
 * bit-exact), "crc16_fused_fold" (the encode with the CRC-16 fused in, on
 * 16-byte-aligned layouts: 1 = default, rs_fused_mfma_kernel folds on the matrix cores; 0 = the
 * nibble-table variants), "crc32_fold" (the mutcask CRC-32 rows pass: 1 = the fold on the
 * matrix cores, 0 = the nibble-table fold; both bit-exact), "inject_host_fault" (test hook: the
 * next N coalesced batches, or direct rsmi_encode_batch_host* calls, throw std::bad_alloc, so their
 * requests return RSMI_ERR_HOST; default 0), "inject_lane_fault" (test hook: the next N coalescing lane contexts
 * fail to open, as a device error would; default 0), "coalesce_lanes" (coalesced batches coded at
 * once, 1-16, default 2; every option but the test hooks also applies to the lanes' child
 * contexts), "coalesce_carry"
 * (batches a lane's executor goes on to when they are queued by the time its own completes,
 * before it hands the lane to a waiting caller, 0-16, default 1), "coalesce_pipeline" (1 =
 * default: a coalesced batch coded by the table kernels is left in flight behind an event while
 * the lane's next queued batch is launched behind it, and its callers return when the event
 * completes; 0 = every batch synchronises before the next is launched), "coalesce_flag" (1 =
 * default: a coalesced group coded by one table launch of the encode + CRC-16, and a one-block
 * in-place host call (encode + CRC-16, reconstruct, verified reconstruct), signal their end through
 * a page-locked flag the launch's last workgroup releases, which the caller polls instead of
 * synchronising -- blocking in the synchronisation after 200 us; 0 = event / stream
 * synchronisation).  Kernel variants measured slower than the defaults are not
 * built into the library.  Returns RSMI_ERR_INVALID_ARG for unknown keys or
 * values. */
int rsmi_set_option(rsmi_ctx* ctx, const char* key, long value);
/* Name of the kernel the last device launch on this context used ("" if none); a copy owned by
 * the calling thread, valid until its next rsmi_last_kernel call. */
const char* rsmi_last_kernel(const rsmi_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* RSMI_H */
