/* rs_oracle.h -- TEST INFRASTRUCTURE ONLY.  CPU restatement of klauspost/reedsolomon
 * v1.11.0 as used by dag/node/dagnode/erasure.go (see rs_oracle.c header).  Never linked
 * into the product library. */
#ifndef RS_ORACLE_H
#define RS_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* error codes: numbering matches include/rsmi.h so tests can compare directly */
enum {
    RS_ORACLE_OK = 0,
    RS_ORACLE_ERR_SHORT_DATA = 1,     /* reedsolomon.ErrShortData   */
    RS_ORACLE_ERR_TOO_FEW_SHARDS = 2, /* reedsolomon.ErrTooFewShards */
    RS_ORACLE_ERR_SHARD_NO_DATA = 3,  /* reedsolomon.ErrShardNoData  */
    RS_ORACLE_ERR_SHARD_SIZE = 4,     /* reedsolomon.ErrShardSize    */
    RS_ORACLE_ERR_INV_SHARD_NUM = 5,  /* reedsolomon.ErrInvShardNum  */
    RS_ORACLE_ERR_MAX_SHARD_NUM = 6,  /* reedsolomon.ErrMaxShardNum  */
    RS_ORACLE_ERR_SINGULAR = 7,       /* reedsolomon errSingular     */
    RS_ORACLE_ERR_INVALID = 8
};

uint8_t rs_oracle_gal_mul(uint8_t a, uint8_t b);
uint8_t rs_oracle_gal_exp(uint8_t a, int n);
int rs_oracle_invert(const uint8_t* in, uint8_t* out, int size);
int rs_oracle_build_matrix(int k, int m, uint8_t* out);
size_t rs_oracle_shard_size(size_t block_size, int k);
int rs_oracle_split(int k, int m, const uint8_t* block, size_t B, uint8_t* shards);
int rs_oracle_encode(int k, int m, uint8_t* shards, size_t S);
int rs_oracle_reconstruct(int k, int m, uint8_t* shards, size_t S, const uint8_t* present, int data_only);
int rs_oracle_check_shards(int n, const size_t* lens, int nil_ok, size_t* S_out);
int rs_oracle_selftest(void);

/* datanode entry checksum (crc16_oracle.c): howeyc/crc16 Checksum(p, IBMTable), and the
 * checksum server.go:70 stores for an entry holding meta and data */
uint16_t rs_oracle_crc16_ibm(const uint8_t* p, size_t n);
uint32_t rs_oracle_datanode_entry_crc(const uint8_t* meta, size_t meta_len, const uint8_t* data, size_t data_len);

/* mutcask value checksum (crc32_oracle.c): Go crc32.ChecksumIEEE(p), and the checksum
 * kv/mutcask/cask.go:73-79 stores for a datanode entry (entry_crc16 = its server.go:70 sum) */
uint32_t rs_oracle_crc32_ieee(const uint8_t* p, size_t n);
uint32_t rs_oracle_mutcask_entry_crc(uint32_t entry_crc16, const uint8_t* meta, size_t meta_len, const uint8_t* data,
                                     size_t data_len);

/* fast multi-threaded CPU path (rs_cpu_fast.c): same results, used only as bench.py's
 * cpu_baseline and cross-checked against the scalar path in tests */
int rs_cpu_encode_batch(int k, int m, const uint8_t* data, size_t data_block_stride,
                        uint8_t* parity, size_t parity_block_stride, size_t S, size_t nblocks,
                        int threads);
int rs_cpu_reconstruct_batch(int k, int m, uint8_t* shards, size_t block_stride, size_t S,
                             size_t nblocks, const uint8_t* present, int data_only, int threads);
const char* rs_cpu_isa(void);

#ifdef __cplusplus
}
#endif
#endif
