/* crc32_oracle.c -- TEST INFRASTRUCTURE ONLY (tests/).
 *
 * Bit-serial CPU restatement of the mutcask value checksum:
 *   kv/mutcask/cask.go:73-79  EncodeValue: ret = |crc32 (4 LE)|v|, crc32 = crc32.ChecksumIEEE(v)
 *   kv/mutcask/cask.go:81-97  DecodeValue(buf, verify) re-checks it (cask.go:250: on every read)
 * crc32.ChecksumIEEE is Go's standard library: the reflected polynomial 0xEDB88320, register
 * complemented on entry and exit -- the same function as zlib's crc32, so the tests pin this
 * restatement against Python's zlib.crc32 and the check value 0xCBF43926 ("123456789").
 * The datanode hands mutcask its whole entry (server.go:58-75, 207), so a shard's value
 * checksum covers |crc16|meta size|data size|meta|data|.  Never linked into the product. */
#include <stdlib.h>
#include <string.h>

#include "rs_oracle.h"

uint32_t rs_oracle_crc32_ieee(const uint8_t* p, size_t n) {
    uint32_t crc = 0xFFFFFFFFu;
    for (size_t i = 0; i < n; i++) {
        crc ^= p[i];
        for (int b = 0; b < 8; b++) crc = (crc & 1) ? (crc >> 1) ^ 0xEDB88320u : crc >> 1;
    }
    return ~crc;
}

/* the mutcask value checksum of a datanode entry: ChecksumIEEE(|crc16 (4 LE)|meta size|data
 * size|meta|data|), with crc16 the entry's own datanode checksum (server.go:70) */
uint32_t rs_oracle_mutcask_entry_crc(uint32_t entry_crc16, const uint8_t* meta, size_t meta_len, const uint8_t* data,
                                     size_t data_len) {
    const size_t n = 12 + meta_len + data_len;
    uint8_t* e = (uint8_t*)calloc(n, 1);
    if (!e) return 0;
    for (int i = 0; i < 4; i++) {
        e[i] = (uint8_t)(entry_crc16 >> (8 * i));
        e[4 + i] = (uint8_t)((uint32_t)meta_len >> (8 * i));
        e[8 + i] = (uint8_t)((uint32_t)data_len >> (8 * i));
    }
    if (meta_len) memcpy(e + 12, meta, meta_len);
    if (data_len) memcpy(e + 12 + meta_len, data, data_len);
    const uint32_t crc = rs_oracle_crc32_ieee(e, n);
    free(e);
    return crc;
}
