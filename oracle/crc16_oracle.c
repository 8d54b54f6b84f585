/* crc16_oracle.c -- TEST INFRASTRUCTURE ONLY (tests/, bench.py's cpu_baseline leg).
 *
 * Byte-serial CPU restatement of the datanode entry checksum:
 *   dag/node/datanode/server.go:58-75  Put: entry = |crc (4 LE)|meta size (4 LE)|data size (4 LE)|meta|data|,
 *                                      crc = uint32(crc16.Checksum(entry[4:], crc16.IBMTable))
 *   dag/node/datanode/server.go:93-97  Get re-checks the same sum.
 * The checksum comes from github.com/howeyc/crc16 @ 2b2a61e366a6 (go.mod), absent from
 * /root/reference and from this image.  Restated from its published source:
 *   IBM = 0xA001; makeTable(poly): for i in 0..255 { crc = i; 8x: crc = crc&1 ? (crc>>1)^poly : crc>>1 }
 *   Checksum(data, tab) = Update(0, tab, data); for a non-reversed, XOR-ing table
 *   update(): crc = ^crc; per byte crc = tab[byte(crc)^v] ^ (crc >> 8); return ^crc
 * i.e. CRC-16/USB (check("123456789") = 0xB4C8).  No reference test pins a value, so this
 * variant is "parity unpinned" (DESIGN.md section 2).  Never linked into the product. */
#include <stdlib.h>
#include <string.h>

#include "rs_oracle.h"

static uint16_t ibm_table[256];
static int ibm_ready;

static void make_table(void) {
    for (int i = 0; i < 256; i++) {
        uint16_t crc = (uint16_t)i;
        for (int j = 0; j < 8; j++) crc = (crc & 1) ? (uint16_t)((crc >> 1) ^ 0xA001) : (uint16_t)(crc >> 1);
        ibm_table[i] = crc;
    }
    ibm_ready = 1;
}

uint16_t rs_oracle_crc16_ibm(const uint8_t* p, size_t n) {
    if (!ibm_ready) make_table();
    uint16_t crc = 0xFFFF; /* crc = ^crc with crc = 0 */
    for (size_t i = 0; i < n; i++) crc = (uint16_t)(ibm_table[(uint8_t)(crc ^ p[i])] ^ (crc >> 8));
    return (uint16_t)~crc;
}

static void put_le32(uint8_t* p, uint32_t v) {
    for (int i = 0; i < 4; i++) p[i] = (uint8_t)(v >> (8 * i));
}

/* server.go:58-75: the Header{Checksum, MetaSize, DataSize} is written little-endian, then
 * meta, then data; the checksum covers everything after its own 4 bytes. */
uint32_t rs_oracle_datanode_entry_crc(const uint8_t* meta, size_t meta_len, const uint8_t* data, size_t data_len) {
    const size_t n = 12 + meta_len + data_len;
    uint8_t* e = (uint8_t*)calloc(n, 1);
    if (!e) return 0xFFFFFFFFu;
    put_le32(e + 4, (uint32_t)meta_len);
    put_le32(e + 8, (uint32_t)data_len);
    if (meta_len) memcpy(e + 12, meta, meta_len);
    if (data_len) memcpy(e + 12 + meta_len, data, data_len);
    const uint32_t crc = rs_oracle_crc16_ibm(e + 4, n - 4);
    free(e);
    return crc;
}
