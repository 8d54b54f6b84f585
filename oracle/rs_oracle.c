/*
 * rs_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * Plain-C CPU restatement of the Reed-Solomon codec that filedag-storage's Dag Node
 * uses for every block it stores.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this file's library; the product path
 * (filedag-storage_amd/csrc) never links or calls it.
 *
 * Where the algorithm lives: dag/node/dagnode/erasure.go:4 imports
 * github.com/klauspost/reedsolomon, pinned at v1.11.0 (go.mod:31, go.sum:553-554).
 * That module is NOT vendored under /root/reference and no Go toolchain exists here,
 * so this file restates its published algorithm:
 *
 *   - GF(2^8), generator polynomial x^8+x^4+x^3+x^2+1 (0x11D), generator 2 (A.1)
 *   - galExp(a,n): 1 if n==0, 0 if a==0, else exp[(log a * n) mod 255]  (A.1)
 *   - encode matrix: vm[r][c] = galExp(r,c) (n x k Vandermonde), M = vm * inv(vm[0:k]) (A.2)
 *   - Split: S = ceil(B/k), data zero-padded to k*S, parity rows zeroed      (A.5)
 *   - Encode: parity[j][x] = XOR_c M[k+j][c] * data[c][x]                   (A.2)
 *   - Reconstruct / ReconstructData: first-k-present rule, inverse of the
 *     k x k sub-matrix, missing data rows = inv rows x survivors, missing
 *     parity = parity rows x data                                          (A.3)
 *   - error sentinels ErrShortData, ErrTooFewShards, ErrShardNoData,
 *     ErrShardSize, ErrInvShardNum, ErrMaxShardNum                         (A.3, erasure.go:18-24)
 *
 * Reference-side call sites this follows:
 *   dag/node/dagnode/erasure.go:16-47  NewErasure (k>0, m>0, k+m<=256)
 *   dag/node/dagnode/erasure.go:51-65  EncodeData = Split + Encode (B==0 -> k+m nil shards)
 *   dag/node/dagnode/erasure.go:70-83  DecodeDataBlocks -> ReconstructData
 *   dag/node/dagnode/erasure.go:87-93  DecodeDataAndParityBlocks -> Reconstruct
 *   dag/node/dagnode/erasure.go:96-98, utils.go:6-21  ShardSize = ceilFrac(B, k)
 *
 * Pinning: rs_oracle_selftest() checks the upstream known-answer tests recalled in
 * SURVEY.md A.4 (galMultiply, galExp, the 3x3 inverse, TestOneEncode RS(5,5)) and the
 * reference's own RS(2,1) "123456" fixture (node_test.go:33, parity 3b 3c 39).
 * The reference itself is unbuildable here (Go), see DESIGN.md "Oracle".
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "rs_oracle.h"

/* ---------------------------------------------------------------- GF(2^8) (A.1) */
static uint8_t g_exp[510];
static uint8_t g_log[256];
static int g_init = 0;

static void gf_init(void) {
    if (g_init) return;
    unsigned x = 1;
    for (int i = 0; i < 255; i++) {
        g_exp[i] = (uint8_t)x;
        g_log[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    for (int i = 255; i < 510; i++) g_exp[i] = g_exp[i - 255];
    g_log[0] = 0; /* never consulted: mul/div short-circuit zero */
    g_init = 1;
}

uint8_t rs_oracle_gal_mul(uint8_t a, uint8_t b) {
    gf_init();
    if (a == 0 || b == 0) return 0;
    return g_exp[g_log[a] + g_log[b]];
}

static uint8_t gal_div(uint8_t a, uint8_t b) {
    /* b != 0 guaranteed by the callers (pivots are non-zero) */
    if (a == 0) return 0;
    int l = (int)g_log[a] - (int)g_log[b];
    if (l < 0) l += 255;
    return g_exp[l];
}

uint8_t rs_oracle_gal_exp(uint8_t a, int n) {
    gf_init();
    if (n == 0) return 1;
    if (a == 0) return 0;
    int l = ((int)g_log[a] * n) % 255;
    return g_exp[l];
}

/* ---------------------------------------------------------------- matrices (A.2) */
/* Gauss-Jordan inverse of a size x size matrix over GF(2^8), row-major.
 * Returns 0 on success, RS_ORACLE_ERR_SINGULAR if no inverse exists. */
int rs_oracle_invert(const uint8_t* in, uint8_t* out, int size) {
    gf_init();
    int w = 2 * size;
    uint8_t* a = (uint8_t*)malloc((size_t)size * w);
    if (!a) return RS_ORACLE_ERR_INVALID;
    for (int r = 0; r < size; r++) {
        for (int c = 0; c < size; c++) a[r * w + c] = in[r * size + c];
        for (int c = 0; c < size; c++) a[r * w + size + c] = (uint8_t)(r == c);
    }
    for (int r = 0; r < size; r++) {
        if (a[r * w + r] == 0) {
            int s = r + 1;
            while (s < size && a[s * w + r] == 0) s++;
            if (s == size) { free(a); return RS_ORACLE_ERR_SINGULAR; }
            for (int c = 0; c < w; c++) {
                uint8_t t = a[r * w + c]; a[r * w + c] = a[s * w + c]; a[s * w + c] = t;
            }
        }
        uint8_t p = a[r * w + r];
        if (p != 1) {
            for (int c = 0; c < w; c++) a[r * w + c] = gal_div(a[r * w + c], p);
        }
        for (int o = 0; o < size; o++) {
            if (o == r) continue;
            uint8_t f = a[o * w + r];
            if (!f) continue;
            for (int c = 0; c < w; c++) a[o * w + c] ^= rs_oracle_gal_mul(f, a[r * w + c]);
        }
    }
    for (int r = 0; r < size; r++)
        for (int c = 0; c < size; c++) out[r * size + c] = a[r * w + size + c];
    free(a);
    return 0;
}

/* n x k systematic encode matrix: Vandermonde times the inverse of its top square. */
int rs_oracle_build_matrix(int k, int m, uint8_t* out /* (k+m)*k */) {
    gf_init();
    int n = k + m;
    if (k <= 0 || m <= 0) return RS_ORACLE_ERR_INV_SHARD_NUM;
    if (n > 256) return RS_ORACLE_ERR_MAX_SHARD_NUM;
    uint8_t* vm = (uint8_t*)malloc((size_t)n * k);
    uint8_t* inv = (uint8_t*)malloc((size_t)k * k);
    for (int r = 0; r < n; r++)
        for (int c = 0; c < k; c++) vm[r * k + c] = rs_oracle_gal_exp((uint8_t)r, c);
    int rc = rs_oracle_invert(vm, inv, k);
    if (rc == 0) {
        for (int r = 0; r < n; r++)
            for (int c = 0; c < k; c++) {
                uint8_t acc = 0;
                for (int i = 0; i < k; i++) acc ^= rs_oracle_gal_mul(vm[r * k + i], inv[i * k + c]);
                out[r * k + c] = acc;
            }
    }
    free(vm);
    free(inv);
    return rc;
}

/* ---------------------------------------------------------------- codec (A.2, A.3, A.5) */
size_t rs_oracle_shard_size(size_t block_size, int k) {
    /* ceilFrac (utils.go:6-21) for positive operands */
    if (k <= 0) return 0;
    return (block_size + (size_t)k - 1) / (size_t)k;
}

int rs_oracle_split(int k, int m, const uint8_t* block, size_t B, uint8_t* shards /* (k+m)*S */) {
    if (B == 0) return RS_ORACLE_ERR_SHORT_DATA;
    size_t S = rs_oracle_shard_size(B, k);
    memset(shards, 0, (size_t)(k + m) * S);
    memcpy(shards, block, B);
    return 0;
}

/* rows x cols coefficient matrix applied to `cols` input rows of S bytes. */
static void code_rows(const uint8_t* coef, int rows, int cols, const uint8_t* const* in,
                      uint8_t* const* out, size_t S) {
    for (int j = 0; j < rows; j++) {
        uint8_t* o = out[j];
        memset(o, 0, S);
        for (int c = 0; c < cols; c++) {
            uint8_t f = coef[j * cols + c];
            if (!f) continue;
            const uint8_t* s = in[c];
            for (size_t x = 0; x < S; x++) o[x] ^= rs_oracle_gal_mul(f, s[x]);
        }
    }
}

int rs_oracle_encode(int k, int m, uint8_t* shards /* (k+m)*S contiguous */, size_t S) {
    if (S == 0) return RS_ORACLE_ERR_SHARD_NO_DATA;
    uint8_t* M = (uint8_t*)malloc((size_t)(k + m) * k);
    int rc = rs_oracle_build_matrix(k, m, M);
    if (rc) { free(M); return rc; }
    const uint8_t** in = (const uint8_t**)malloc(sizeof(uint8_t*) * k);
    uint8_t** out = (uint8_t**)malloc(sizeof(uint8_t*) * m);
    for (int c = 0; c < k; c++) in[c] = shards + (size_t)c * S;
    for (int j = 0; j < m; j++) out[j] = shards + (size_t)(k + j) * S;
    code_rows(M + (size_t)k * k, m, k, in, out, S);
    free(in); free(out); free(M);
    return 0;
}

/* shards: (k+m)*S contiguous; present[i] != 0 marks shard i as available.
 * Missing rows are overwritten; present rows are read only.
 * Mirrors upstream reconstruct(): quick return when nothing to do, ErrTooFewShards
 * when fewer than k present, first-k-present sub-matrix, data rows then parity rows. */
int rs_oracle_reconstruct(int k, int m, uint8_t* shards, size_t S, const uint8_t* present, int data_only) {
    int n = k + m;
    if (S == 0) return RS_ORACLE_ERR_SHARD_NO_DATA;
    int np = 0, dp = 0;
    for (int i = 0; i < n; i++) if (present[i]) { np++; if (i < k) dp++; }
    if (np == n || (data_only && dp == k)) return 0;
    if (np < k) return RS_ORACLE_ERR_TOO_FEW_SHARDS;

    uint8_t* M = (uint8_t*)malloc((size_t)n * k);
    int rc = rs_oracle_build_matrix(k, m, M);
    if (rc) { free(M); return rc; }
    uint8_t* sub = (uint8_t*)malloc((size_t)k * k);
    uint8_t* dec = (uint8_t*)malloc((size_t)k * k);
    const uint8_t** in = (const uint8_t**)malloc(sizeof(uint8_t*) * n);
    uint8_t** out = (uint8_t**)malloc(sizeof(uint8_t*) * n);
    uint8_t* coef = (uint8_t*)malloc((size_t)n * k);
    int row = 0;
    for (int i = 0; i < n && row < k; i++) {
        if (!present[i]) continue;
        memcpy(sub + (size_t)row * k, M + (size_t)i * k, (size_t)k);
        in[row] = shards + (size_t)i * S;
        row++;
    }
    rc = rs_oracle_invert(sub, dec, k);
    if (rc == 0) {
        int no = 0;
        for (int i = 0; i < k; i++) {
            if (present[i]) continue;
            memcpy(coef + (size_t)no * k, dec + (size_t)i * k, (size_t)k);
            out[no++] = shards + (size_t)i * S;
        }
        code_rows(coef, no, k, in, out, S);
        if (!data_only) {
            no = 0;
            for (int c = 0; c < k; c++) in[c] = shards + (size_t)c * S;
            for (int i = k; i < n; i++) {
                if (present[i]) continue;
                memcpy(coef + (size_t)no * k, M + (size_t)i * k, (size_t)k);
                out[no++] = shards + (size_t)i * S;
            }
            code_rows(coef, no, k, in, out, S);
        }
    }
    free(M); free(sub); free(dec); free(in); free(out); free(coef);
    return rc;
}

/* checkShards + shardSize restated: lens[i]==0 means missing. */
int rs_oracle_check_shards(int n, const size_t* lens, int nil_ok, size_t* S_out) {
    size_t S = 0;
    for (int i = 0; i < n; i++) if (lens[i]) { S = lens[i]; break; }
    if (S_out) *S_out = S;
    if (S == 0) return RS_ORACLE_ERR_SHARD_NO_DATA;
    for (int i = 0; i < n; i++) {
        if (lens[i] != S && (lens[i] != 0 || !nil_ok)) return RS_ORACLE_ERR_SHARD_SIZE;
    }
    return 0;
}

/* ---------------------------------------------------------------- KATs (A.4) */
static int eq(const uint8_t* a, const uint8_t* b, size_t n) { return memcmp(a, b, n) == 0; }

/* Returns 0 when every known answer matches, else the 1-based index of the first failure. */
int rs_oracle_selftest(void) {
    gf_init();
    /* galMultiply KATs */
    if (rs_oracle_gal_mul(3, 4) != 12) return 1;
    if (rs_oracle_gal_mul(7, 7) != 21) return 2;
    if (rs_oracle_gal_mul(23, 45) != 41) return 3;
    /* galExp KATs */
    if (rs_oracle_gal_exp(2, 2) != 4) return 4;
    if (rs_oracle_gal_exp(5, 20) != 235) return 5;
    if (rs_oracle_gal_exp(13, 7) != 43) return 6;
    if (rs_oracle_gal_exp(0, 0) != 1) return 7;
    /* 3x3 inverse KAT */
    {
        const uint8_t m3[9] = {56, 23, 98, 3, 100, 200, 45, 201, 123};
        const uint8_t want[9] = {175, 133, 33, 130, 13, 245, 112, 35, 126};
        uint8_t got[9];
        if (rs_oracle_invert(m3, got, 3) != 0 || !eq(got, want, 9)) return 8;
    }
    /* TestOneEncode: RS(5,5), 2-byte shards */
    {
        uint8_t sh[10 * 2] = {0, 1, 4, 5, 2, 3, 6, 7, 8, 9};
        const uint8_t want[10] = {12, 13, 10, 11, 14, 15, 90, 91, 94, 95};
        if (rs_oracle_encode(5, 5, sh, 2) != 0 || !eq(sh + 10, want, 10)) return 9;
    }
    /* reference fixture: RS(2,1) of "123456" (node_test.go:33) */
    {
        uint8_t sh[9];
        const uint8_t want[3] = {0x3b, 0x3c, 0x39};
        if (rs_oracle_split(2, 1, (const uint8_t*)"123456", 6, sh) != 0) return 10;
        if (rs_oracle_encode(2, 1, sh, 3) != 0 || !eq(sh + 6, want, 3)) return 11;
    }
    /* parity rows quoted in SURVEY A.2 */
    {
        uint8_t M[14 * 10];
        const uint8_t r42[8] = {27, 28, 18, 20, 28, 27, 20, 18};
        const uint8_t r104[10] = {129, 150, 175, 184, 210, 196, 254, 232, 3, 2};
        if (rs_oracle_build_matrix(4, 2, M) != 0 || !eq(M + 16, r42, 8)) return 12;
        if (rs_oracle_build_matrix(10, 4, M) != 0 || !eq(M + 100, r104, 10)) return 13;
    }
    return 0;
}
