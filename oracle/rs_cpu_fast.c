/*
 * rs_cpu_fast.c -- TEST/BENCH INFRASTRUCTURE ONLY (bench.py cpu_baseline leg, tests).
 *
 * Multi-threaded SIMD restatement of the reference CPU path: klauspost/reedsolomon
 * v1.11.0 codeSomeShards as called from dag/node/dagnode/erasure.go:60 (Encode) and
 * :82/:88 (ReconstructData/Reconstruct), with WithAutoGoroutines-style fan-out (:37)
 * replaced by one pthread per core over independent blocks.  Same ISA family that
 * upstream selects by cpuid: AVX2 split-nibble VPSHUFB tables, or AVX-512 + GFNI
 * affine multiply (vgf2p8affineqb) when the host has it.  Results are byte-identical
 * to the scalar restatement in rs_oracle.c (checked in tests/test_oracle.py).
 * Never linked into the product library.
 */
#include <immintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "rs_oracle.h"

typedef struct {
    int rows, cols;
    uint8_t coef[256 * 256];
    /* per coefficient: 16-entry low/high nibble product tables (AVX2 path) */
    uint8_t* nib; /* rows*cols*32 */
    uint64_t* aff; /* rows*cols affine matrices (GFNI path) */
} coder_t;

static int g_isa = -1; /* 0 scalar, 1 avx2, 2 avx512+gfni */

static int detect_isa(void) {
    if (g_isa >= 0) return g_isa;
    __builtin_cpu_init();
    if (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
        __builtin_cpu_supports("gfni"))
        g_isa = 2;
    else if (__builtin_cpu_supports("avx2"))
        g_isa = 1;
    else
        g_isa = 0;
    const char* force = getenv("RS_CPU_ISA");
    if (force) {
        if (!strcmp(force, "scalar")) g_isa = 0;
        else if (!strcmp(force, "avx2") && g_isa >= 1) g_isa = 1;
    }
    return g_isa;
}

const char* rs_cpu_isa(void) {
    static const char* names[] = {"scalar", "avx2-vpshufb", "avx512-gfni"};
    return names[detect_isa()];
}

static void coder_setup(coder_t* cd, const uint8_t* coef, int rows, int cols) {
    cd->rows = rows;
    cd->cols = cols;
    memcpy(cd->coef, coef, (size_t)rows * cols);
    /* C11 aligned_alloc: the size must be a multiple of the alignment */
    cd->nib = (uint8_t*)aligned_alloc(64, ((size_t)rows * cols * 32 + 127) / 64 * 64);
    cd->aff = (uint64_t*)aligned_alloc(64, ((size_t)rows * cols * 8 + 127) / 64 * 64);
    for (int i = 0; i < rows * cols; i++) {
        uint8_t a = coef[i];
        for (int v = 0; v < 16; v++) {
            cd->nib[i * 32 + v] = rs_oracle_gal_mul(a, (uint8_t)v);
            cd->nib[i * 32 + 16 + v] = rs_oracle_gal_mul(a, (uint8_t)(v << 4));
        }
        /* affine matrix: result bit r = parity(byte[7-r] & x); byte[7-r] bit j = bit r of a*2^j */
        uint64_t q = 0;
        for (int r = 0; r < 8; r++) {
            uint8_t row = 0;
            for (int j = 0; j < 8; j++)
                row |= (uint8_t)(((rs_oracle_gal_mul(a, (uint8_t)(1u << j)) >> r) & 1u) << j);
            q |= (uint64_t)row << (8 * (7 - r));
        }
        cd->aff[i] = q;
    }
}

static void coder_free(coder_t* cd) {
    free(cd->nib);
    free(cd->aff);
}

static void code_scalar(const coder_t* cd, const uint8_t* const* in, uint8_t* const* out, size_t lo, size_t hi) {
    for (int j = 0; j < cd->rows; j++)
        for (size_t x = lo; x < hi; x++) {
            uint8_t acc = 0;
            for (int c = 0; c < cd->cols; c++) acc ^= rs_oracle_gal_mul(cd->coef[j * cd->cols + c], in[c][x]);
            out[j][x] = acc;
        }
}

__attribute__((target("avx2"))) static void code_avx2(const coder_t* cd, const uint8_t* const* in,
                                                      uint8_t* const* out, size_t S) {
    const __m256i mask = _mm256_set1_epi8(0x0f);
    size_t x = 0;
    const int R = cd->rows, C = cd->cols;
    for (; x + 32 <= S; x += 32) {
        for (int j0 = 0; j0 < R; j0 += 4) {
            int jn = R - j0 < 4 ? R - j0 : 4;
            __m256i acc[4] = {_mm256_setzero_si256(), _mm256_setzero_si256(), _mm256_setzero_si256(),
                              _mm256_setzero_si256()};
            for (int c = 0; c < C; c++) {
                __m256i v = _mm256_loadu_si256((const __m256i*)(in[c] + x));
                __m256i l = _mm256_and_si256(v, mask);
                __m256i h = _mm256_and_si256(_mm256_srli_epi64(v, 4), mask);
                for (int j = 0; j < jn; j++) {
                    const uint8_t* t = cd->nib + ((size_t)(j0 + j) * C + c) * 32;
                    __m256i tl = _mm256_broadcastsi128_si256(_mm_load_si128((const __m128i*)t));
                    __m256i th = _mm256_broadcastsi128_si256(_mm_load_si128((const __m128i*)(t + 16)));
                    acc[j] = _mm256_xor_si256(acc[j], _mm256_xor_si256(_mm256_shuffle_epi8(tl, l),
                                                                       _mm256_shuffle_epi8(th, h)));
                }
            }
            for (int j = 0; j < jn; j++) _mm256_storeu_si256((__m256i*)(out[j0 + j] + x), acc[j]);
        }
    }
    if (x < S) code_scalar(cd, in, out, x, S);
}

__attribute__((target("avx512f,avx512bw,gfni"))) static void code_gfni(const coder_t* cd, const uint8_t* const* in,
                                                                        uint8_t* const* out, size_t S) {
    size_t x = 0;
    const int R = cd->rows, C = cd->cols;
    for (; x + 64 <= S; x += 64) {
        for (int j0 = 0; j0 < R; j0 += 4) {
            int jn = R - j0 < 4 ? R - j0 : 4;
            __m512i acc[4] = {_mm512_setzero_si512(), _mm512_setzero_si512(), _mm512_setzero_si512(),
                              _mm512_setzero_si512()};
            for (int c = 0; c < C; c++) {
                __m512i v = _mm512_loadu_si512((const void*)(in[c] + x));
                for (int j = 0; j < jn; j++) {
                    __m512i A = _mm512_set1_epi64((long long)cd->aff[(size_t)(j0 + j) * C + c]);
                    acc[j] = _mm512_xor_si512(acc[j], _mm512_gf2p8affine_epi64_epi8(v, A, 0));
                }
            }
            for (int j = 0; j < jn; j++) _mm512_storeu_si512((void*)(out[j0 + j] + x), acc[j]);
        }
    }
    if (x < S) code_scalar(cd, in, out, x, S);
}

static void code_rows(const coder_t* cd, const uint8_t* const* in, uint8_t* const* out, size_t S) {
    switch (detect_isa()) {
        case 2: code_gfni(cd, in, out, S); break;
        case 1: code_avx2(cd, in, out, S); break;
        default: code_scalar(cd, in, out, 0, S); break;
    }
}

/* ---------------------------------------------------------------- batch drivers */
typedef struct {
    const coder_t* cd;
    const uint8_t* in_base;
    uint8_t* out_base;
    size_t in_stride, out_stride, S;
    const int* in_rows;  /* row indices inside a block, in units of S */
    const int* out_rows;
    size_t b0, b1;
    int out_same_buffer;
} job_t;

static void* run_job(void* p) {
    job_t* jb = (job_t*)p;
    const uint8_t* in[256];
    uint8_t* out[256];
    for (size_t b = jb->b0; b < jb->b1; b++) {
        const uint8_t* ib = jb->in_base + b * jb->in_stride;
        uint8_t* ob = jb->out_base + b * jb->out_stride;
        for (int c = 0; c < jb->cd->cols; c++) in[c] = ib + (size_t)jb->in_rows[c] * jb->S;
        for (int j = 0; j < jb->cd->rows; j++) out[j] = ob + (size_t)jb->out_rows[j] * jb->S;
        code_rows(jb->cd, in, out, jb->S);
    }
    return NULL;
}

static void run_batch(const coder_t* cd, const uint8_t* in_base, size_t in_stride, uint8_t* out_base,
                      size_t out_stride, size_t S, size_t nblocks, const int* in_rows, const int* out_rows,
                      int threads) {
    if (threads < 1) threads = 1;
    if ((size_t)threads > nblocks) threads = (int)(nblocks ? nblocks : 1);
    pthread_t th[256];
    job_t jobs[256];
    if (threads > 256) threads = 256;
    for (int t = 0; t < threads; t++) {
        jobs[t] = (job_t){cd, in_base, out_base, in_stride, out_stride, S, in_rows, out_rows,
                          nblocks * t / threads, nblocks * (t + 1) / threads, 0};
    }
    for (int t = 1; t < threads; t++) pthread_create(&th[t], NULL, run_job, &jobs[t]);
    run_job(&jobs[0]);
    for (int t = 1; t < threads; t++) pthread_join(th[t], NULL);
}

int rs_cpu_encode_batch(int k, int m, const uint8_t* data, size_t data_block_stride, uint8_t* parity,
                        size_t parity_block_stride, size_t S, size_t nblocks, int threads) {
    if (k <= 0 || m <= 0) return RS_ORACLE_ERR_INV_SHARD_NUM;
    if (k + m > 256) return RS_ORACLE_ERR_MAX_SHARD_NUM;
    if (S == 0) return RS_ORACLE_ERR_SHARD_NO_DATA;
    uint8_t* M = (uint8_t*)malloc((size_t)(k + m) * k);
    int rc = rs_oracle_build_matrix(k, m, M);
    if (rc) { free(M); return rc; }
    coder_t* cd = (coder_t*)malloc(sizeof(coder_t));
    coder_setup(cd, M + (size_t)k * k, m, k);
    int in_rows[256], out_rows[256];
    for (int c = 0; c < k; c++) in_rows[c] = c;
    for (int j = 0; j < m; j++) out_rows[j] = j;
    run_batch(cd, data, data_block_stride, parity, parity_block_stride, S, nblocks, in_rows, out_rows, threads);
    coder_free(cd);
    free(cd);
    free(M);
    return 0;
}

/* Batch reconstruct, one erasure pattern for every block (the RepairDataNode shape,
 * data_recovery.go:16-112).  shards: per block (k+m) rows of S bytes. */
int rs_cpu_reconstruct_batch(int k, int m, uint8_t* shards, size_t block_stride, size_t S, size_t nblocks,
                             const uint8_t* present, int data_only, int threads) {
    int n = k + m;
    if (k <= 0 || m <= 0) return RS_ORACLE_ERR_INV_SHARD_NUM;
    if (n > 256) return RS_ORACLE_ERR_MAX_SHARD_NUM;
    if (S == 0) return RS_ORACLE_ERR_SHARD_NO_DATA;
    int np = 0, dp = 0;
    for (int i = 0; i < n; i++) if (present[i]) { np++; if (i < k) dp++; }
    if (np == n || (data_only && dp == k)) return 0;
    if (np < k) return RS_ORACLE_ERR_TOO_FEW_SHARDS;
    uint8_t* M = (uint8_t*)malloc((size_t)n * k);
    int rc = rs_oracle_build_matrix(k, m, M);
    if (rc) { free(M); return rc; }
    uint8_t sub[256 * 256], dec[256 * 256], coef[256 * 256];
    int in_rows[256], out_rows[256];
    int row = 0;
    for (int i = 0; i < n && row < k; i++) {
        if (!present[i]) continue;
        memcpy(sub + row * k, M + (size_t)i * k, (size_t)k);
        in_rows[row++] = i;
    }
    rc = rs_oracle_invert(sub, dec, k);
    if (rc) { free(M); return rc; }
    coder_t* cd = (coder_t*)malloc(sizeof(coder_t));
    int no = 0;
    for (int i = 0; i < k; i++) {
        if (present[i]) continue;
        memcpy(coef + no * k, dec + i * k, (size_t)k);
        out_rows[no++] = i;
    }
    if (no) {
        coder_setup(cd, coef, no, k);
        run_batch(cd, shards, block_stride, shards, block_stride, S, nblocks, in_rows, out_rows, threads);
        coder_free(cd);
    }
    if (!data_only) {
        no = 0;
        for (int i = k; i < n; i++) {
            if (present[i]) continue;
            memcpy(coef + no * k, M + (size_t)i * k, (size_t)k);
            out_rows[no++] = i;
        }
        for (int c = 0; c < k; c++) in_rows[c] = c;
        if (no) {
            coder_setup(cd, coef, no, k);
            run_batch(cd, shards, block_stride, shards, block_stride, S, nblocks, in_rows, out_rows, threads);
            coder_free(cd);
        }
    }
    free(cd);
    free(M);
    return 0;
}
