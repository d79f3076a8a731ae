/*
 * gol_fastcpu.c — TEST / BENCH INFRASTRUCTURE ONLY (a CPU comparator).
 *
 * Not a restatement of the reference: this is the "honest fast-CPU
 * comparator" of SURVEY.md §8(c)/(d) — a bit-packed, bit-sliced B3/S23 torus
 * step on the host (64 cells per uint64, OpenMP over row chunks), timed by
 * bench.py beside the reference worker-pool port so the GPU number can be read
 * against a good CPU implementation too.  Rule and wrap are the reference's
 * (gol/distributor.go:350-417); tests/test_oracle_golden.py checks this file
 * against oracle_run on random boards and the golden fixtures.
 *
 * Layout: H rows x W/64 words, bit b of word k = column 64k + b (W % 64 == 0).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <omp.h>

int fastcpu_pack(const uint8_t *cells, int W, int H, uint64_t *words) {
    if (W <= 0 || H <= 0 || W % 64) return -1;
    const int nw = W / 64;
    for (int64_t y = 0; y < H; y++)
        for (int k = 0; k < nw; k++) {
            const uint8_t *c = cells + y * W + 64 * k;
            uint64_t v = 0;
            for (int b = 0; b < 64; b++) v |= (uint64_t)(c[b] == 255) << b;
            words[y * nw + k] = v;
        }
    return 0;
}

int fastcpu_unpack(const uint64_t *words, int W, int H, uint8_t *cells) {
    if (W <= 0 || H <= 0 || W % 64) return -1;
    const int nw = W / 64;
    for (int64_t y = 0; y < H; y++)
        for (int k = 0; k < nw; k++) {
            const uint64_t v = words[y * nw + k];
            for (int b = 0; b < 64; b++) cells[y * W + 64 * k + b] = (v >> b & 1) ? 255 : 0;
        }
    return 0;
}

/* 3-cell horizontal sums of one row (2-bit: h0 + 2 h1), torus in x. */
static inline __attribute__((always_inline)) void hsum_row(const uint64_t *r, int nw, uint64_t *h0, uint64_t *h1) {
    for (int i = 0; i < nw; i++) {
        const uint64_t x = r[i], p = r[i ? i - 1 : nw - 1], n = r[i + 1 < nw ? i + 1 : 0];
        const uint64_t w = (x << 1) | (p >> 63);  /* bit b = cell b-1 */
        const uint64_t e = (x >> 1) | (n << 63);  /* bit b = cell b+1 */
        h0[i] = w ^ x ^ e;
        h1[i] = (w & x) | (w & e) | (x & e);
    }
}

/* Output rows [y0, y1) of one turn: sum9 = three row sums, next = sum9 == 3 or
 * (alive and sum9 == 4). */
__attribute__((target_clones("avx512f", "avx2", "default")))
static void step_rows(const uint64_t *in, uint64_t *out, int nw, int H, int y0, int y1, uint64_t *scratch) {
    uint64_t *h0[3], *h1[3];
    for (int s = 0; s < 3; s++) {
        h0[s] = scratch + (size_t)(2 * s) * nw;
        h1[s] = scratch + (size_t)(2 * s + 1) * nw;
    }
    hsum_row(in + (size_t)((y0 - 1 + H) % H) * nw, nw, h0[0], h1[0]);
    hsum_row(in + (size_t)y0 * nw, nw, h0[1], h1[1]);
    for (int y = y0; y < y1; y++) {
        const int a = (y - y0) % 3, c = (y - y0 + 1) % 3, b = (y - y0 + 2) % 3;
        hsum_row(in + (size_t)((y + 1) % H) * nw, nw, h0[b], h1[b]);
        const uint64_t *cur = in + (size_t)y * nw;
        uint64_t *o = out + (size_t)y * nw;
        for (int i = 0; i < nw; i++) {
            const uint64_t a0 = h0[a][i], a1 = h1[a][i], c0 = h0[c][i], c1 = h1[c][i];
            const uint64_t b0 = h0[b][i], b1 = h1[b][i];
            const uint64_t t0 = a0 ^ c0 ^ b0, k0 = (a0 & c0) | (a0 & b0) | (c0 & b0);
            const uint64_t u = a1 ^ c1 ^ b1, v = (a1 & c1) | (a1 & b1) | (c1 & b1);
            const uint64_t p1 = u ^ k0, q = u & k0;
            const uint64_t p2 = v ^ q, p3 = v & q;
            o[i] = ~p3 & ((t0 & p1 & ~p2) | (cur[i] & ~t0 & ~p1 & p2));
        }
    }
}

/* ---- full-size fixture helpers (tests/golden/make_fullsize.py) ------------
 * The BASELINE configs' synthetic boards generated directly
 * in the packed layout: cell (y, x) alive <=> (splitmix64(seed ^ (y*W + x)) & 3)
 * == 0, the same rule as oracle_fill_random in gol_oracle.c. */
static inline uint64_t fc_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__attribute__((target_clones("avx512f", "avx2", "default")))
static uint64_t fill_word(uint64_t seed, uint64_t base) {
    uint64_t v = 0;
    for (int b = 0; b < 64; b++) v |= (uint64_t)((fc_splitmix64(seed ^ (base + (uint64_t)b)) & 3u) == 0) << b;
    return v;
}

/* Rows [row0, row0 + H) of a W-wide synthetic board (strips agree with the whole). */
int fastcpu_fill_random(uint64_t *words, int W, int H, int64_t row0, uint64_t seed, int threads) {
    if (W <= 0 || H <= 0 || W % 64 || threads < 1) return -1;
    const int nw = W / 64;
#pragma omp parallel for num_threads(threads) schedule(static)
    for (int64_t y = 0; y < H; y++)
        for (int k = 0; k < nw; k++)
            words[y * nw + k] = fill_word(seed, (uint64_t)(row0 + y) * (uint64_t)W + 64u * (uint64_t)k);
    return 0;
}

/* golhip_board_hash of the same board (include/golhip.h): the sum mod 2^64
 * over canonical 32-bit words i (row-major, W/32 per row) of
 * splitmix64((i << 32) | word_i); word 2k of a row is the low half of the
 * packed uint64 k, word 2k + 1 the high half.  word0 = the global index of
 * the first 32-bit word (strips add up). */
uint64_t fastcpu_hash(const uint64_t *words, int W, int H, int64_t word0, int threads) {
    if (W <= 0 || H <= 0 || W % 64 || threads < 1) return 0;
    const int64_t n = (int64_t)H * (W / 64);
    uint64_t h = 0;
#pragma omp parallel for num_threads(threads) reduction(+ : h) schedule(static)
    for (int64_t i = 0; i < n; i++) {
        const uint64_t v = words[i], j = (uint64_t)(word0 + 2 * i);
        h += fc_splitmix64((j << 32) | (v & 0xFFFFFFFFu)) + fc_splitmix64(((j + 1) << 32) | (v >> 32));
    }
    return h;
}

uint64_t fastcpu_popcount(const uint64_t *words, int W, int H, int threads) {
    if (W <= 0 || H <= 0 || W % 64 || threads < 1) return 0;
    const int64_t n = (int64_t)H * (W / 64);
    uint64_t c = 0;
#pragma omp parallel for num_threads(threads) reduction(+ : c) schedule(static)
    for (int64_t i = 0; i < n; i++) c += (uint64_t)__builtin_popcountll(words[i]);
    return c;
}

/* `turns` turns in place on H x W/64 words with `threads` OpenMP threads. */
int fastcpu_run(uint64_t *words, int W, int H, long turns, int threads) {
    if (W <= 0 || H < 3 || W % 64 || threads < 1) return -1;
    const int nw = W / 64;
    const size_t n = (size_t)H * nw;
    uint64_t *tmp = (uint64_t *)malloc(n * sizeof(uint64_t));
    uint64_t *scratch = (uint64_t *)malloc((size_t)threads * 6 * nw * sizeof(uint64_t));
    if (!tmp || !scratch) {
        free(tmp);
        free(scratch);
        return -1;
    }
    uint64_t *src = words, *dst = tmp;
    for (long t = 0; t < turns; t++) {
#pragma omp parallel num_threads(threads)
        {
            const int id = omp_get_thread_num(), nt = omp_get_num_threads();
            const int y0 = (int)((int64_t)H * id / nt), y1 = (int)((int64_t)H * (id + 1) / nt);
            if (y1 > y0) step_rows(src, dst, nw, H, y0, y1, scratch + (size_t)id * 6 * nw);
        }
        uint64_t *s = src;
        src = dst;
        dst = s;
    }
    if (src != words) memcpy(words, src, n * sizeof(uint64_t));
    free(tmp);
    free(scratch);
    return 0;
}
