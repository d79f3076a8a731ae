/* Exhaustive search for a cheaper pair rule.
 *
 * K1w's pair rule computes an output row from the row sum A of one input row
 * (two bits, a 2-LUT XOR3 / MAJ of the shifted row), the pair sum P of the two
 * middle rows (shared by the two output rows of the pair) and the centre c:
 *   next = (A + P == 3) | (c & A + P == 4).
 * gol_bits.h encodes P in binary (4 LUTs a pair) and needs 4 LUTs for the rule
 * (none with 3 exists for that encoding).  This program asks whether ANY
 * 3-bit code q of P (P = 0..6; the code of a P value may be any of several)
 * admits a 3-gate v_bitop3 rule R(a0, a1, c, q0, q1, q2):
 *   for every P there is a code q such that R(A, c, q) = next(A + P, c)
 *   for every A and every reachable c (c = 1 only if P >= 1: the centre is
 *   one of the pair's cells).
 * A rule found here would need an encoder (S, T) -> q of at most 4 gates from
 * the two rows' codes to beat 8 LUTs a word-turn; with none found, 8 is the
 * bound for this family of circuits (3-input LUTs, per-row sums, shared pairs).
 *
 * usage: rule_search [A encoding 0|1|2] [threads]
 *   encoding 0: A = a0 + 2 a1 (binary), 1: Gray (0 00, 1 01, 2 11, 3 10),
 *   2: 0 00, 1 11, 2 01, 3 10 (the three classes of 2-bit codes of a count
 *   under input swap and complement, which a LUT absorbs).
 * Build: gcc -O3 -march=native -fopenmp scripts/rule_search.c -o /tmp/rule_search
 * (-DCODE4: codes of four bits, 128-entry tables: a 4-gate pair encoder
 * has four outputs, e.g. gol_bits.h's carry k beside p0, p1, p2). */
#include <omp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#ifdef CODE4
enum { NQ = 4 };
typedef unsigned __int128 u64;  // truth tables over (a0, a1, c, q0..q3)
#else
enum { NQ = 3 };
typedef uint64_t u64;  // truth tables over (a0, a1, c, q0, q1, q2)
#endif
enum { NIN = 3 + NQ, NT = 1 << NIN };
static u64 IN[NIN];
static uint8_t care[7], tgt[7];

static u64 bitop(unsigned L, u64 x, u64 y, u64 z) {
    u64 r = 0;
    for (int m = 0; m < 8; ++m)
        if (L >> m & 1) r |= ((m & 4) ? x : ~x) & ((m & 2) ? y : ~y) & ((m & 1) ? z : ~z);
    return r;
}

static int valid(u64 T) {
    for (int P = 0; P < 7; ++P) {
        int ok = 0;
        for (int q = 0; q < (1 << NQ) && !ok; ++q) ok = (((uint8_t)(T >> (8 * q))) & care[P]) == tgt[P];
        if (!ok) return 0;
    }
    return 1;
}

int main(int argc, char **argv) {
    const int encsel = argc > 1 ? atoi(argv[1]) : 0;
    if (argc > 2) omp_set_num_threads(atoi(argv[2]));
    static const int ENC[3][4] = {{0, 1, 2, 3}, {0, 1, 3, 2}, {0, 3, 1, 2}};  // count -> (a0 | a1 << 1)
    for (int k = 0; k < NIN; ++k) {
        IN[k] = 0;
        for (int i = 0; i < NT; ++i)
            if (i >> k & 1) IN[k] |= (u64)1 << i;
    }
    for (int P = 0; P < 7; ++P) {
        care[P] = tgt[P] = 0;
        for (int A = 0; A < 4; ++A)
            for (int c = 0; c < 2; ++c) {
                if (c && P == 0) continue;
                const int idx = ENC[encsel][A] | c << 2;
                care[P] |= 1u << idx;
                if (A + P == 3 || (c && A + P == 4)) tgt[P] |= 1u << idx;
            }
    }
    if (encsel == 0) {  // sanity: gol_bits.h's 4-gate rule on the binary code is valid
        const u64 a0 = IN[0], a1 = IN[1], c = IN[2], p0 = IN[3], p1 = IN[4], p2 = IN[5];
        const u64 s6 = bitop(0x16, a0, p0, c), s7 = bitop(0x43, a1, p1, p2), s8 = bitop(0x94, c, s6, s7);
        if (!valid(bitop(0x8a, p2, s7, s8))) {
            printf("sanity check failed\n");
            return 1;
        }
    }
    // every one-gate function of three of the six inputs, deduplicated
    static u64 G1[35 * 256];
    int n1 = 0;
    for (int a = 0; a < NIN; ++a)
        for (int b = a + 1; b < NIN; ++b)
            for (int c = b + 1; c < NIN; ++c)
                for (unsigned L = 0; L < 256; ++L) {
                    const u64 t = bitop(L, IN[a], IN[b], IN[c]);
                    int dup = 0;
                    for (int j = 0; j < n1 && !dup; ++j) dup = G1[j] == t;
                    if (!dup) G1[n1++] = t;
                }
    long long found = 0, checked = 0;
    int printed = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : found, checked)
    for (int i1 = 0; i1 < n1; ++i1) {
        // signals: the inputs, then g1 (S[NIN]) and g2 (S[NIN + 1])
        u64 S[NIN + 2];
        memcpy(S, IN, sizeof IN);
        S[NIN] = G1[i1];
        if (valid(S[NIN])) {
#pragma omp critical
            printf("1-gate rule #%d\n", i1);
        }
        for (int a = 0; a < NIN + 1; ++a)
            for (int b = a + 1; b < NIN + 1; ++b)
                for (int c = b + 1; c < NIN + 1; ++c)
                    for (unsigned L2 = 0; L2 < 256; ++L2) {
                        S[NIN + 1] = bitop(L2, S[a], S[b], S[c]);
                        if (valid(S[NIN + 1])) {
#pragma omp critical
                            if (printed++ < 20) printf("2-gate rule: g1 #%d g2 = L%02x(s%d,s%d,s%d)\n", i1, L2, a, b, c);
                        }
                        // the last gate reads g2 and two other signals
                        for (int x = 0; x < NIN + 1; ++x)
                            for (int y = x + 1; y < NIN + 1; ++y) {
                                u64 mt[8];
                                const u64 g2 = S[NIN + 1];
                                for (int m = 0; m < 8; ++m)
                                    mt[m] = ((m & 4) ? g2 : ~g2) & ((m & 2) ? S[x] : ~S[x]) & ((m & 1) ? S[y] : ~S[y]);
                                // Gray-code walk over the 256 tables: minterms are disjoint
                                u64 T = 0;
                                for (unsigned g = 1; g < 256; ++g) {
                                    const int bit = __builtin_ctz(g);
                                    T ^= mt[bit];
                                    ++checked;
                                    if (valid(T)) {
                                        ++found;
#pragma omp critical
                                        if (printed++ < 40)
                                            printf("3-gate rule: g1 #%d g2 = L%02x(s%d,s%d,s%d) g3 = L%02x(g2,s%d,s%d)\n",
                                                   i1, L2, a, b, c, g ^ (g >> 1), x, y);
                                    }
                                }
                            }
                    }
    }
    printf("%d-bit codes, encoding %d: %d one-gate functions, %lld three-gate circuits checked, %lld valid\n", NQ, encsel, n1, checked,
           found);
    return 0;
}
