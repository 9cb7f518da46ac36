/*
 * oracle/bitref.c — bit-packed CPU oracle for large boards.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle/refcpu.c header).  Never linked into
 * or called by the product library.
 *
 * It computes the same toroidal B3/S23 turn as calculateNextState
 * (SubServer/distributor.go:119-208), 64 cells per uint64 word with
 * LSB = lowest x, using an adder formulation deliberately different from the
 * GPU kernel's (8-neighbour carry-save count mod 8 here, 9-cell window there)
 * so the two are independent.  It is cross-checked against refcpu.c (the
 * literal restatement) and the reference's golden fixtures in
 * tests/test_oracle.py before it is trusted at 5120^2 .. 65536^2.
 *
 * Non-binary bytes (neither 0 nor 255): they count as dead neighbours and a
 * non-binary centre cell yields 0 (SubServer/distributor.go:178-200 with the
 * zero-initialised output of :122-125).  pack() returns a `blocked` mask of
 * those cells; step() clears them in its output when the mask is given.
 *
 * Random boards: word (y, j) = splitmix64((seed << 40) + y * nw + j), bits at
 * x >= W in the last word cleared.  The product's device-side generator uses
 * the same definition (conway-s-gol-distributed_amd/csrc/gol_kernels.hip).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static inline int nwords(int W) { return (W + 63) / 64; }
static inline uint64_t last_mask(int W)
{
    int nb = W - 64 * (nwords(W) - 1);
    return nb == 64 ? ~0ull : ((1ull << nb) - 1);
}

uint64_t bit_splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void bit_gen_random(uint64_t seed, int W, int H, uint64_t *words)
{
    int nw = nwords(W);
    uint64_t lm = last_mask(W);
    #pragma omp parallel for schedule(static)
    for (int y = 0; y < H; y++)
        for (int j = 0; j < nw; j++) {
            uint64_t v = bit_splitmix64((seed << 40) + (uint64_t)y * nw + j);
            words[(size_t)y * nw + j] = (j == nw - 1) ? (v & lm) : v;
        }
}

/* bytes -> packed bits (alive iff == 255). Returns the number of non-binary cells. */
long long bit_pack(const uint8_t *bytes, int W, int H, uint64_t *words, uint64_t *blocked)
{
    int nw = nwords(W);
    long long nonbin = 0;
    #pragma omp parallel for schedule(static) reduction(+:nonbin)
    for (int y = 0; y < H; y++) {
        const uint8_t *row = bytes + (size_t)y * W;
        for (int j = 0; j < nw; j++) {
            uint64_t a = 0, b = 0;
            for (int k = 0; k < 64; k++) {
                int x = 64 * j + k;
                if (x >= W) break;
                uint8_t v = row[x];
                if (v == 255) a |= 1ull << k;
                else if (v != 0) { b |= 1ull << k; nonbin++; }
            }
            words[(size_t)y * nw + j] = a;
            if (blocked) blocked[(size_t)y * nw + j] = b;
        }
    }
    return nonbin;
}

void bit_unpack(const uint64_t *words, int W, int H, uint8_t *bytes)
{
    int nw = nwords(W);
    #pragma omp parallel for schedule(static)
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++)
            bytes[(size_t)y * W + x] = ((words[(size_t)y * nw + x / 64] >> (x % 64)) & 1) ? 255 : 0;
}

/* west word: bit k = cell (x-1) of bit k's x, torus. */
static inline uint64_t westw(const uint64_t *row, int j, int nw, int nb)
{
    uint64_t carry = (j > 0) ? (row[j - 1] >> 63) : ((row[nw - 1] >> (nb - 1)) & 1);
    return (row[j] << 1) | carry;
}
/* east word: bit k = cell (x+1), torus. */
static inline uint64_t eastw(const uint64_t *row, int j, int nw, int nb)
{
    if (j < nw - 1) return (row[j] >> 1) | (row[j + 1] << 63);
    return (row[j] >> 1) | ((row[0] & 1) << (nb - 1));
}

void bit_step(const uint64_t *in, uint64_t *out, int W, int H, const uint64_t *blocked)
{
    int nw = nwords(W);
    int nb = W - 64 * (nw - 1);
    uint64_t lm = last_mask(W);
    #pragma omp parallel for schedule(static)
    for (int y = 0; y < H; y++) {
        const uint64_t *rn = in + (size_t)((y + H - 1) % H) * nw;
        const uint64_t *rc = in + (size_t)y * nw;
        const uint64_t *rs = in + (size_t)((y + 1) % H) * nw;
        for (int j = 0; j < nw; j++) {
            uint64_t n[8] = {
                westw(rn, j, nw, nb), rn[j], eastw(rn, j, nw, nb),
                westw(rc, j, nw, nb),        eastw(rc, j, nw, nb),
                westw(rs, j, nw, nb), rs[j], eastw(rs, j, nw, nb)};
            /* running 3-bit counter (b2 b1 b0), count mod 8 (count 8 -> 0, never 2/3) */
            uint64_t b0 = 0, b1 = 0, b2 = 0;
            for (int k = 0; k < 8; k++) {
                uint64_t c0 = b0 & n[k];
                b0 ^= n[k];
                uint64_t c1 = b1 & c0;
                b1 ^= c0;
                b2 ^= c1;
            }
            uint64_t alive = rc[j];
            uint64_t nx = ~b2 & b1 & (b0 | alive);
            if (blocked) nx &= ~blocked[(size_t)y * nw + j];
            if (j == nw - 1) nx &= lm;
            out[(size_t)y * nw + j] = nx;
        }
    }
}

uint64_t bit_popcount(const uint64_t *words, int W, int H)
{
    size_t n = (size_t)nwords(W) * H;
    uint64_t s = 0;
    #pragma omp parallel for schedule(static) reduction(+:s)
    for (long long i = 0; i < (long long)n; i++) s += (uint64_t)__builtin_popcountll(words[i]);
    return s;
}

/*
 * bit_run — `turns` turns in place.  `blocked` (nullable) applies to the first
 * turn only (after it every cell is 0 or 255).  counts (nullable) receives the
 * alive count after each turn (counts[t-1] for turn t).
 */
int bit_run(uint64_t *words, int W, int H, long long turns, const uint64_t *blocked,
            uint64_t *counts, int ncores)
{
    if (W < 2 || H < 1) return -1;
#ifdef _OPENMP
    if (ncores > 0) omp_set_num_threads(ncores);
#else
    (void)ncores;
#endif
    size_t n = (size_t)nwords(W) * H;
    uint64_t *tmp = (uint64_t *)malloc(n * sizeof(uint64_t));
    if (!tmp) return -1;
    uint64_t *a = words, *b = tmp;
    for (long long t = 0; t < turns; t++) {
        bit_step(a, b, W, H, t == 0 ? blocked : NULL);
        uint64_t *s = a; a = b; b = s;
        if (counts) counts[t] = bit_popcount(a, W, H);
    }
    if (a != words) memcpy(words, a, n * sizeof(uint64_t));
    free(tmp);
    return 0;
}
