/*
 * bsdb_oracle.c -- CPU restatement of bsdb's index-build arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY (see bsdb_oracle.h).  Written from the behaviour
 * of the reference, each function citing the file:line it restates.  Paths are
 * relative to the reference root (yc-huang/bsdb):
 *   spooky.c = src/main/c/spooky.c, mph.c = src/main/c/mph.c,
 *   GOV  = src/main/java/it/unimi/dsi/sux4j/mph/GOVMinimalPerfectHashFunctionModified.java
 *   CBHS = src/main/java/it/unimi/dsi/sux4j/io/ConcurrentBucketedHashStore.java
 */
#define _GNU_SOURCE
#include "bsdb_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* spooky.c:39 -- the SpookyHash constant. */
#define SPOOKY_CONST 0x9e3779b97f4a7c13ULL

static inline uint64_t rotl(uint64_t x, unsigned k) { return (x << k) | (x >> (64 - k)); }

/* Little-endian gather of up to 8 bytes into a word (byte j -> bits 8j..8j+7). */
static inline uint64_t le_bytes(const uint8_t *p, unsigned cnt) {
    uint64_t w = 0;
    for (unsigned j = 0; j < cnt; j++) w |= (uint64_t)p[j] << (8 * j);
    return w;
}

/* spooky.c:55-68 -- ShortMix: 12 (rot, add, xor) steps. */
static const unsigned MIX_ROT[12] = {50, 52, 30, 41, 54, 48, 38, 37, 62, 34, 5, 36};
static void short_mix(uint64_t h[4]) {
    for (int s = 0; s < 12; s++) {
        const int a = (s + 2) & 3, b = (s + 3) & 3, c = s & 3;
        h[a] = rotl(h[a], MIX_ROT[s]);
        h[a] += h[b];
        h[c] ^= h[a];
    }
}

/* spooky.c:72-84 -- ShortEnd: 11 (xor, rot, add) steps. */
static const unsigned END_ROT[11] = {15, 52, 26, 51, 28, 9, 47, 54, 32, 25, 63};
static void short_end(uint64_t h[4]) {
    for (int s = 0; s < 11; s++) {
        const int d = (s + 3) & 3, c = (s + 2) & 3;
        h[d] ^= h[c];
        h[c] = rotl(h[c], END_ROT[s]);
        h[d] += h[c];
    }
}

/* spooky.c:94-175.  Full 32-byte blocks go through ShortMix with the first
 * two words added to h2,h3 and the last two to h0,h1 after the mix; a 16-byte
 * remainder adds to h2,h3 and mixes; the last 0..15 bytes add little-endian
 * into h2 (bytes 0-7) and h3 (bytes 8-14); an empty tail adds the constant to
 * both.  h0 += 8*len (bit length, matching sux4j's BitVector length). */
void bo_spooky_short(const uint8_t *msg, uint64_t len, uint64_t seed, uint64_t out[4]) {
    uint64_t h[4] = {seed, seed, SPOOKY_CONST, SPOOKY_CONST};
    uint64_t rem = len & 31;
    const uint8_t *p = msg;
    if (len > 15) {
        for (uint64_t blk = 0; blk < len / 32; blk++, p += 32) {
            h[2] += le_bytes(p, 8);
            h[3] += le_bytes(p + 8, 8);
            short_mix(h);
            h[0] += le_bytes(p + 16, 8);
            h[1] += le_bytes(p + 24, 8);
        }
        if (rem >= 16) {
            h[2] += le_bytes(p, 8);
            h[3] += le_bytes(p + 8, 8);
            short_mix(h);
            p += 16;
            rem -= 16;
        }
    }
    if (rem == 0) {
        h[2] += SPOOKY_CONST;
        h[3] += SPOOKY_CONST;
    } else if (rem >= 8) {
        h[2] += le_bytes(p, 8);
        h[3] += le_bytes(p + 8, (unsigned)rem - 8);
    } else {
        h[2] += le_bytes(p, (unsigned)rem);
    }
    h[0] += len * 8;
    short_end(h);
    memcpy(out, h, sizeof h);
}

/* spooky.c:86-92 -- rehash of a signature into the equation triple. */
void bo_spooky_rehash(const uint64_t sig[2], uint64_t seed, uint64_t out[4]) {
    uint64_t h[4] = {seed, SPOOKY_CONST + sig[0], SPOOKY_CONST + sig[1], SPOOKY_CONST};
    short_mix(h);
    memcpy(out, h, sizeof h);
}

/* GOV:281,350 -- numBuckets = n / BUCKET_SIZE + 1 with BUCKET_SIZE = 1500. */
uint64_t bo_num_buckets(uint64_t n) { return n / 1500 + 1; }

/* GOV:559, CBHS:900,965 -- Math.multiplyHigh(sig0 >>> 1, 2m). */
uint32_t bo_bucket(uint64_t sig0, uint64_t num_buckets) {
    const unsigned __int128 prod = (unsigned __int128)(sig0 >> 1) * (unsigned __int128)(num_buckets * 2);
    return (uint32_t)(prod >> 64);
}

/* bucket of every signature (batched GOV:559) */
void bo_bucket_batch(const uint64_t *sig, uint64_t n, uint64_t num_buckets, uint32_t *out) {
    for (uint64_t i = 0; i < n; i++) out[i] = bo_bucket(sig[2 * i], num_buckets);
}

/* GOV:155-162,315-317 -- OFFSET_MASK = 2^56-1, C_TIMES_256 = floor(1.10*256) = 281. */
uint64_t bo_vertex_offset(uint64_t eos) { return ((eos & (~0ULL >> 8)) * 281) >> 8; }

/* mph.c:63-71 (sux4j Linear3SystemSolver.signatureToEquation, GOV:564,577). */
void bo_signature_to_equation(const uint64_t sig[2], uint64_t seed_bits, uint32_t nv, uint32_t e[3]) {
    uint64_t t[4];
    /* nv == 0 (an empty bucket, reachable only by absent keys): Java's
     * numberOfLeadingZeros(0) = 64 and shifts mod 64 give e = 0 */
    if (nv == 0) { e[0] = e[1] = e[2] = 0; return; }
    bo_spooky_rehash(sig, seed_bits, t);
    const int shift = __builtin_clzll((uint64_t)nv);
    const uint64_t mask = (1ULL << shift) - 1;
    for (int i = 0; i < 3; i++) e[i] = (uint32_t)(((t[i] & mask) * (uint64_t)nv) >> shift);
}

/* GOV:171-173 */
static inline uint64_t nz_pairs(uint64_t x) { return (uint64_t)__builtin_popcountll((x | x >> 1) & 0x5555555555555555ULL); }

/* GOV:183-197, mph.c:49-60 -- nonzero 2-bit fields in [start, end). */
uint64_t bo_count_nonzero_pairs(uint64_t start, uint64_t end, const uint64_t *array) {
    uint64_t blk = start >> 5;
    const uint64_t end_blk = end >> 5;
    const unsigned so = (unsigned)(start & 31), eo = (unsigned)(end & 31);
    if (blk == end_blk) return nz_pairs((array[blk] & ((1ULL << (eo * 2)) - 1)) >> (so * 2));
    uint64_t pairs = 0;
    if (so) pairs += nz_pairs(array[blk++] >> (so * 2));
    while (blk < end_blk) pairs += nz_pairs(array[blk++]);
    if (eo) pairs += nz_pairs(array[blk] & ((1ULL << (eo * 2)) - 1));
    return pairs;
}

void bo_hash_fixed(const uint8_t *keys, uint32_t key_len, uint64_t n, uint64_t seed, uint64_t *sig) {
    uint64_t t[4];
    for (uint64_t i = 0; i < n; i++) {
        bo_spooky_short(keys + i * key_len, key_len, seed, t);
        sig[2 * i] = t[0];
        sig[2 * i + 1] = t[1];
    }
}

void bo_hash_var(const uint8_t *blob, const uint64_t *off, uint64_t n, uint64_t seed, uint64_t *sig) {
    uint64_t t[4];
    for (uint64_t i = 0; i < n; i++) {
        bo_spooky_short(blob + off[i], off[i + 1] - off[i], seed, t);
        sig[2 * i] = t[0];
        sig[2 * i + 1] = t[1];
    }
}

void bo_histogram_fixed(const uint8_t *keys, uint32_t key_len, uint64_t n, uint64_t seed,
                        uint64_t m, uint32_t *counts) {
    uint64_t t[4];
    for (uint64_t i = 0; i < n; i++) {
        bo_spooky_short(keys + i * key_len, key_len, seed, t);
        counts[bo_bucket(t[0], m)]++;
    }
}

void bo_histogram_var(const uint8_t *blob, const uint64_t *off, uint64_t n, uint64_t seed,
                      uint64_t m, uint32_t *counts) {
    uint64_t t[4];
    for (uint64_t i = 0; i < n; i++) {
        bo_spooky_short(blob + off[i], off[i + 1] - off[i], seed, t);
        counts[bo_bucket(t[0], m)]++;
    }
}

/* GOV:391-393 */
void bo_edge_offsets(const uint32_t *counts, uint64_t m, uint64_t *E) {
    E[0] = 0;
    for (uint64_t b = 0; b < m; b++) E[b + 1] = E[b] + counts[b];
}

/* SURVEY.md §8(d) D2 synthetic keys.  splitmix64 is a bijection on u64, so
 * bytes 0-7 = splitmix64(i ^ 0xB5DB0001) make keys distinct by construction. */
uint64_t bo_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9e3779b97f4a7c15ULL;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

static inline void gen_key13(uint64_t i, uint8_t k[16]) {
    const uint64_t w0 = bo_splitmix64(i ^ 0xB5DB0001ULL);
    const uint64_t w1 = (i ^ (bo_splitmix64(i + 1) >> 24)) & 0xFFFFFFFFFFULL;
    memcpy(k, &w0, 8);
    memcpy(k + 8, &w1, 8);   /* little-endian host: bytes 8..12 = low 40 bits */
}

void bo_gen_keys13(uint64_t first, uint64_t n, uint8_t *out) {
    uint8_t k[16];
    for (uint64_t i = 0; i < n; i++) {
        gen_key13(first + i, k);
        memcpy(out + 13 * i, k, 13);
    }
}

/* Config C5 generator (the device's k_gen_var_len / k_gen_var_fill restated):
 * floor(CDF(r) * 2^64) of Zipf(s = 1.1) over ranks r = 1..57, r = 1..56. */
static const uint64_t ZIPF_CDF[56] = {
    0x415ff50621eab000ULL, 0x5fdf8ea4661c1800ULL, 0x7365cc48cd422800ULL, 0x81a02c160ca0d800ULL,
    0x8cc1c51827e0f000ULL, 0x95dd881c0eabb000ULL, 0x9d8d9c8bd387d800ULL, 0xa430d6d3c06da800ULL,
    0xaa0593efa19cb800ULL, 0xaf36f652f272a000ULL, 0xb3e4079390b42800ULL, 0xb823d5bdeb558000ULL,
    0xbc07f52bb16ae800ULL, 0xbf9e197287e21000ULL, 0xc2f123c939aa0800ULL, 0xc609db869ad6f800ULL,
    0xc8ef6f73a3a9d800ULL, 0xcba7d2952de20000ULL, 0xce38001f766e2000ULL, 0xd0a42e21797a3800ULL,
    0xd2eff3ea03b6c000ULL, 0xd51e678ba501e800ULL, 0xd73234d900b38000ULL, 0xd92daf816c491000ULL,
    0xdb12e17da86ff800ULL, 0xdce396a9b5e6c000ULL, 0xdea1662ec6fe5800ULL, 0xe04dba370d317800ULL,
    0xe1e9d64761753000ULL, 0xe376dc8509ffe800ULL, 0xe4f5d21dcfad2800ULL, 0xe667a2fc93d9d000ULL,
    0xe7cd24eb876f7000ULL, 0xe9271a3e3b92e800ULL, 0xea76341874c6f000ULL, 0xebbb14628b26f800ULL,
    0xecf64f78eaa7d000ULL, 0xee286da1bdeba000ULL, 0xef51ec51cc50e000ULL, 0xf0733f47f9ee2000ULL,
    0xf18cd1858f189800ULL, 0xf29f062863636800ULL, 0xf3aa392b30515800ULL, 0xf4aec00f9fea5000ULL,
    0xf5acea751b007800ULL, 0xf6a5029ee3f44800ULL, 0xf7974deba8448800ULL, 0xf8840d40614fb000ULL,
    0xf96b7d68184c6800ULL, 0xfa4dd769e82e0000ULL, 0xfb2b50d667f27000ULL, 0xfc041c0d7f209800ULL,
    0xfcd8687d83bcc000ULL, 0xfda862dc63a64800ULL, 0xfe74355b824d6000ULL, 0xff3c07d6de49e800ULL};

uint32_t bo_varkey_len(uint64_t i) {
    const uint64_t u = bo_splitmix64(i ^ 0xB5DB0005ULL);
    uint32_t r = 0;
    for (int t = 0; t < 56; t++) r += u >= ZIPF_CDF[t];
    return 8 + r;
}

static uint32_t gen_varkey(uint64_t i, uint8_t *d) {
    const uint32_t len = bo_varkey_len(i);
    for (int b = 0; b < 8; b++) d[b] = (uint8_t)(i >> (56 - 8 * b));
    for (uint32_t j = 8; j < len; j += 8) {
        const uint64_t w = bo_splitmix64(((i << 3) + ((j - 8) >> 3)) ^ 0xB5DB0005A5A5A5A5ULL);
        for (uint32_t b = 0; b < 8 && j + b < len; b++) d[j + b] = (uint8_t)(w >> (8 * b));
    }
    return len;
}

void bo_gen_keys_var(uint64_t first, uint64_t n, uint64_t *offsets, uint8_t *blob) {
    offsets[0] = 0;
    for (uint64_t k = 0; k < n; k++) {
        const uint32_t len = blob ? gen_varkey(first + k, blob + offsets[k]) : bo_varkey_len(first + k);
        offsets[k + 1] = offsets[k] + len;
    }
}

/* ---- threaded CPU baseline --------------------------------------------- */
typedef struct { uint64_t first, lo, hi; uint8_t *out; } gen_job;
static void *mt_gen_only(void *arg) {
    gen_job *j = (gen_job *)arg;
    bo_gen_keys13(j->first + j->lo, j->hi - j->lo, j->out + 13 * j->lo);
    return NULL;
}

void bo_gen_keys13_mt(uint64_t first, uint64_t n, uint8_t *out, int threads) {
    if (threads < 1) threads = 1;
    gen_job jobs[256];
    pthread_t tid[256];
    if (threads > 256) threads = 256;
    for (int t = 0; t < threads; t++) {
        jobs[t] = (gen_job){first, n * t / threads, n * (t + 1) / threads, out};
        pthread_create(&tid[t], NULL, mt_gen_only, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
}

typedef struct {
    const uint8_t *keys;
    uint32_t key_len;
    uint64_t first, lo, hi, seed, m;
    uint32_t *local;
} mt_job;

static void *mt_gen13(void *arg) {
    mt_job *j = (mt_job *)arg;
    uint8_t k[16];
    uint64_t t[4];
    for (uint64_t i = j->lo; i < j->hi; i++) {
        gen_key13(j->first + i, k);
        bo_spooky_short(k, 13, j->seed, t);
        j->local[bo_bucket(t[0], j->m)]++;
    }
    return NULL;
}

static void *mt_fixed(void *arg) {
    mt_job *j = (mt_job *)arg;
    uint64_t t[4];
    for (uint64_t i = j->lo; i < j->hi; i++) {
        bo_spooky_short(j->keys + i * j->key_len, j->key_len, j->seed, t);
        j->local[bo_bucket(t[0], j->m)]++;
    }
    return NULL;
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static double run_mt(void *(*fn)(void *), const uint8_t *keys, uint32_t key_len, uint64_t first,
                     uint64_t n, uint64_t seed, uint64_t m, uint32_t *counts, int threads) {
    if (threads < 1) threads = 1;
    mt_job *jobs = calloc((size_t)threads, sizeof *jobs);
    pthread_t *tid = calloc((size_t)threads, sizeof *tid);
    for (int t = 0; t < threads; t++) jobs[t].local = calloc(m, sizeof(uint32_t));
    const double t0 = now_s();
    for (int t = 0; t < threads; t++) {
        jobs[t] = (mt_job){keys, key_len, first, n * t / threads, n * (t + 1) / threads, seed, m, jobs[t].local};
        pthread_create(&tid[t], NULL, fn, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    for (int t = 0; t < threads; t++)
        for (uint64_t b = 0; b < m; b++) counts[b] += jobs[t].local[b];
    const double dt = now_s() - t0;
    for (int t = 0; t < threads; t++) free(jobs[t].local);
    free(jobs);
    free(tid);
    return dt;
}

double bo_histogram_gen13_mt(uint64_t first, uint64_t n, uint64_t seed, uint64_t m, uint32_t *counts,
                             int threads) {
    return run_mt(mt_gen13, NULL, 13, first, n, seed, m, counts, threads);
}

double bo_histogram_fixed_mt(const uint8_t *keys, uint32_t key_len, uint64_t n, uint64_t seed,
                             uint64_t m, uint32_t *counts, int threads) {
    return run_mt(mt_fixed, keys, key_len, 0, n, seed, m, counts, threads);
}

static void *mt_genvar(void *arg) {
    mt_job *j = (mt_job *)arg;
    uint8_t k[72];
    uint64_t t[4];
    for (uint64_t i = j->lo; i < j->hi; i++) {
        const uint32_t len = gen_varkey(j->first + i, k);
        bo_spooky_short(k, len, j->seed, t);
        j->local[bo_bucket(t[0], j->m)]++;
    }
    return NULL;
}

double bo_histogram_genvar_mt(uint64_t first, uint64_t n, uint64_t seed, uint64_t m, uint32_t *counts,
                              int threads) {
    return run_mt(mt_genvar, NULL, 0, first, n, seed, m, counts, threads);
}

/* ---- A12 lookup ---------------------------------------------------------- */
/* dsiutils LongArrayBitVector.asLongBigList(width): element i occupies bits
 * [i*w, (i+1)*w) of the little-endian word array (GOV:494,503). */
uint64_t bo_bitlist_get(const uint64_t *w, uint64_t i, uint32_t width) {
    const uint64_t bit = i * width, word = bit >> 6;
    const unsigned off = (unsigned)(bit & 63);
    const uint64_t mask = width == 64 ? ~0ULL : ((1ULL << width) - 1);
    uint64_t v = w[word] >> off;
    if (off + width > 64) v |= w[word + 1] << (64 - off);
    return v & mask;
}

void bo_bitlist_set(uint64_t *w, uint64_t i, uint32_t width, uint64_t v) {
    const uint64_t bit = i * width, word = bit >> 6;
    const unsigned off = (unsigned)(bit & 63);
    const uint64_t mask = width == 64 ? ~0ULL : ((1ULL << width) - 1);
    v &= mask;
    w[word] = (w[word] & ~(mask << off)) | (v << off);
    if (off + width > 64) {
        const unsigned hi = off + width - 64;
        const uint64_t hmask = (1ULL << hi) - 1;
        w[word + 1] = (w[word + 1] & ~hmask) | (v >> (64 - off));
    }
}

static inline uint64_t two_bit(const uint64_t *a, uint64_t pos) {
    pos *= 2;
    return (a[pos >> 6] >> (pos & 63)) & 3;
}

/* GOV:573-580 */
int64_t bo_lookup_nocheck(const bo_mph *m, const uint64_t sig[2]) {
    const uint32_t b = bo_bucket(sig[0], m->multiplier / 2);
    const uint64_t eos = m->E[b];
    const uint64_t vo = bo_vertex_offset(eos);
    const uint32_t nv = (uint32_t)(bo_vertex_offset(m->E[b + 1]) - vo);
    uint32_t e[3];
    bo_signature_to_equation(sig, eos & ~(~0ULL >> 8), nv, e);
    const uint64_t h = (two_bit(m->array, e[0] + vo) + two_bit(m->array, e[1] + vo) +
                        two_bit(m->array, e[2] + vo)) % 3;
    return (int64_t)((eos & (~0ULL >> 8)) + bo_count_nonzero_pairs(vo, vo + e[h], m->array));
}

/* GOV:557-569 -- with the checksum test of hash.checksum.bits. */
int64_t bo_lookup(const bo_mph *m, const uint64_t sig[2]) {
    const int64_t r = bo_lookup_nocheck(m, sig);
    if ((uint64_t)r >= m->n) return -1;
    if (m->sig_width) {
        const uint64_t mask = ~0ULL >> (64 - m->sig_width);
        if (bo_bitlist_get(m->signatures, (uint64_t)r, m->sig_width) != (sig[0] & mask)) return -1;
    }
    return r;
}

/* GOV:357,483-485 -- bitVector of 2*(1 + V) bits, V = n*281>>8. */
uint64_t bo_values_words(uint64_t n) { return (2 * (1 + ((n * 281) >> 8)) + 63) / 64; }

/* ======================================================================== *
 * GOV build (A5 sort, A8 per-bucket solve, A11 signing).                   *
 *                                                                          *
 * Follows the GOV construction of GOV:329-508: bucket b holds the keys     *
 * whose signature maps to b, sorted by unsigned (sig0, sig1) (CBHS:939-955)*
 * with duplicates rejected (CBHS:969-972); its nv = vo(E[b+1]) - vo(E[b])  *
 * variables (GOV:421-423); each key's equation is signatureToEquation     *
 * (mph.c:63-71) under local seed j<<56, j = 0..255 (GOV:425-432); the     *
 * solution stores 3 for a hinge whose value is 0 (GOV:126-139) and the    *
 * lookup returns E[b] + #nonzero pairs before the hinge (GOV:557-580).    *
 *                                                                          *
 * The hinge assignment (orientation) and therefore the chosen solution is *
 * this project's own deterministic algorithm, NOT sux4j 5.4.1's           *
 * Linear3SystemSolver/Orient3Hypergraph (third-party, absent): parity     *
 * unpinned; validity is checked through the reference's mph.c lookup.     *
 *   1. peeling in rounds: every vertex of degree 1 at the start of a round *
 *      claims its edge, the smallest such vertex of an edge wins;          *
 *   2. the 2-core is oriented by greedy matching in edge order (the free   *
 *      vertex with the fewest core edges still to come) plus BFS          *
 *      augmenting paths in edge order;                                     *
 *   3. the core system (unknowns = core hinges, non-hinge vertices = 0) is *
 *      solved over F3 block by block on the SCCs of its dependency graph   *
 *      (Gauss-Jordan per block, columns in increasing edge order);         *
 *   4. peeled edges are solved in reverse round order.                     *
 *                                                                          *
 * Seed rule (GOV:425-432): the next local seed only when the bucket's      *
 * system has NO solution -- an unorientable core (sux4j's "unorientable",  *
 * GOV:427) or an inconsistent block ("unsolvable", GOV:428).  A singular   *
 * but consistent block is solved: its solution is the one whose free       *
 * columns (the columns of its reduced row echelon form without a pivot,    *
 * in increasing edge order) are 0.  That choice is a function of the block *
 * alone, whatever elimination reaches it, which keeps the device's         *
 * feedback-vertex-set solver bit-identical to this one.                    *
 * ======================================================================== */

/* attempts and their outcomes (bo_solve_stats), summed over threads */
static uint64_t g_stats[5];  /* attempts, unorientable, inconsistent, degenerate edge, singular solved */

void bo_solve_stats(uint64_t out[5], int reset) {
    for (int i = 0; i < 5; i++) {
        out[i] = __atomic_load_n(&g_stats[i], __ATOMIC_RELAXED);
        if (reset) __atomic_store_n(&g_stats[i], 0, __ATOMIC_RELAXED);
    }
}

static inline void stat_add(int i) { __atomic_fetch_add(&g_stats[i], 1, __ATOMIC_RELAXED); }

static int cmp_i32(const void *a, const void *b) {
    const int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
    return x < y ? -1 : x > y;
}

static int cmp_sig(const void *a, const void *b) {
    const uint64_t *x = (const uint64_t *)a, *y = (const uint64_t *)b;
    if (x[0] != y[0]) return x[0] < y[0] ? -1 : 1;
    if (x[1] != y[1]) return x[1] < y[1] ? -1 : 1;
    return 0;
}

/* bit-sliced GF(3): value = p1 ? 1 : p2 ? 2 : 0 */
static inline void gf3_add(uint64_t *x1, uint64_t *x2, const uint64_t y1, const uint64_t y2) {
    const uint64_t a1 = *x1, a2 = *x2;
    *x1 = (a1 & ~y1 & ~y2) | (~a1 & ~a2 & y1) | (a2 & y2);
    *x2 = (a2 & ~y1 & ~y2) | (~a1 & ~a2 & y2) | (a1 & y1);
}

/* Solves one bucket.  sig: cnt sorted signatures; writes vals[nv] (0..3).
 * Returns 0 solved, 1 no solution under this seed (try the next one). */
static int solve_bucket(const uint64_t *sig, uint32_t cnt, uint32_t nv, uint64_t seed_bits, uint8_t *vals,
                        int32_t *ws) {
    memset(vals, 0, nv);
    if (cnt == 0) return 0;
    stat_add(0);
    /* one key on one vertex: its edge is (0,0,0); h = 0 holds for any value and
     * the hinge stores 3 (GOV:126-139).  Other triple edges take the next seed. */
    if (cnt == 1 && nv == 1) { vals[0] = 3; return 0; }
    int tiny = cnt <= 12;
    /* workspace layout */
    uint32_t *e = (uint32_t *)ws;                     /* 3*cnt */
    uint32_t *deg = e + 3 * cnt;                      /* nv */
    uint32_t *xe = deg + nv;                          /* nv: xor of incident edges */
    int32_t *hinge = (int32_t *)(xe + nv);            /* cnt: hinge vertex of edge or -1 */
    int32_t *round_of = hinge + cnt;                  /* cnt: peel round or -1 (core) */
    int32_t *vowner = round_of + cnt;                 /* nv: edge owning vertex as hinge or -1 */
    int32_t *claim = vowner + nv;                     /* cnt */
    int32_t *bfs_prev = claim + cnt;                  /* cnt */
    int32_t *bfs_via = bfs_prev + cnt;                /* cnt */
    int32_t *queue = bfs_via + cnt;                   /* cnt */
    uint8_t *seen_v = (uint8_t *)(queue + cnt);       /* nv */
    uint8_t *xval = seen_v + nv;                      /* nv: solved F3 value per vertex */

    for (uint32_t k = 0; k < cnt; k++) {
        uint32_t ee[3];
        bo_signature_to_equation(sig + 2 * k, seed_bits, nv, ee);
        /* a repeated vertex is kept (coefficient 2); a triple one makes the
         * equation 0 = h unsatisfiable for its orientation: next seed */
        if (ee[0] == ee[1] && ee[1] == ee[2] && !tiny) { stat_add(3); return 1; }
        e[3 * k] = ee[0]; e[3 * k + 1] = ee[1]; e[3 * k + 2] = ee[2];
    }
    memset(deg, 0, nv * sizeof *deg);
    memset(xe, 0, nv * sizeof *xe);
    for (uint32_t k = 0; k < cnt; k++)
        for (int i = 0; i < 3; i++) { deg[e[3 * k + i]]++; xe[e[3 * k + i]] ^= k; }
    for (uint32_t k = 0; k < cnt; k++) { hinge[k] = -1; round_of[k] = -1; }
    for (uint32_t v = 0; v < nv; v++) vowner[v] = -1;

    /* 1. peeling in rounds */
    int rounds = 0;
    for (;;) {
        int any = 0;
        for (uint32_t k = 0; k < cnt; k++) claim[k] = -1;
        for (uint32_t v = 0; v < nv; v++) {
            if (deg[v] != 1) continue;
            const uint32_t k = xe[v];
            if (claim[k] < 0 || (uint32_t)claim[k] > v) claim[k] = (int32_t)v;
        }
        for (uint32_t k = 0; k < cnt; k++) {
            if (claim[k] < 0) continue;
            any = 1;
            hinge[k] = claim[k];
            vowner[claim[k]] = (int32_t)k;
            round_of[k] = rounds;
        }
        if (!any) break;
        for (uint32_t k = 0; k < cnt; k++) {
            if (round_of[k] != rounds) continue;
            for (int i = 0; i < 3; i++) { deg[e[3 * k + i]]--; xe[e[3 * k + i]] ^= k; }
        }
        rounds++;
    }

    /* 2. orientation of the 2-core: greedy, then BFS augmenting paths.  The
     * greedy takes core edges in increasing order; each takes, among its free
     * vertices, the one with the fewest core edges still to come (deg: the
     * peel's degrees, decremented as edges pass; ties: first in the edge). */
    uint32_t ncore = 0;
    for (uint32_t k = 0; k < cnt; k++) {
        if (round_of[k] >= 0) continue;
        ncore++;
        int32_t best = -1;
        uint32_t bd = 0xFFFFFFFFu;
        for (int i = 0; i < 3; i++) {
            const uint32_t v = e[3 * k + i];
            if (vowner[v] < 0 && deg[v] < bd) { bd = deg[v]; best = (int32_t)v; }
        }
        for (int i = 0; i < 3; i++) deg[e[3 * k + i]]--;
        if (best >= 0) { vowner[best] = (int32_t)k; hinge[k] = best; }
    }
    for (uint32_t k0 = 0; k0 < cnt; k0++) {
        if (round_of[k0] >= 0 || hinge[k0] >= 0) continue;
        /* BFS over edges: from edge k through vertex v to the edge owning v */
        memset(seen_v, 0, nv);
        int qh = 0, qt = 0, found_v = -1, found_e = -1;
        queue[qt++] = (int32_t)k0;
        bfs_prev[k0] = -1;
        while (qh < qt && found_v < 0) {
            const int32_t k = queue[qh++];
            for (int i = 0; i < 3; i++) {
                const uint32_t v = e[3 * k + i];
                if (seen_v[v]) continue;
                seen_v[v] = 1;
                const int32_t o = vowner[v];
                if (o < 0) { found_v = (int32_t)v; found_e = k; break; }
                bfs_prev[o] = k;
                bfs_via[o] = (int32_t)v;
                queue[qt++] = o;
            }
        }
        if (found_v < 0) { stat_add(1); return 1; } /* unorientable */
        /* flip along the path: found_e takes found_v, its old hinge goes to prev ... */
        int32_t k = found_e, v = found_v;
        for (;;) {
            const int32_t old = hinge[k];
            hinge[k] = v;
            vowner[v] = k;
            if (k == (int32_t)k0) break;
            v = old;                 /* the vertex k gave up ... */
            k = bfs_prev[k];         /* ... is taken by the edge we came from */
            (void)bfs_via;
        }
    }

    memset(xval, 0, nv);
    /* tiny buckets (<= 12 keys: only in sets of n < ~1500) can be singular as a
     * whole (nv == cnt makes every row sum to 0 mod 3): take the first assignment
     * of the hinge values, in base-3 order with edge 0 least significant, that
     * satisfies every equation */
    if (tiny) {
        uint32_t total = 1;
        for (uint32_t k = 0; k < cnt; k++) total *= 3;
        for (uint32_t a = 0; a < total; a++) {
            uint32_t t = a;
            for (uint32_t k = 0; k < cnt; k++) { xval[hinge[k]] = (uint8_t)(t % 3); t /= 3; }
            int ok = 1;
            for (uint32_t k = 0; k < cnt && ok; k++) {
                int h = 0;
                while (e[3 * k + h] != (uint32_t)hinge[k]) h++;
                const uint32_t sum = xval[e[3 * k]] + xval[e[3 * k + 1]] + xval[e[3 * k + 2]];
                ok = sum % 3 == (uint32_t)h;
            }
            if (ok) {
                for (uint32_t k = 0; k < cnt; k++) vals[hinge[k]] = xval[hinge[k]] ? xval[hinge[k]] : 3;
                return 0;
            }
        }
        return 1;
    }
    /* 3. the core system, unknowns = core hinges (non-hinge vertices are 0),
     * solved block by block over the strongly connected components of "edge k
     * uses the hinge of edge k'" (Tarjan, iterative, edges in increasing order;
     * components come out sinks first, so every block sees its dependencies
     * solved).  An inconsistent block fails the seed; a consistent singular
     * one takes its free columns = 0 (the header's seed rule). */
    if (ncore) {
        int32_t *tidx = (int32_t *)malloc(cnt * sizeof(int32_t));
        int32_t *tlow = (int32_t *)malloc(cnt * sizeof(int32_t));
        int32_t *tstk = (int32_t *)malloc(cnt * sizeof(int32_t));
        int32_t *cstk = (int32_t *)malloc(cnt * sizeof(int32_t));
        uint8_t *cpos = (uint8_t *)malloc(cnt);
        uint8_t *onst = (uint8_t *)calloc(cnt, 1);
        int32_t *members = (int32_t *)malloc(cnt * sizeof(int32_t));
        int32_t *col_of = (int32_t *)malloc(cnt * sizeof(int32_t));
        int32_t *pivrow = (int32_t *)malloc(cnt * sizeof(int32_t));
        int fail = 0, counter = 0, sp = 0;
        for (uint32_t k = 0; k < cnt; k++) { tidx[k] = -1; col_of[k] = -1; }
        /* successor i (0..2) of core edge k: owner of e_k[i] when that vertex is
         * another edge's hinge */
#define BO_SUCC(k, i) ((e[3 * (k) + (i)] != (uint32_t)hinge[k] && vowner[e[3 * (k) + (i)]] >= 0) ? vowner[e[3 * (k) + (i)]] : -1)
        for (uint32_t r0 = 0; r0 < cnt && !fail; r0++) {
            if (round_of[r0] >= 0 || tidx[r0] >= 0) continue;
            int csp = 0;
            cstk[csp] = (int32_t)r0; cpos[csp] = 0; csp++;
            tidx[r0] = tlow[r0] = counter++; tstk[sp++] = (int32_t)r0; onst[r0] = 1;
            while (csp && !fail) {
                const int32_t k = cstk[csp - 1];
                if (cpos[csp - 1] < 3) {
                    const int32_t w = BO_SUCC(k, cpos[csp - 1]);
                    cpos[csp - 1]++;
                    if (w < 0) continue;
                    if (tidx[w] < 0) {
                        tidx[w] = tlow[w] = counter++; tstk[sp++] = w; onst[w] = 1;
                        cstk[csp] = w; cpos[csp] = 0; csp++;
                    } else if (onst[w] && tidx[w] < tlow[k]) {
                        tlow[k] = tidx[w];
                    }
                    continue;
                }
                csp--;
                if (csp && tlow[k] < tlow[cstk[csp - 1]]) tlow[cstk[csp - 1]] = tlow[k];
                if (tlow[k] != tidx[k]) continue;
                /* pop one component: members in stack order */
                int sz = 0;
                for (;;) {
                    const int32_t w = tstk[--sp];
                    onst[w] = 0;
                    members[sz++] = w;
                    if (w == k) break;
                }
                /* columns (and rows) in increasing edge order */
                qsort(members, sz, sizeof(int32_t), cmp_i32);
                for (int i = 0; i < sz; i++) col_of[members[i]] = i;
                /* dense block: rows/cols = members (col i = hinge of members[i]) */
                const int W = (sz + 1 + 63) / 64;
                uint64_t *m1 = (uint64_t *)calloc((size_t)sz * W, 8), *m2 = (uint64_t *)calloc((size_t)sz * W, 8);
                for (int r = 0; r < sz; r++) {
                    const uint32_t kk = (uint32_t)members[r];
                    uint32_t rhs_sub = 0;
                    int h = 0;
                    while (e[3 * kk + h] != (uint32_t)hinge[kk]) h++;
                    for (int i = 0; i < 3; i++) {
                        const uint32_t v = e[3 * kk + i];
                        const int32_t o = vowner[v];
                        if (o >= 0 && col_of[o] >= 0) {  /* a hinge of this block */
                            const int c = col_of[o];
                            gf3_add(&m1[(size_t)r * W + (c >> 6)], &m2[(size_t)r * W + (c >> 6)], 1ULL << (c & 63), 0);
                        } else {
                            rhs_sub += xval[v];
                        }
                    }
                    const uint32_t rhs = ((uint32_t)h + 6 - rhs_sub % 3) % 3;
                    if (rhs == 1) m1[(size_t)r * W + (sz >> 6)] |= 1ULL << (sz & 63);
                    if (rhs == 2) m2[(size_t)r * W + (sz >> 6)] |= 1ULL << (sz & 63);
                }
                /* reduced row echelon form: column c takes the first row at or
                 * below `pr` with a nonzero there (swapped up, scaled to 1,
                 * eliminated from every other row); a column with none is free */
                int pr = 0;
                for (int c = 0; c < sz; c++) {
                    const int wc = c >> 6;
                    const uint64_t bit = 1ULL << (c & 63);
                    int p = pr;
                    while (p < sz && !((m1[(size_t)p * W + wc] | m2[(size_t)p * W + wc]) & bit)) p++;
                    if (p == sz) { pivrow[c] = -1; continue; }
                    if (p != pr)
                        for (int w2 = 0; w2 < W; w2++) {
                            uint64_t t = m1[(size_t)p * W + w2]; m1[(size_t)p * W + w2] = m1[(size_t)pr * W + w2]; m1[(size_t)pr * W + w2] = t;
                            t = m2[(size_t)p * W + w2]; m2[(size_t)p * W + w2] = m2[(size_t)pr * W + w2]; m2[(size_t)pr * W + w2] = t;
                        }
                    if (m2[(size_t)pr * W + wc] & bit)
                        for (int w2 = 0; w2 < W; w2++) {
                            const uint64_t t = m1[(size_t)pr * W + w2]; m1[(size_t)pr * W + w2] = m2[(size_t)pr * W + w2]; m2[(size_t)pr * W + w2] = t;
                        }
                    for (int r = 0; r < sz; r++) {
                        if (r == pr) continue;
                        const uint64_t f1 = m1[(size_t)r * W + wc] & bit, f2 = m2[(size_t)r * W + wc] & bit;
                        if (!f1 && !f2) continue;
                        for (int w2 = 0; w2 < W; w2++) {
                            const uint64_t y1 = f1 ? m2[(size_t)pr * W + w2] : m1[(size_t)pr * W + w2];
                            const uint64_t y2 = f1 ? m1[(size_t)pr * W + w2] : m2[(size_t)pr * W + w2];
                            gf3_add(&m1[(size_t)r * W + w2], &m2[(size_t)r * W + w2], y1, y2);
                        }
                    }
                    pivrow[c] = pr++;
                }
                /* rows without a pivot are 0 = rhs: the block is solvable iff
                 * every such rhs is 0 (GOV:428 "unsolvable" otherwise) */
                {
                    const uint64_t bit = 1ULL << (sz & 63);
                    const int wn = sz >> 6;
                    for (int r = pr; r < sz; r++)
                        if ((m1[(size_t)r * W + wn] | m2[(size_t)r * W + wn]) & bit) fail = 1;
                    if (fail) stat_add(2);
                    else if (pr < sz) stat_add(4);
                    if (!fail)
                        for (int c = 0; c < sz; c++) {
                            const int q = pivrow[c];  /* free column: 0 */
                            xval[hinge[members[c]]] = q < 0 ? 0 : (m1[(size_t)q * W + wn] & bit) ? 1 : (m2[(size_t)q * W + wn] & bit) ? 2 : 0;
                        }
                }
                for (int i = 0; i < sz; i++) col_of[members[i]] = -1;
                free(m1); free(m2);
            }
        }
#undef BO_SUCC
        free(tidx); free(tlow); free(tstk); free(cstk); free(cpos); free(onst); free(members); free(col_of); free(pivrow);
        if (fail) return 1;
    }
    /* 4. peeled edges, last round first */
    for (int r = rounds - 1; r >= 0; r--)
        for (uint32_t k = 0; k < cnt; k++) {
            if (round_of[k] != r) continue;
            int h = 0;
            while (e[3 * k + h] != (uint32_t)hinge[k]) h++;
            uint32_t s = 0, coef = 0;
            for (int i = 0; i < 3; i++) {
                if (e[3 * k + i] == (uint32_t)hinge[k]) coef++;
                else s += xval[e[3 * k + i]];
            }
            const uint32_t rhs = ((uint32_t)h + 6 - s) % 3;
            xval[hinge[k]] = (uint8_t)(coef == 1 ? rhs : (2 * rhs) % 3);  /* 2^-1 = 2 in F3 */
        }
    for (uint32_t k = 0; k < cnt; k++) vals[hinge[k]] = xval[hinge[k]] ? xval[hinge[k]] : 3;
    return 0;
}

/* Scratch words needed by solve_bucket for a bucket of cnt keys, nv vertices. */
static size_t solve_ws_words(uint32_t cnt, uint32_t nv) {
    return (size_t)14 * cnt + 6 * (size_t)nv + 64;  /* 12 cnt + 4.5 nv + 1 used */
}

int bo_gov_build(const uint64_t *sig_in, uint64_t n, uint32_t sig_width, uint64_t *E, uint64_t *values,
                 uint64_t values_words, uint64_t *signatures, uint64_t sig_words) {
    const uint64_t m = bo_num_buckets(n);
    uint64_t *sig = (uint64_t *)malloc((n ? n : 1) * 16);
    memcpy(sig, sig_in, n * 16);
    qsort(sig, n, 16, cmp_sig);
    for (uint64_t i = 1; i < n; i++)
        if (sig[2 * i] == sig[2 * i - 2] && sig[2 * i + 1] == sig[2 * i - 1]) { free(sig); return -1; }
    /* A6: bucket histogram -> E low 56 bits (bucket is monotone in sig0) */
    memset(E, 0, (m + 1) * sizeof *E);
    for (uint64_t i = 0; i < n; i++) E[bo_bucket(sig[2 * i], m) + 1]++;
    for (uint64_t b = 0; b < m; b++) E[b + 1] += E[b];
    memset(values, 0, values_words * 8);
    uint32_t maxc = 0;
    for (uint64_t b = 0; b < m; b++) if (E[b + 1] - E[b] > maxc) maxc = (uint32_t)(E[b + 1] - E[b]);
    const uint32_t maxnv = (uint32_t)(bo_vertex_offset(E[m]) + 2);
    int32_t *ws = (int32_t *)malloc(solve_ws_words(maxc + 1, maxnv + 1) * 4 + 64);
    uint8_t *vals = (uint8_t *)malloc(maxnv + 1);
    int rc = 0;
    for (uint64_t b = 0; b < m && !rc; b++) {
        const uint64_t lo = E[b] & (~0ULL >> 8), hi = E[b + 1] & (~0ULL >> 8);
        const uint64_t vo = bo_vertex_offset(lo);
        const uint32_t nv = (uint32_t)(bo_vertex_offset(hi) - vo);
        uint64_t j = 0;
        for (; j < 256; j++)
            if (!solve_bucket(sig + 2 * lo, (uint32_t)(hi - lo), nv, j << 56, vals, ws)) break;
        if (j == 256) { rc = -2; break; }
        E[b] |= j << 56;
        for (uint32_t v = 0; v < nv; v++) values[(vo + v) >> 5] |= (uint64_t)vals[v] << (2 * ((vo + v) & 31));
    }
    free(ws);
    free(vals);
    if (!rc && sig_width) {
        /* A11: signatures[rank] = sig0 & mask (GOV:492-508) */
        memset(signatures, 0, sig_words * 8);
        bo_mph mp = {n, 2 * m, 0, m, E, values, 0, NULL};
        const uint64_t mask = sig_width == 64 ? ~0ULL : (1ULL << sig_width) - 1;
        for (uint64_t i = 0; i < n; i++) {
            const int64_t r = bo_lookup_nocheck(&mp, sig + 2 * i);
            bo_bitlist_set(signatures, (uint64_t)r, sig_width, sig[2 * i] & mask);
        }
    }
    free(sig);
    return rc;
}

/* Batch lookup with or without the checksum test. */
void bo_lookup_batch(const bo_mph *m, const uint64_t *sig, uint64_t n, int check, int64_t *out) {
    for (uint64_t i = 0; i < n; i++) out[i] = check ? bo_lookup(m, sig + 2 * i) : bo_lookup_nocheck(m, sig + 2 * i);
}

/* ---- threaded forms (CPU full-build baseline; same results) -------------- */
typedef struct {
    int kind;  /* 0 hash13, 1 lookups, 2 bucket counts, 3 scatter, 4 solve, 5 sign */
    const uint8_t *keys; uint32_t key_len; uint64_t seed;
    const uint64_t *sig; uint64_t lo, hi; uint64_t *out64; int64_t *outi; int check;
    const bo_mph *mp; uint64_t m; uint32_t *local; uint64_t *cursor; uint64_t *sorted;
    uint64_t *E; uint64_t *values; int32_t *ws; uint8_t *vals; int rc;
    uint32_t width; uint64_t *sigs;
    uint64_t b0, e0;  /* range build: first bucket, keys before it */
} gv_job;

static void run_jobs(gv_job *jobs, int threads, void *(*fn)(void *)) {
    pthread_t tid[256];
    for (int t = 0; t < threads; t++) pthread_create(&tid[t], NULL, fn, &jobs[t]);
    for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
}

static void *gv_worker(void *arg) {
    gv_job *j = (gv_job *)arg;
    uint64_t t4[4];
    switch (j->kind) {
    case 0:
        for (uint64_t i = j->lo; i < j->hi; i++) {
            bo_spooky_short(j->keys + i * j->key_len, j->key_len, j->seed, t4);
            j->out64[2 * i] = t4[0];
            j->out64[2 * i + 1] = t4[1];
        }
        break;
    case 1:
        for (uint64_t i = j->lo; i < j->hi; i++)
            j->outi[i] = j->check ? bo_lookup(j->mp, j->sig + 2 * i) : bo_lookup_nocheck(j->mp, j->sig + 2 * i);
        break;
    case 2:
        for (uint64_t i = j->lo; i < j->hi; i++) j->local[bo_bucket(j->sig[2 * i], j->m) - j->b0]++;
        break;
    case 3:
        for (uint64_t i = j->lo; i < j->hi; i++) {
            const uint64_t p = j->cursor[bo_bucket(j->sig[2 * i], j->m) - j->b0]++;
            j->sorted[2 * p] = j->sig[2 * i];
            j->sorted[2 * p + 1] = j->sig[2 * i + 1];
        }
        break;
    case 4:  /* buckets [lo, hi): sort, duplicate check, solve (GOV:405-440) */
        for (uint64_t b = j->lo; b < j->hi && !j->rc; b++) {
            const uint64_t glo = j->E[b] & (~0ULL >> 8), ghi = j->E[b + 1] & (~0ULL >> 8);
            const uint64_t lo = glo - j->e0, hi = ghi - j->e0;  /* positions in the range's sorted array */
            qsort(j->sorted + 2 * lo, hi - lo, 16, cmp_sig);
            for (uint64_t i = lo + 1; i < hi; i++)
                if (j->sorted[2 * i] == j->sorted[2 * i - 2] && j->sorted[2 * i + 1] == j->sorted[2 * i - 1]) j->rc = -1;
            if (j->rc) break;
            const uint64_t vo = bo_vertex_offset(glo);
            const uint32_t nv = (uint32_t)(bo_vertex_offset(ghi) - vo);
            uint64_t s = 0;
            for (; s < 256; s++)
                if (!solve_bucket(j->sorted + 2 * lo, (uint32_t)(hi - lo), nv, s << 56, j->vals, j->ws)) break;
            if (s == 256) { j->rc = -2; break; }
            j->E[b] |= s << 56;  /* (E[b+1]'s offset bits are all another range reads) */
            for (uint32_t v = 0; v < nv; v++)
                if (j->vals[v]) __atomic_fetch_or(&j->values[(vo + v) >> 5], (uint64_t)j->vals[v] << (2 * ((vo + v) & 31)), __ATOMIC_RELAXED);
        }
        break;
    case 5: {
        const uint64_t mask = j->width == 64 ? ~0ULL : (1ULL << j->width) - 1;
        for (uint64_t i = j->lo; i < j->hi; i++) {
            const uint64_t r = (uint64_t)bo_lookup_nocheck(j->mp, j->sorted + 2 * i);
            const uint64_t v = j->sorted[2 * i] & mask, bit = r * j->width, w = bit >> 6;
            const unsigned off = (unsigned)(bit & 63);
            if (v) {
                __atomic_fetch_or(&j->sigs[w], v << off, __ATOMIC_RELAXED);
                if (off + j->width > 64) __atomic_fetch_or(&j->sigs[w + 1], v >> (64 - off), __ATOMIC_RELAXED);
            }
        }
        break;
    }
    }
    return NULL;
}

static int clamp_threads(int threads) { return threads < 1 ? 1 : threads > 256 ? 256 : threads; }

void bo_hash_fixed_mt(const uint8_t *keys, uint32_t key_len, uint64_t n, uint64_t seed, uint64_t *sig, int threads) {
    threads = clamp_threads(threads);
    gv_job jobs[256];
    for (int t = 0; t < threads; t++)
        jobs[t] = (gv_job){.kind = 0, .keys = keys, .key_len = key_len, .seed = seed, .lo = n * t / threads,
                           .hi = n * (t + 1) / threads, .out64 = sig};
    run_jobs(jobs, threads, gv_worker);
}

void bo_lookup_batch_mt(const bo_mph *mp, const uint64_t *sig, uint64_t n, int check, int64_t *out, int threads) {
    threads = clamp_threads(threads);
    gv_job jobs[256];
    for (int t = 0; t < threads; t++)
        jobs[t] = (gv_job){.kind = 1, .sig = sig, .lo = n * t / threads, .hi = n * (t + 1) / threads, .outi = out,
                           .check = check, .mp = mp};
    run_jobs(jobs, threads, gv_worker);
}

/* The build of buckets [b_lo, b_hi) of a GOV structure over n_global keys
 * from the n_local signatures of that range (any order), e_lo = keys in the
 * buckets below b_lo: writes E[b_lo..b_hi) (E[m] too when b_hi == m), the
 * range's 2-bit fields and checksum fields into FULL-size arrays the caller
 * zeroed (fields of different ranges are disjoint bits, so the ranges' arrays
 * add up to the whole build).  The restatement of bsdb_dev_gov_build_range. */
int bo_gov_build_range_mt(const uint64_t *sig, uint64_t n_local, uint64_t n_global, uint64_t b_lo, uint64_t b_hi,
                          uint64_t e_lo, uint32_t sig_width, uint64_t *E, uint64_t *values, uint64_t *signatures,
                          int threads) {
    threads = clamp_threads(threads);
    const uint64_t m = bo_num_buckets(n_global), nb = b_hi - b_lo, n = n_local;
    gv_job jobs[256];
    uint64_t *sorted = (uint64_t *)malloc((n ? n : 1) * 16);
    uint32_t *local = (uint32_t *)calloc((size_t)threads * (nb + 1), 4);
    uint64_t *cursor = (uint64_t *)malloc((size_t)threads * (nb + 1) * 8);
    /* A6 histogram of the range, per thread slice (bucket b at b - b_lo) */
    for (int t = 0; t < threads; t++)
        jobs[t] = (gv_job){.kind = 2, .sig = sig, .lo = n * t / threads, .hi = n * (t + 1) / threads, .m = m,
                           .b0 = b_lo, .local = local + (size_t)t * (nb + 1)};
    run_jobs(jobs, threads, gv_worker);
    uint64_t acc = 0;
    for (uint64_t i = 0; i < nb; i++) {
        E[b_lo + i] = e_lo + acc;
        for (int t = 0; t < threads; t++) {
            cursor[(size_t)t * (nb + 1) + i] = acc;
            acc += local[(size_t)t * (nb + 1) + i];
        }
    }
    E[b_hi] = e_lo + acc;  /* the next range's offset (cleared below unless b_hi == m) */
    for (int t = 0; t < threads; t++)
        jobs[t] = (gv_job){.kind = 3, .sig = sig, .lo = n * t / threads, .hi = n * (t + 1) / threads, .m = m,
                           .b0 = b_lo, .cursor = cursor + (size_t)t * (nb + 1), .sorted = sorted};
    run_jobs(jobs, threads, gv_worker);
    uint32_t maxc = 0;
    for (uint64_t i = 0; i < nb; i++) {
        const uint64_t c = (E[b_lo + i + 1] & (~0ULL >> 8)) - (E[b_lo + i] & (~0ULL >> 8));
        if (c > maxc) maxc = (uint32_t)c;
    }
    free(local);
    free(cursor);
    const uint32_t maxnv = (uint32_t)(bo_vertex_offset(maxc) + 4);
    uint64_t b0 = b_lo;
    for (int t = 0; t < threads; t++) {
        uint64_t b1 = b0;
        const uint64_t target = e_lo + n * (t + 1) / threads;
        while (b1 < b_hi && (t == threads - 1 || E[b1] < target)) b1++;
        jobs[t] = (gv_job){.kind = 4, .lo = b0, .hi = b1, .E = E, .values = values, .sorted = sorted, .e0 = e_lo,
                           .ws = (int32_t *)malloc(solve_ws_words(maxc + 1, maxnv + 1) * 4 + 64),
                           .vals = (uint8_t *)malloc(maxnv + 1)};
        b0 = b1;
    }
    run_jobs(jobs, threads, gv_worker);
    int rc = 0;
    for (int t = 0; t < threads; t++) {
        if (jobs[t].rc == -1 || (jobs[t].rc && !rc)) rc = jobs[t].rc;
        free(jobs[t].ws);
        free(jobs[t].vals);
    }
    if (!rc && sig_width) {
        bo_mph mp = {n_global, 2 * m, 0, m, E, values, 0, NULL};
        for (int t = 0; t < threads; t++)
            jobs[t] = (gv_job){.kind = 5, .lo = n * t / threads, .hi = n * (t + 1) / threads, .mp = &mp,
                               .sorted = sorted, .width = sig_width, .sigs = signatures};
        run_jobs(jobs, threads, gv_worker);
    }
    if (b_hi < m) E[b_hi] = 0;
    free(sorted);
    return rc;
}

int bo_gov_build_mt(const uint64_t *sig, uint64_t n, uint32_t sig_width, uint64_t *E, uint64_t *values,
                    uint64_t values_words, uint64_t *signatures, uint64_t sig_words, int threads, double *seconds) {
    const double t0 = now_s();
    const uint64_t m = bo_num_buckets(n);
    memset(values, 0, values_words * 8);
    if (sig_width) memset(signatures, 0, sig_words * 8);
    const int rc = bo_gov_build_range_mt(sig, n, n, 0, m, 0, sig_width, E, values, signatures, threads);
    if (seconds) *seconds = now_s() - t0;
    return rc;
}
