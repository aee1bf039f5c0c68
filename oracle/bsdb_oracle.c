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

/* GOV:155-162,315-317 -- OFFSET_MASK = 2^56-1, C_TIMES_256 = floor(1.10*256) = 281. */
uint64_t bo_vertex_offset(uint64_t eos) { return ((eos & (~0ULL >> 8)) * 281) >> 8; }

/* mph.c:63-71 (sux4j Linear3SystemSolver.signatureToEquation, GOV:564,577). */
void bo_signature_to_equation(const uint64_t sig[2], uint64_t seed_bits, uint32_t nv, uint32_t e[3]) {
    uint64_t t[4];
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
