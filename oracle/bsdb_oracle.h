/*
 * bsdb_oracle.h -- CPU restatement of bsdb's index-build arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the checker for the MI355X
 * product path (bsdb_amd/csrc) and the CPU baseline leg of bench.py.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may load it.
 * The product path never links or calls it.
 *
 * Parity anchor: every function is checked against the reference's own C
 * (/root/reference/src/main/c/spooky.c, mph.c, compiled by oracle/Makefile
 * into oracle/_ref/) through the fixtures in tests/golden/.
 */
#ifndef BSDB_ORACLE_H
#define BSDB_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* --- A3: SpookyHash V2 "short" as bsdb uses it (spooky.c:94-175). ------- */
void bo_spooky_short(const uint8_t *msg, uint64_t len, uint64_t seed, uint64_t out[4]);
/* --- A9: equation rehash (spooky.c:86-92). ------------------------------ */
void bo_spooky_rehash(const uint64_t sig[2], uint64_t seed, uint64_t out[4]);

/* --- GOV constants / bucket math (GOV:281,315-317,350-351,559). --------- */
uint64_t bo_num_buckets(uint64_t n);                       /* n/1500 + 1            */
uint32_t bo_bucket(uint64_t sig0, uint64_t num_buckets);   /* multiplyHigh(sig0>>>1, 2m) */
uint64_t bo_vertex_offset(uint64_t edge_offset_seed);      /* ((x & 2^56-1)*281)>>8  */
void bo_bucket_batch(const uint64_t *sig /* 2n */, uint64_t n, uint64_t num_buckets, uint32_t *out);
void bo_signature_to_equation(const uint64_t sig[2], uint64_t seed_bits, uint32_t nv,
                              uint32_t e[3]);              /* mph.c:63-71 */
uint64_t bo_count_nonzero_pairs(uint64_t start, uint64_t end, const uint64_t *array);

/* --- Batched restatements used as the GPU parity checker. --------------- */
void bo_hash_fixed(const uint8_t *keys, uint32_t key_len, uint64_t n, uint64_t seed,
                   uint64_t *sig /* 2n */);
void bo_hash_var(const uint8_t *blob, const uint64_t *offsets /* n+1 */, uint64_t n,
                 uint64_t seed, uint64_t *sig /* 2n */);
/* Bucket-occupancy histogram, accumulated into counts[num_buckets]. */
void bo_histogram_fixed(const uint8_t *keys, uint32_t key_len, uint64_t n, uint64_t seed,
                        uint64_t num_buckets, uint32_t *counts);
void bo_histogram_var(const uint8_t *blob, const uint64_t *offsets, uint64_t n, uint64_t seed,
                      uint64_t num_buckets, uint32_t *counts);
/* A6: E[0]=0, E[b+1]=E[b]+counts[b]  (GOV:391-393). */
void bo_edge_offsets(const uint32_t *counts, uint64_t num_buckets, uint64_t *E /* m+1 */);

/* --- Synthetic workload of SURVEY.md §8(d) D2 (13-byte keys). ----------- */
uint64_t bo_splitmix64(uint64_t x);
void bo_gen_keys13(uint64_t first, uint64_t n, uint8_t *out /* 13n */);
void bo_gen_keys13_mt(uint64_t first, uint64_t n, uint8_t *out, int threads);
/* Multi-threaded fused gen+hash+histogram over key indices [first, first+n):
 * the CPU baseline leg.  Returns elapsed seconds. */
double bo_histogram_gen13_mt(uint64_t first, uint64_t n, uint64_t seed, uint64_t num_buckets,
                             uint32_t *counts, int threads);
/* Config C5 keys: key i has length 8 + r, r drawn
 * Zipf(1.1) over 8..64 by inverse CDF on splitmix64(i ^ 0xB5DB0005); bytes
 * 0-7 = i big-endian (BaseTest.java:16-24); tail word w = splitmix64(((i<<3)
 * + w) ^ 0xB5DB0005A5A5A5A5) little-endian.  len() gives the length; gen
 * writes offsets[n+1] (from 0) and, with blob != NULL, the key bytes. */
uint32_t bo_varkey_len(uint64_t i);
void bo_gen_keys_var(uint64_t first, uint64_t n, uint64_t *offsets, uint8_t *blob);
double bo_histogram_genvar_mt(uint64_t first, uint64_t n, uint64_t seed, uint64_t num_buckets, uint32_t *counts,
                              int threads);
/* Multi-threaded histogram over a resident fixed-length key blob. */
double bo_histogram_fixed_mt(const uint8_t *keys, uint32_t key_len, uint64_t n, uint64_t seed,
                             uint64_t num_buckets, uint32_t *counts, int threads);

/* --- A12 lookup over a solved MPHF (GOV:557-580, mph.c:86-96). ---------- */
typedef struct {
    uint64_t n;
    uint64_t multiplier;      /* 2 * num_buckets */
    uint64_t global_seed;
    uint64_t num_buckets;
    const uint64_t *E;        /* edgeOffsetAndSeed, num_buckets + 1 entries */
    const uint64_t *array;    /* 2-bit values */
    uint32_t sig_width;       /* checksum bits (0 = unsigned) */
    const uint64_t *signatures; /* packed sig_width-bit list, LongArrayBitVector layout */
} bo_mph;

int64_t bo_lookup_nocheck(const bo_mph *m, const uint64_t sig[2]);
int64_t bo_lookup(const bo_mph *m, const uint64_t sig[2]);  /* -1 if rejected */
/* Reads element i of a LongArrayBitVector.asLongBigList(width) (LSB-first). */
uint64_t bo_bitlist_get(const uint64_t *words, uint64_t i, uint32_t width);
void bo_bitlist_set(uint64_t *words, uint64_t i, uint32_t width, uint64_t v);

/* --- A5/A8/A11: GOV build (sort, per-bucket solve, sign). --------------- */
/* Builds the MPHF over n signatures.  Outputs:
 *   E[num_buckets+1] (offset | seed<<56), values words (2-bit, ceil(2(V+1)/64)),
 *   signatures words (ceil(n*w/64)) when sig_width > 0.
 * Returns 0, -1 on duplicate signature, -2 on seed exhaustion.
 * The per-bucket solver follows the GOV construction (peel, then F3
 * elimination of the 2-core); its choice among valid solutions is NOT pinned
 * against sux4j 5.4.1 (absent here): see DESIGN.md "parity unpinned". */
/* Solver counters since the last reset (threads summed): attempts (seeds
 * tried), unorientable cores, inconsistent blocks, degenerate edges, singular
 * but consistent blocks solved.  reset != 0 zeroes them after reading. */
void bo_solve_stats(uint64_t out[5], int reset);

int bo_gov_build(const uint64_t *sig /* 2n, any order */, uint64_t n, uint32_t sig_width,
                 uint64_t *E, uint64_t *values, uint64_t values_words,
                 uint64_t *signatures, uint64_t sig_words);
uint64_t bo_values_words(uint64_t n);    /* words of the 2-bit value array */
/* The same build, threads over bucket ranges (identical output: every bucket
 * is solved exactly as by bo_gov_build).  Also the CPU full-build baseline
 * ("port") of bench.py.  Returns as bo_gov_build; *seconds = elapsed. */
int bo_gov_build_mt(const uint64_t *sig, uint64_t n, uint32_t sig_width, uint64_t *E, uint64_t *values,
                    uint64_t values_words, uint64_t *signatures, uint64_t sig_words, int threads, double *seconds);
/* One bucket range [b_lo, b_hi) of a build over n_global keys into zeroed
 * full-size arrays (the multi-GPU build's per-rank step). */
int bo_gov_build_range_mt(const uint64_t *sig, uint64_t n_local, uint64_t n_global, uint64_t b_lo, uint64_t b_hi,
                          uint64_t e_lo, uint32_t sig_width, uint64_t *E, uint64_t *values, uint64_t *signatures,
                          int threads);
/* Threaded lookups (bench / large tests). */
void bo_lookup_batch_mt(const bo_mph *m, const uint64_t *sig, uint64_t n, int check, int64_t *out, int threads);
/* Threaded signatures of 13-byte keys (full-build baseline input). */
void bo_hash_fixed_mt(const uint8_t *keys, uint32_t key_len, uint64_t n, uint64_t seed, uint64_t *sig, int threads);
void bo_lookup_batch(const bo_mph *m, const uint64_t *sig, uint64_t n, int check, int64_t *out);

#ifdef __cplusplus
}
#endif
#endif
