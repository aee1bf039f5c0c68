/*
 * bsdb_mi355x.h -- C ABI of the MI355X index-build hot path for bsdb.
 *
 * This is the boundary a JNI shim binds: plain pointers and
 * sizes, no JNI/torch types, int return codes (0 or a negative errno-style
 * code, mirroring src/main/c/native.c:29-34,54 where negative returns become
 * Java exceptions).  Reference paths below are relative to yc-huang/bsdb:
 *   W    = src/main/java/tech/bsdb/write/BSDBWriter.java
 *   CBHS = src/main/java/it/unimi/dsi/sux4j/io/ConcurrentBucketedHashStore.java
 *   GOV  = src/main/java/it/unimi/dsi/sux4j/mph/GOVMinimalPerfectHashFunctionModified.java
 *
 * Two families of entry points:
 *   bsdb_dev_*  operate on DEVICE pointers (HBM-resident keys) on a caller
 *               stream (hipStream_t passed as void*; NULL = the HIP null stream).
 *               Asynchronous: they enqueue and return.
 *   bsdb_*      (no dev_) take HOST pointers (a Java DirectByteBuffer / LBuffer
 *               address), stream them through the context's device staging
 *               buffers and return when the result is in host memory.
 *
 * Key layouts (W:75 put(byte[] key, ...) keys are 1..255 bytes, Common.java MAX_KEY_SIZE):
 *   fixed  n keys of key_len bytes, packed back to back (no padding).
 *   var    a byte blob of blob_bytes plus offsets[n+1] (u64); key i = blob[off[i] .. off[i+1]).
 *          No read goes past blob_bytes.
 *
 * Thread safety: calls on one context are serialised by the context.  put()
 * is concurrent in the reference (W:75, Builder.java:144-160); callers batch
 * per thread and submit through one context or one context per thread.
 */
#ifndef BSDB_MI355X_H
#define BSDB_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BSDB_ABI_VERSION 1

/* Return codes (negative errno-style). */
#define BSDB_OK          0
#define BSDB_EINVAL    (-22)  /* bad argument (null pointer, key_len 0/255+, n too large) */
#define BSDB_ENOMEM    (-12)  /* device allocation failed                                  */
#define BSDB_EIO        (-5)  /* HIP runtime / kernel launch error                         */
#define BSDB_ENODEV    (-19)  /* no such HIP device                                        */
#define BSDB_EDUP      (-17)  /* duplicate 128-bit signature (CBHS:969-972, GOV:471-473)   */
#define BSDB_ESEEDS    (-34)  /* a bucket exhausted its 255 local seeds (GOV:431)          */

typedef struct bsdb_ctx bsdb_ctx;

int         bsdb_abi_version(void);
const char *bsdb_strerror(int code);

/* Opens a context on HIP device `device` (like Native.loadHash returning an
 * mph* as a jlong, native.c:50-59; unlike it, there is a matching close). */
int bsdb_open(int device, bsdb_ctx **out);
int bsdb_close(bsdb_ctx *ctx);

/* GOV:281,350-351 -- numBuckets = n/1500 + 1; multiplier = 2*numBuckets. */
uint64_t bsdb_num_buckets(uint64_t n);

/* ---------------------------------------------------------------------------
 * A3: per-key SpookyHash-short signature (sig0, sig1) = Hashes.spooky4(key, seed)
 * (CBHS:360-364 add(); in-tree C spec spooky.c:94-175).  d_sig receives 2n u64
 * (sig0, sig1 interleaved).  seed is the store seed (0 for BSDBWriter, CBHS:209).
 * ------------------------------------------------------------------------- */
int bsdb_dev_hash_fixed(bsdb_ctx *ctx, const uint8_t *d_keys, uint32_t key_len, uint64_t n,
                        uint64_t seed, uint64_t *d_sig, void *stream);
int bsdb_dev_hash_var(bsdb_ctx *ctx, const uint8_t *d_blob, uint64_t blob_bytes,
                      const uint64_t *d_offsets, uint64_t n, uint64_t seed, uint64_t *d_sig,
                      void *stream);

/* ---------------------------------------------------------------------------
 * A3+A4+A6 fused: hash -> bucket = multiplyHigh(sig0>>>1, 2*num_buckets)
 * (CBHS:900,965; GOV:559) -> bucket-occupancy histogram, ACCUMULATED into
 * d_counts[num_buckets] (u32).  Nothing per key is materialised in HBM beyond
 * a 2-byte partition id stream kept in the context workspace.  This is the
 * replacement for the producer loop GOV:385-402 (edgeOffsetAndSeed[b+1] =
 * edgeOffsetAndSeed[b] + bucket.size()).  Calling it once per key shard and
 * summing d_counts across devices (RCCL all-reduce) gives the global histogram.
 * ------------------------------------------------------------------------- */
int bsdb_dev_histogram_fixed(bsdb_ctx *ctx, const uint8_t *d_keys, uint32_t key_len, uint64_t n,
                             uint64_t seed, uint64_t num_buckets, uint32_t *d_counts, void *stream);
int bsdb_dev_histogram_var(bsdb_ctx *ctx, const uint8_t *d_blob, uint64_t blob_bytes,
                           const uint64_t *d_offsets, uint64_t n, uint64_t seed,
                           uint64_t num_buckets, uint32_t *d_counts, void *stream);

/* A6: E[0] = 0, E[b+1] = E[b] + counts[b] (GOV:391-393), u64, m+1 entries.
 * The low 56 bits of edgeOffsetAndSeed; seeds are OR-ed in by the solver. */
int bsdb_dev_edge_offsets(bsdb_ctx *ctx, const uint32_t *d_counts, uint64_t num_buckets,
                          uint64_t *d_E, void *stream);

/* ---------------------------------------------------------------------------
 * MPHF evaluation over a solved GOV structure (sux4j layout, GOV:292-313):
 *   d_E       edgeOffsetAndSeed[num_buckets+1] (offset | local seed << 56)
 *   d_values  the 2-bit value array (LongArrayBitVector words, LSB first)
 *   d_sigbits the hash.checksum.bits list (width bits per rank), or NULL when width = 0
 * A12 (GOV:557-569, mph.c:86-96): out[i] = rank of signature i, or -1 when the
 * rank is >= n or the checksum bits differ (check != 0); check == 0 returns the
 * unchecked rank (GOV:573-580).
 * A11 (GOV:492-508): OR-s sig0 & mask(width) into d_sigbits at each key's rank
 * (d_sigbits zeroed by the caller, ceil(n*width/64)+1 words).
 * A13 (W:129-145): for records whose rank lies in [start, start+len):
 * index[rank-start] = byte-reversed addr (REVERSE_ORDER, Common.java:61); with
 * d_index_a, also the first min(value_len, 8) bytes of value8 (index.approximate).
 * ------------------------------------------------------------------------- */
int bsdb_dev_lookup(bsdb_ctx *ctx, const uint64_t *d_sig, uint64_t nq, uint64_t n, uint64_t num_buckets,
                    const uint64_t *d_E, const uint64_t *d_values, uint32_t width,
                    const uint64_t *d_sigbits, int check, int64_t *d_out, void *stream);
int bsdb_dev_sign(bsdb_ctx *ctx, const uint64_t *d_sig, uint64_t n, uint64_t num_buckets,
                  const uint64_t *d_E, const uint64_t *d_values, uint32_t width, uint64_t *d_sigbits,
                  void *stream);
int bsdb_dev_index_scatter(bsdb_ctx *ctx, const int64_t *d_rank, const uint64_t *d_addr, uint64_t count,
                           uint64_t start, uint64_t len, uint64_t *d_index, const uint64_t *d_value8,
                           const uint8_t *d_value_len, uint8_t *d_index_a, void *stream);

/* ---------------------------------------------------------------------------
 * A5 + A6 + A8 + A11 on the device: GOV MPHF over n signatures (any order).
 * Buckets are sorted by unsigned (sig0, sig1) (CBHS:939-955), duplicates
 * rejected (BSDB_EDUP, CBHS:969-972), every bucket solved with local seeds
 * 0..255 (BSDB_ESEEDS when exhausted, GOV:431), values written with 3 for a
 * zero hinge (GOV:126-139), and, for width > 0, the checksum list signed
 * (GOV:492-508).  Outputs: d_E[num_buckets+1], d_values[bsdb_values_words(n)],
 * d_sigbits[(n*width+63)/64 + 1] (zeroed here).  The solution choice is this
 * project's deterministic solver (bit-identical to oracle/bo_gov_build), not
 * sux4j's; synchronous (returns after the device finished).
 * ------------------------------------------------------------------------- */
#define BSDB_E2BIG     (-7)   /* a bucket holds more keys than the solver supports */
uint64_t bsdb_values_words(uint64_t n);
int bsdb_dev_gov_build(bsdb_ctx *ctx, const uint64_t *d_sig, uint64_t n, uint32_t width, uint64_t *d_E,
                       uint64_t *d_values, uint64_t *d_sigbits, void *stream);

/* Histogram path selection for bsdb_dev_histogram_* (benchmarks/tests):
 *   0 = auto (partitioned two-pass), 1 = partitioned two-pass, 2 = direct atomics. */
int bsdb_set_histogram_mode(bsdb_ctx *ctx, int mode);
/* Key-load front end (for comparison runs; results are identical):
 * 0 = auto: 13-byte keys by the persistent binned kernel (dword-aligned
 *     16-byte windows), variable-length keys by the persistent binned kernel
 *     with per-wave LDS staging of 128-key groups;
 * 1 = the one-tile-per-workgroup kernel with LDS-staged sub-tiles;
 * 2 = the one-tile-per-workgroup kernel with direct reads. */
int bsdb_set_frontend(bsdb_ctx *ctx, int frontend);
/* Per-chunk key count of the partitioned path (0 = default). */
int bsdb_set_chunk_keys(bsdb_ctx *ctx, uint64_t chunk_keys);
/* Chunks the partitioned path recounted with direct atomics since open
 * because a partition region or LDS bin overflowed (adversarial key sets,
 * e.g. many duplicates).  Synchronises the device.  0 for normal inputs. */
int bsdb_fallback_count(bsdb_ctx *ctx, uint64_t *out);

/* Live per-kernel timing with HIP events recorded on the launch stream around
 * every pass-1 (hash+partition) and pass-2 (partition histogram) launch.
 * bsdb_profile_read synchronises those events and returns, for `kind`
 * (0 = pass 1, 1 = pass 2, 2 = edge-offset scan), the summed milliseconds, the
 * number of launches and the keys they processed; then clears that kind. */
int bsdb_set_profiling(bsdb_ctx *ctx, int enable);
int bsdb_profile_read(bsdb_ctx *ctx, int kind, double *total_ms, uint64_t *launches, uint64_t *keys);

/* ---------------------------------------------------------------------------
 * Host-buffer entry points (what the JNI shim calls with DirectByteBuffer
 * addresses).  Keys are copied H2D through pinned staging in the context;
 * counts are accumulated into the host array h_counts[num_buckets].
 * ------------------------------------------------------------------------- */
int bsdb_histogram_fixed(bsdb_ctx *ctx, const uint8_t *h_keys, uint32_t key_len, uint64_t n,
                         uint64_t seed, uint64_t num_buckets, uint32_t *h_counts);
int bsdb_hash_fixed(bsdb_ctx *ctx, const uint8_t *h_keys, uint32_t key_len, uint64_t n,
                    uint64_t seed, uint64_t *h_sig);
/* Variable-length keys in host memory, as BSDBWriter.put receives them
 * (byte[] of 0..255 bytes, kLen u8, BaseKVWriter.java:44-49): key i is
 * h_blob[h_off[i] .. h_off[i+1]), h_off[0..n] non-decreasing.  Same results
 * as bsdb_dev_{histogram,hash}_var on the same bytes; the keys are copied H2D
 * in batches of <= 256 MiB of key bytes (offsets rebased per batch). */
int bsdb_histogram_var(bsdb_ctx *ctx, const uint8_t *h_blob, const uint64_t *h_off, uint64_t n,
                       uint64_t seed, uint64_t num_buckets, uint32_t *h_counts);
int bsdb_hash_var(bsdb_ctx *ctx, const uint8_t *h_blob, const uint64_t *h_off, uint64_t n,
                  uint64_t seed, uint64_t *h_sig);

/* Synthetic SURVEY.md §8(d) D2 13-byte keys for indices [first, first+n),
 * written on device (benchmark input generator; not part of the build path). */
int bsdb_dev_gen_keys13(bsdb_ctx *ctx, uint64_t first, uint64_t n, uint8_t *d_keys, void *stream);

/* Config C5 synthetic var-len keys: lengths 8..64 drawn
 * Zipf(1.1), bytes 0-7 = i big-endian, splitmix tail.  Writes d_offsets[n+1]
 * (offsets[0] = 0); with d_blob != NULL also the key bytes, after checking
 * offsets[n] <= blob_cap (synchronises).  Bench/test input generator only. */
int bsdb_dev_gen_keys_var(bsdb_ctx *ctx, uint64_t first, uint64_t n, uint64_t *d_offsets, uint8_t *d_blob,
                          uint64_t blob_cap, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* BSDB_MI355X_H */
