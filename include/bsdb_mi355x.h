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
 * Thread safety: calls on one context are serialised by the context's lock,
 * and the context orders its own work across streams: a call that uses the
 * context's workspace on a stream other than the previous call's first waits
 * (hipStreamWaitEvent) for the previous call's work.  put() is concurrent in
 * the reference (W:75, Builder.java:144-160); callers batch per thread and
 * submit through one shared context or one context per thread.
 *
 * Object handles (all opaque, passed to Java as jlong like native.c:50-59's
 * mph*, but every one has a matching free/close):
 *   bsdb_ctx    one HIP device: stream, workspace, host staging, RCCL rank
 *   bsdb_mph    a GOV MPHF resident on one device (E, 2-bit values, checksum bits)
 *   bsdb_index  the index.db / index_a.db writer of BSDBWriter.buildIndex
 *   bsdb_multi  one context per device of this process + an RCCL communicator
 *   bsdb_builder keys streamed into one device's HBM, built by bucket-range passes
 */
#ifndef BSDB_MI355X_H
#define BSDB_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BSDB_ABI_VERSION 6

/* Return codes (negative errno-style). */
#define BSDB_OK          0
#define BSDB_EINVAL    (-22)  /* bad argument (null pointer, key_len 0 or > 255, n too large) */
#define BSDB_ENOMEM    (-12)  /* device allocation failed                                  */
#define BSDB_EIO        (-5)  /* HIP runtime / kernel launch error                         */
#define BSDB_ENODEV    (-19)  /* no such HIP device                                        */
#define BSDB_EDUP      (-17)  /* duplicate 128-bit signature (CBHS:969-972, GOV:471-473)   */
#define BSDB_ESEEDS    (-34)  /* a bucket exhausted its 255 local seeds (GOV:431)          */
#define BSDB_ECOMM     (-70)  /* RCCL unavailable or a collective failed                   */
#define BSDB_EFILE     (-9)   /* file open/read/write failed (index / dump files)          */
#define BSDB_EVERIFY   (-74)  /* a built MPHF failed its on-device bijection check         */

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

/* F2: the same build, also returning d_rank[i] = the rank (getLong) of d_sig[i],
 * computed inside the solve (E[b] + the hinge vertices before the key's hinge:
 * the lookup's nonzero-pair count, GOV:557-580) -- no lookup pass over the
 * keys is needed to place records in index.db (W:129-145).  The
 * checksum bits are always signed this way (A11 fused into the solve). */
int bsdb_dev_gov_build_ranks(bsdb_ctx *ctx, const uint64_t *d_sig, uint64_t n, uint32_t width, uint64_t *d_E,
                             uint64_t *d_values, uint64_t *d_sigbits, int64_t *d_rank, void *stream);
/* E4: the same build restricted to the buckets [b_lo, b_hi) of a GOV structure
 * over n_global keys (one rank of the multi-GPU build).  d_sig
 * holds exactly the n_local signatures whose bucket lies in the range (any
 * order); e_lo = keys in buckets below b_lo.  d_E (num_buckets(n_global)+1),
 * d_values (bsdb_values_words(n_global)) and d_sigbits ((n_global*width+63)/64
 * + 1) are FULL-size arrays zeroed by the caller; the call writes E[b_lo..b_hi)
 * (plus E[m] on the last range), the 2-bit fields of the range's vertices and
 * the checksum fields of its ranks, and nothing else.  Fields of different
 * ranges are disjoint bits, so summing the ranks' arrays (one RCCL all-reduce
 * or reduce, ncclSum) assembles the global structure.  d_rank (optional):
 * the global rank of each of the n_local signatures, as bsdb_dev_gov_build_ranks. */
int bsdb_dev_gov_build_range(bsdb_ctx *ctx, const uint64_t *d_sig, uint64_t n_local, uint64_t n_global,
                             uint64_t b_lo, uint64_t b_hi, uint64_t e_lo, uint32_t width, uint64_t *d_E,
                             uint64_t *d_values, uint64_t *d_sigbits, int64_t *d_rank, void *stream);
/* E4 with O(n/G) memory per rank (ABI 6): the same range build into windows
 * of the structure instead of full-size arrays.  d_E_win holds E[b_lo..b_hi]
 * (b_hi - b_lo + 1 entries; E[b_hi] is zeroed again unless b_hi == m, as
 * above); d_values_win the value words [values_w0, values_w0 + values_words);
 * d_sigbits_win the checksum words [sig_w0, sig_w0 + sig_words) -- all zeroed
 * by the caller, and covering the words the range writes, which
 * bsdb_gov_range_windows gives as {values_w0, values_words, sig_w0, sig_words}
 * (BSDB_EINVAL otherwise).  A word shared with the next or the previous range
 * holds only this range's bits: the structure is the windows OR-ed at their
 * positions (distributed.py's assembly on rank 0). */
int bsdb_gov_range_windows(uint64_t n_global, uint32_t width, uint64_t e_lo, uint64_t n_local, uint64_t *out4);
int bsdb_dev_gov_build_window(bsdb_ctx *ctx, const uint64_t *d_sig, uint64_t n_local, uint64_t n_global,
                              uint64_t b_lo, uint64_t b_hi, uint64_t e_lo, uint32_t width, uint64_t *d_E_win,
                              uint64_t *d_values_win, uint64_t values_w0, uint64_t values_words,
                              uint64_t *d_sigbits_win, uint64_t sig_w0, uint64_t sig_words, int64_t *d_rank,
                              void *stream);
/* The whole build of a key set resident in this device's HBM (C4: 13.19e9 x
 * 13 B; C5: 4e9 var-len) by sequential bucket-range passes: pass p of P covers
 * buckets [p*m/P, (p+1)*m/P) (the reference's 256 spill segments are such
 * ranges, CBHS:379-395, solved one at a time, CBHS:852-978 / GOV:385-448).
 * Every pass re-hashes all keys and keeps its range's: no signature array for
 * the whole set.  Writes d_E / d_values / d_sigbits (sizes as
 * bsdb_dev_gov_build; zeroed here) and, optionally, index.db's slots
 * (W:129-145): slot rank(key i) = byte-reversed addr(i), addr(i) = d_addr[i]
 * when d_addr != NULL, else addr_base + addr_stride * i (fixed-size records of
 * one data file).  The slots go to d_index[n] (device) or h_index[n] (host
 * memory: each pass's contiguous slice is copied out while the next pass
 * solves) or nowhere when both are NULL.  passes = 0 picks the fewest passes
 * that fit the free HBM; *passes_used (optional) returns the count.  Results
 * equal bsdb_dev_gov_build's on the same keys.  Synchronous. */
int bsdb_dev_mph_build_index_passes_fixed(bsdb_ctx *ctx, const uint8_t *d_keys, uint32_t key_len, uint64_t n,
                                          uint32_t width, uint32_t passes, const uint64_t *d_addr, uint64_t addr_base,
                                          uint64_t addr_stride, uint64_t *d_E, uint64_t *d_values, uint64_t *d_sigbits,
                                          uint64_t *d_index, uint64_t *h_index, uint32_t *passes_used, void *stream);
int bsdb_dev_mph_build_index_passes_var(bsdb_ctx *ctx, const uint8_t *d_blob, uint64_t blob_bytes,
                                        const uint64_t *d_off, uint64_t n, uint32_t width, uint32_t passes,
                                        const uint64_t *d_addr, uint64_t addr_base, uint64_t addr_stride,
                                        uint64_t *d_E, uint64_t *d_values, uint64_t *d_sigbits, uint64_t *d_index,
                                        uint64_t *h_index, uint32_t *passes_used, void *stream);
/* E4 ownership: rank g of `nranks` owns buckets [g*m/nranks, (g+1)*m/nranks)
 * (m = num_buckets; the bucket is monotone in sig0, CBHS:129-138).  Groups the n
 * signatures of d_sig by owning rank into d_out (rank 0's first; order within a
 * rank unspecified) together with one u64 payload per key (the record address
 * of the index stage; d_payload / d_payload_out may be NULL), and writes the
 * per-rank counts to h_counts[nranks] (synchronises). */
int bsdb_dev_partition_owners(bsdb_ctx *ctx, const uint64_t *d_sig, const uint64_t *d_payload, uint64_t n,
                              uint64_t num_buckets, int nranks, uint64_t *d_out, uint64_t *d_payload_out,
                              uint64_t *h_counts, void *stream);
/* Frees the context's grown workspace (histogram id stream, GOV build
 * buffers, host staging): a long-lived context hands its HBM back between
 * builds (the next call grows what it needs again).  Synchronises the device. */
int bsdb_release_workspace(bsdb_ctx *ctx);
/* Debug/test option: after every GOV build, look every key up again on the
 * device and check the ranks form a permutation of [0, n) (BSDB_EVERIFY if not). */
int bsdb_set_verify(bsdb_ctx *ctx, int enable);

/* Histogram path selection for bsdb_dev_histogram_* (benchmarks/tests):
 *   0 = auto, 1 = partitioned two-pass, 2 = direct atomics,
 *   3 = single pass (13-byte keys on a 256-CU device, m <= 9 436 672 buckets,
 *       >= 4 * 256 * 16384 keys, <= 16384 keys per bucket on average: bucket owners per CU, ids exchanged through an
 *       on-die ring; other key sets, and the tail past its whole super-tiles,
 *       take the two-pass path).  Results are identical in every mode. */
int bsdb_set_histogram_mode(bsdb_ctx *ctx, int mode);
/* Key-load front end (for comparison runs; results are identical):
 * 0 = auto: 13-byte keys by the persistent binned kernel (dword-aligned
 *     16-byte windows), variable-length keys by the persistent binned kernel
 *     with per-wave LDS staging of 128-key groups;
 * 1 = the one-tile-per-workgroup kernel with LDS-staged sub-tiles;
 * 2 = the one-tile-per-workgroup kernel with direct reads. */
int bsdb_set_frontend(bsdb_ctx *ctx, int frontend);
/* Two-pass path, 13-byte keys: pass 2 of chunk i runs beside pass 1 of chunk
 * i + 1 (two id buffers; pass 2 keeps `p2_cus` CUs, pass 1 the rest; the
 * first pass 1 and the last pass 2 use the whole chip).  mode -1 = default,
 * 0 = serial chunks, 1 = pipelined; chunks / p2_cus 0 = defaults (8 chunks,
 * CUs / 8).  Results are identical either way. */
int bsdb_set_pipeline(bsdb_ctx *ctx, int mode, uint64_t chunks, uint32_t p2_cus);
/* Per-chunk key count of the partitioned path (0 = default). */
int bsdb_set_chunk_keys(bsdb_ctx *ctx, uint64_t chunk_keys);
/* Chunks the partitioned path recounted with direct atomics since open
 * because a partition region or LDS bin overflowed (adversarial key sets,
 * e.g. many duplicates).  Synchronises the device.  0 for normal inputs. */
int bsdb_fallback_count(bsdb_ctx *ctx, uint64_t *out);
/* Single-pass histogram (mode 3): launches enqueued since open, and those
 * whose bounded waits timed out (a workgroup never became resident; nothing
 * was added and the keys were recounted).  Synchronises the device. */
int bsdb_fused_status(bsdb_ctx *ctx, uint64_t *launches, uint64_t *timeouts);

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

/* ---------------------------------------------------------------------------
 * B4: the one collective of the histogram stage, inside
 * this library.  RCCL is loaded at first use (dlopen librccl.so.1; BSDB_ECOMM
 * when absent).  Per-process ranks (one JVM or one torchrun rank per GPU):
 * rank 0 creates the 128-byte id, the host ships it to the other ranks over
 * its own channel, every rank calls bsdb_comm_init with it.
 * bsdb_dev_histogram_finalize then all-reduces the local counts over xGMI --
 * packed as u16 pairs (m/2 u32 words, 17.6 MB at C4), redone as u32 only if a
 * count does not fit -- and scans them into E[0..m] (every rank the same E);
 * it checks E[m] == n_total (synchronises; BSDB_ECOMM on mismatch).  d_counts
 * holds the global counts afterwards.
 * ------------------------------------------------------------------------- */
#define BSDB_COMM_ID_BYTES 128
/* 1 when this process can load RCCL (every rank should agree on it before
 * bsdb_comm_init, which is collective and waits for every rank), else 0. */
int bsdb_comm_available(void);
int bsdb_comm_unique_id(uint8_t *id /* [BSDB_COMM_ID_BYTES] */);
int bsdb_comm_init(bsdb_ctx *ctx, int nranks, int rank, const uint8_t *id);
int bsdb_dev_histogram_finalize(bsdb_ctx *ctx, uint32_t *d_counts, uint64_t num_buckets, uint64_t n_total,
                                uint64_t *d_E, void *stream);
/* Sum-all-reduce of u64 words on the context's communicator (assembles the
 * disjoint fields of bsdb_dev_gov_build_range outputs; BSDB_ECOMM without one). */
int bsdb_dev_allreduce_u64(bsdb_ctx *ctx, uint64_t *d_buf, uint64_t count, void *stream);

/* ---------------------------------------------------------------------------
 * B4: all the devices of one process (the reference's build runs in ONE JVM,
 * SURVEY.md §2.1), one bsdb_ctx per device and an RCCL communicator over them
 * (ncclCommInitAll, created by the first histogram call; the full build below
 * does not use it).  devices == NULL means 0..ndev-1.  The host-buffer calls
 * shard the keys in input order over the devices (one host thread per device,
 * each copying over its own PCIe link), histogram the shards, all-reduce the
 * counts with ONE collective and return E[0..m] (u64, offsets only) in h_E.
 * ------------------------------------------------------------------------- */
typedef struct bsdb_multi bsdb_multi;
int bsdb_multi_open(int ndev, const int *devices, bsdb_multi **out);
int bsdb_multi_close(bsdb_multi *mc);
int bsdb_multi_size(const bsdb_multi *mc);
int bsdb_multi_ctx(bsdb_multi *mc, int i, bsdb_ctx **out);
int bsdb_multi_histogram_fixed(bsdb_multi *mc, const uint8_t *h_keys, uint32_t key_len, uint64_t n, uint64_t seed,
                               uint64_t *h_E);
int bsdb_multi_histogram_var(bsdb_multi *mc, const uint8_t *h_blob, const uint64_t *h_off, uint64_t n,
                             uint64_t seed, uint64_t *h_E);
/* E4: the whole build over every device of the process --
 * the single-device F2 call bsdb_mph_build_index_* with the key set sharded
 * over the devices.  Device g owns the buckets [g*m/G, (g+1)*m/G) (a sig0
 * range, CBHS:129-138; buckets are independent, GOV:405-448): each device
 * hashes its input-order shard, groups the signatures (and the records' addr /
 * value8 / vlen) by owner, ONE device-to-device exchange delivers them (xGMI
 * peer copies), each owner solves its range (bsdb_dev_gov_build_range, the
 * solve returning every key's rank) and writes its index slots [e_lo, e_lo +
 * n_g) at byte 8*e_lo of index.db (and index_a.db) in writes of <= 128 MiB.
 * Outputs the assembled structure in host arrays sized as bsdb_mph_export's:
 * h_E[num_buckets+1], h_values[bsdb_values_words(n)], h_sigbits[(n*width+63)/64
 * + 1] (NULL when width == 0) -- the fields of
 * GOVMinimalPerfectHashFunctionModified (GOV:284-313); bit-identical to the
 * one-device build, and the index files byte-identical.  index_path NULL: the
 * MPHF only (records ignored).  A device may be listed more than once (the
 * exchange is then a copy within it). */
int bsdb_multi_mph_build_index_fixed(bsdb_multi *mc, const uint8_t *h_keys, uint32_t key_len, uint64_t n,
                                     uint32_t width, const uint64_t *h_addr, const uint64_t *h_value8,
                                     const uint8_t *h_vlen, int approximate, const char *index_path,
                                     const char *index_a_path, uint64_t *h_E, uint64_t *h_values,
                                     uint64_t *h_sigbits);
int bsdb_multi_mph_build_index_var(bsdb_multi *mc, const uint8_t *h_blob, const uint64_t *h_off, uint64_t n,
                                   uint32_t width, const uint64_t *h_addr, const uint64_t *h_value8,
                                   const uint8_t *h_vlen, int approximate, const char *index_path,
                                   const char *index_a_path, uint64_t *h_E, uint64_t *h_values, uint64_t *h_sigbits);

/* ---------------------------------------------------------------------------
 * A14/A15 + F1/F4 from host buffers: a GOV MPHF built on and resident on one
 * device (the Java side fills GOVMinimalPerfectHashFunctionModified's fields
 * from bsdb_mph_export and stores it with BinIO.storeObject, W:99-105;
 * INTEGRATION.md).  Keys as in bsdb_hash_*; seed 0 (CBHS:209).
 *   build     hash -> sort -> solve -> sign (width = hash.checksum.bits)
 *   info      n, num_buckets, width, words of the values / checksum arrays
 *   export    D2H: E[num_buckets+1] (offset | seed << 56), values words,
 *             checksum words (h_sigbits may be NULL when width == 0)
 *   import    H2D of the same arrays (e.g. from a loaded hash.db)
 *   dump/load the raw layout of GOV.dump (GOV:592-619) read by the
 *             reference's own load_mph (mph.c:28-43): native-endian u64
 *             n, multiplier, globalSeed, len(E), E[], len(array), array[];
 *             no checksum bits (load gives width 0)
 *   lookup    getLong (GOV:528-532, 557-569) of host keys: rank or -1
 *             (check != 0: range and checksum test; 0: unchecked rank)
 *   lifetime  an MPHF belongs to its context: bsdb_close releases the
 *             device arrays of the context's live MPHFs, after which their
 *             calls return BSDB_EINVAL and bsdb_mph_free only frees the
 *             handle (either order of bsdb_close / bsdb_mph_free is safe);
 *             close a bsdb_index before its MPHF
 * ------------------------------------------------------------------------- */
typedef struct bsdb_mph bsdb_mph;
int bsdb_mph_build_fixed(bsdb_ctx *ctx, const uint8_t *h_keys, uint32_t key_len, uint64_t n, uint32_t width,
                         bsdb_mph **out);
int bsdb_mph_build_var(bsdb_ctx *ctx, const uint8_t *h_blob, const uint64_t *h_off, uint64_t n, uint32_t width,
                       bsdb_mph **out);
int bsdb_mph_info(const bsdb_mph *mph, uint64_t *n, uint64_t *num_buckets, uint32_t *width, uint64_t *values_words,
                  uint64_t *sig_words);
/* The sizes of an MPHF's fields on n keys with `width` checksum bits, without
 * a device or a handle (ABI 5; bsdb_mph_info returns the same numbers for a
 * built MPHF): num_buckets = n/1500 + 1 (GOV:350; E has num_buckets + 1
 * words, GOV:355); value_bits = 2 (1 + (n 281 >> 8)), the length of GOV's
 * 2-bit value vector with its trailing 0 (GOV:357,483-485), in values_words
 * u64 words; sig_words = ceil(n width / 64) + 1 words for the n width-bit
 * checksums (GOV:494; one zero word of slack), 0 when width == 0.  A JVM
 * sizes the arrays it exports into and wraps them with these
 * (LongArrayBitVector.wrap(values, value_bits)). */
int bsdb_mph_sizes(uint64_t n, uint32_t width, uint64_t *num_buckets, uint64_t *values_words, uint64_t *value_bits,
                   uint64_t *sig_words);
int bsdb_mph_export(bsdb_mph *mph, uint64_t *h_E, uint64_t *h_values, uint64_t *h_sigbits);
int bsdb_mph_import(bsdb_ctx *ctx, uint64_t n, uint32_t width, const uint64_t *h_E, const uint64_t *h_values,
                    const uint64_t *h_sigbits, bsdb_mph **out);
int bsdb_mph_dump(bsdb_mph *mph, const char *path);
int bsdb_mph_load(bsdb_ctx *ctx, const char *path, bsdb_mph **out);
int bsdb_mph_lookup_fixed(bsdb_mph *mph, const uint8_t *h_keys, uint32_t key_len, uint64_t n, int check,
                          int64_t *h_out);
int bsdb_mph_lookup_var(bsdb_mph *mph, const uint8_t *h_blob, const uint64_t *h_off, uint64_t n, int check,
                        int64_t *h_out);
int bsdb_mph_free(bsdb_mph *mph);

/* ---------------------------------------------------------------------------
 * A13 + F2/F3: BSDBWriter.buildIndex (W:107-155, writeLBuffer W:166-179).
 * open: passSize = min(n, pass_cache_bytes / 8) slots, passes = ceil(n /
 *   passSize) (W:112-118); pass_cache_bytes == 0 sizes the pass cache by the
 *   device instead (a quarter of free HBM: one pass up to ~4 G records on an
 *   MI355X; the files are the same, only the number of kv.db scans changes).
 *   Creates/truncates index_path and index_a_path
 *   (the reference creates index_a.db even in exact mode, W:126; with
 *   index_a_path NULL it is not touched).  For each pass the caller feeds
 *   every record of the kv.db scan (KVWriter.forEach, W:134) with
 *   put_{var,fixed}: the key is looked up on the device (getLong, checked),
 *   and a record whose rank r lies in the pass writes the big-endian address
 *   (REVERSE_ORDER, Common.java:61) at slot r - rangeStart and, in approximate
 *   mode, the first min(len, 8) value bytes (value8 little-endian = the byte
 *   order in the record; a shorter value leaves its slot tail zero -- the
 *   reference leaves it unspecified, W:141).  end_pass writes the pass's slots
 *   in writes of <= 128 MiB.  Record buffers: key blob + offsets (or fixed
 *   keys), addr[count], and for approximate mode value8[count] + vlen[count]
 *   (min(value length, 8)).  Uploads are double-buffered on two streams.
 * ------------------------------------------------------------------------- */
typedef struct bsdb_index bsdb_index;

/* F2: the MPHF and index.db (+ index_a.db) in ONE call from
 * records in host memory -- hash -> GOV build whose solve also returns every
 * key's rank (the input position is carried through the bucket sort as the
 * store's payload, CBHS:386-388) -> addr[i] scattered big-endian at slot
 * rank[i] -> files in writes of <= 128 MiB.  No kv.db rescan and no lookup
 * pass: the files are identical to bsdb_index_* passes over the same
 * records (W:107-155).  The whole index lives on the device (8n B, 17n B more
 * in approximate mode); keys, addr[n], value8[n], vlen[n] as for put_*.
 * index_a_path may be NULL in exact mode (otherwise created empty, W:126). */
int bsdb_mph_build_index_fixed(bsdb_ctx *ctx, const uint8_t *h_keys, uint32_t key_len, uint64_t n, uint32_t width,
                               const uint64_t *h_addr, const uint64_t *h_value8, const uint8_t *h_vlen,
                               int approximate, const char *index_path, const char *index_a_path, bsdb_mph **out);
int bsdb_mph_build_index_var(bsdb_ctx *ctx, const uint8_t *h_blob, const uint64_t *h_off, uint64_t n, uint32_t width,
                             const uint64_t *h_addr, const uint64_t *h_value8, const uint8_t *h_vlen, int approximate,
                             const char *index_path, const char *index_a_path, bsdb_mph **out);
/* F2 + F3 in bounded device memory: the same files and MPHF as
 * bsdb_mph_build_index_* from records in host memory, built by sequential
 * bucket-range passes over the keys kept in HBM (the reference's 256-segment
 * spill and segment-by-segment solve, CBHS:379-395,852-978, W:91-155): the
 * keys go to the device once, every pass re-hashes them and solves its range,
 * and each pass's index slots are written at their offset while the next pass
 * solves.  Reaches README-size sets on one device (C4: 13.19e9 x 13 B).
 * Addresses: h_addr[n], or (h_addr NULL) addr_base + addr_stride * i
 * (fixed-size records of one data file).  Addresses/values that do not fit
 * HBM beside the keys are gathered from the caller's arrays in host memory.
 * passes = 0 picks the fewest passes that fit; *passes_used (optional).
 * bsdb_mph_build_index_* take this path themselves when their one-shot build
 * does not fit the free HBM. */
int bsdb_mph_build_index_passes_fixed(bsdb_ctx *ctx, const uint8_t *h_keys, uint32_t key_len, uint64_t n,
                                      uint32_t width, const uint64_t *h_addr, uint64_t addr_base, uint64_t addr_stride,
                                      const uint64_t *h_value8, const uint8_t *h_vlen, int approximate, uint32_t passes,
                                      const char *index_path, const char *index_a_path, bsdb_mph **out,
                                      uint32_t *passes_used);
int bsdb_mph_build_index_passes_var(bsdb_ctx *ctx, const uint8_t *h_blob, const uint64_t *h_off, uint64_t n,
                                    uint32_t width, const uint64_t *h_addr, uint64_t addr_base, uint64_t addr_stride,
                                    const uint64_t *h_value8, const uint8_t *h_vlen, int approximate, uint32_t passes,
                                    const char *index_path, const char *index_a_path, bsdb_mph **out,
                                    uint32_t *passes_used);

/* The same build fed incrementally, as BSDBWriter.put feeds the hash store
 * (W:75-89 -> CBHS:360-395): a builder owns the keys added so far in HBM (and,
 * unless addr_stride != 0 makes the address addr_base + addr_stride * (add
 * order), each record's address -- plus value8/vlen in approximate mode -- in
 * host memory).  key_len 0 = variable-length keys (add_fixed is accepted too);
 * key_capacity / blob_capacity reserve device memory up front (0 = grow on
 * demand).  Adds are synchronous (the caller may reuse its buffers) and may
 * come in any order: the files do not depend on it.  finish builds everything
 * added (index_path NULL: the MPHF only), releases the keys from HBM and
 * returns the MPHF; free releases the builder (after finish or instead of it).
 * A failed add leaves the builder failed (later calls return that code). */
typedef struct bsdb_builder bsdb_builder;
int bsdb_builder_open(bsdb_ctx *ctx, uint32_t key_len, uint64_t key_capacity, uint64_t blob_capacity, int approximate,
                      uint64_t addr_base, uint64_t addr_stride, bsdb_builder **out);
int bsdb_builder_add_fixed(bsdb_builder *b, const uint8_t *h_keys, uint32_t key_len, uint64_t count,
                           const uint64_t *h_addr, const uint64_t *h_value8, const uint8_t *h_vlen);
int bsdb_builder_add_var(bsdb_builder *b, const uint8_t *h_blob, const uint64_t *h_off, uint64_t count,
                         const uint64_t *h_addr, const uint64_t *h_value8, const uint8_t *h_vlen);
int bsdb_builder_count(const bsdb_builder *b, uint64_t *n);
int bsdb_builder_finish(bsdb_builder *b, uint32_t width, uint32_t passes, const char *index_path,
                        const char *index_a_path, bsdb_mph **out, uint32_t *passes_used);
int bsdb_builder_free(bsdb_builder *b);

int bsdb_index_open(bsdb_mph *mph, int approximate, uint64_t pass_cache_bytes, const char *index_path,
                    const char *index_a_path, bsdb_index **out, uint64_t *passes);
int bsdb_index_begin_pass(bsdb_index *ix, uint64_t pass);
int bsdb_index_put_var(bsdb_index *ix, const uint8_t *h_blob, const uint64_t *h_off, uint64_t count,
                       const uint64_t *h_addr, const uint64_t *h_value8, const uint8_t *h_vlen);
int bsdb_index_put_fixed(bsdb_index *ix, const uint8_t *h_keys, uint32_t key_len, uint64_t count,
                         const uint64_t *h_addr, const uint64_t *h_value8, const uint8_t *h_vlen);
int bsdb_index_end_pass(bsdb_index *ix);
int bsdb_index_close(bsdb_index *ix);

/* ---------------------------------------------------------------------------
 * F3: the kv.db scan that feeds buildIndex (W:134, PartitionedKVWriter.forEach
 * PKV:50-70), native: every partition file <kv_base>.<p> (PKV:79-81) is mapped
 * and parsed by a host thread into packed arrays in partition order -- the key
 * blob (+ offsets), each record's address as the reference computes it, the
 * first <= 8 value bytes (LE) and their count (index_a.db, W:140-142).
 * format 0 = SimpleCompactKVWriter (SimpleCompactKVWriter.java:55-70),
 * 1 = SimpleBlockedKVWriter with block_size-byte blocks (BlockedKVWriter.java:
 * 84-136).  threads <= 0: every hardware thread.  Host only (no device).
 * ------------------------------------------------------------------------- */
typedef struct bsdb_kv_records bsdb_kv_records;
int bsdb_kv_scan(const char *kv_base, int partitions, int format, uint32_t block_size, int threads,
                 bsdb_kv_records **out);
/* n records, their key bytes, and fixed_len = the common key length (0 when lengths differ) */
int bsdb_kv_records_info(const bsdb_kv_records *r, uint64_t *n, uint64_t *key_bytes, uint32_t *fixed_len);
/* borrowed pointers, valid until bsdb_kv_records_free: blob, offsets[n+1], addr[n], value8[n], vlen[n] */
int bsdb_kv_records_arrays(const bsdb_kv_records *r, const uint8_t **blob, const uint64_t **offsets,
                           const uint64_t **addr, const uint64_t **value8, const uint8_t **vlen);
int bsdb_kv_records_free(bsdb_kv_records *r);
/* W:91-155 straight from the data files: scan, then bsdb_mph_build_index_*
 * (hash, GOV build, ranks from the solve, index.db / index_a.db). */
int bsdb_kv_build_index(bsdb_ctx *ctx, const char *kv_base, int partitions, int format, uint32_t block_size,
                        int threads, uint32_t width, int approximate, const char *index_path,
                        const char *index_a_path, bsdb_mph **out);

#ifdef __cplusplus
}
#endif
#endif /* BSDB_MI355X_H */
