// hash_kernels.hip -- the index-build hot path on MI355X (gfx950).
//
// Per key: SpookyHash-short (A3) -> bucket = multiplyHigh(sig0>>>1, 2m) (A4)
// -> bucket-occupancy histogram (A6).  Reference loop being replaced:
// ConcurrentBucketedHashStore.add (CBHS:360-395) + the GOV producer that
// accumulates edgeOffsetAndSeed (GOV:385-402).
//
// Why two passes: m = n/1500+1 buckets (8.8 M at 13 B keys) is a 35 MB
// table, far beyond LDS, and per-key device-scope atomics into it run at the
// memory-side atomic rate (~20 G random adds/s), 20x slower than the key
// stream.  So pass 1 hashes a tile of keys, drops each key's 2-byte
// partition-local id (bucket mod 32768) into an LDS bin of its bucket range,
// and writes the bins out as padded 16-byte runs; pass 2 histograms one
// partition at a time in a 128 KiB LDS table and flushes it with coalesced
// atomics.  Extra traffic is ~4.3 B/key on top of the key bytes.
//
// Pass-1 kernels: k_pass1_d13e (13-byte keys, production), k_pass1_vare
// (variable-length keys, and fixed lengths up to 32 B on computed offsets),
// k_pass1_d13 (13-byte keys past 288 bins), k_pass1 (generic: tails, the
// signature and direct-atomic epilogues, comparison front ends).  DESIGN.md §4.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "spooky_dev.hpp"

namespace bsdb {

constexpr int P1_THREADS = 512;
constexpr int P1_KEYS_PER_THREAD = 16;
constexpr int P1_TILE = P1_THREADS * P1_KEYS_PER_THREAD;  // 8192 keys per workgroup
constexpr int STAGE_BYTES = 26624;                        // 2048 keys x 13 B
constexpr int PART_SHIFT = 15;                            // 32768 buckets per partition
constexpr int PART_BUCKETS = 1 << PART_SHIFT;
constexpr int MAX_PARTS = 512;
constexpr int NCOPY = 8;                                  // cursor/region copies (one per XCD)
constexpr int P2_THREADS = 1024;

enum Epi { EPI_PARTITION = 0, EPI_ATOMIC = 1, EPI_SIG = 2 };
enum Src { SRC_STAGED13 = 0, SRC_STAGED = 1, SRC_FIXED_DIRECT = 2, SRC_VAR = 3, SRC_DIRECT13 = 4, SRC_VARSTAGED = 5 };

struct P1Args {
    const uint8_t *keys;      // fixed: n*key_len bytes; var: blob
    const uint64_t *offsets;  // var only
    uint64_t blob_bytes;      // bytes readable at keys
    uint64_t n;               // keys in this launch
    uint32_t key_len;         // fixed only
    uint64_t seed;
    uint64_t multiplier;      // 2 * num_buckets
    // EPI_PARTITION
    uint16_t *ids;            // [nregions][P][cap]
    uint32_t *cursor;         // [nregions][P] fill of each region
    uint32_t *overflow;       // set when a region would overflow
    uint64_t cap;             // capacity of one (partition, region) slot, multiple of 8
    uint32_t nparts;
    uint32_t nregions;        // regions per partition in the id buffer
    uint32_t region0;         // first region used by k_pass1's NCOPY shared regions
    uint32_t ncopy;           // k_pass1_d13e: region copies (power of 2), copy = tile % ncopy
    uint32_t bin_shift;       // EPI_PARTITION: a key's region bin is bucket >> bin_shift (<= PART_SHIFT);
                              // its 2-byte id stays bucket % 32768 (local to its pass-2 partition)
    uint32_t capb;            // k_pass1_d13e: ids per LDS bin (multiple of 8), nparts*capb <= D13E_BIN_IDS
    // EPI_ATOMIC
    uint32_t *counts;
    // EPI_SIG
    uint64_t *sig;
    // 13-byte kernels: scratch words [0, 2048) unused, [2048, 10240) dummy
    // u16 stores, then 1024 words per workgroup (up to P1_SCRATCH_MAXWG) for
    // the cursor atomics of lanes without a partition
    uint32_t *scratch;
};
constexpr uint32_t P1_SCRATCH_WG = 10240;
constexpr uint32_t P1_SCRATCH_MAXWG = 2048;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2), aligned(8)));
// 16-byte vector with 4-byte alignment: global_load_dwordx4 at a dword-aligned
// address (the 13-byte-key windows of the direct front end).
typedef unsigned int u32x4a __attribute__((ext_vector_type(4), aligned(4)));

// Streaming 16-byte load, read-once data (keys, partition ids): nontemporal so
// the stream does not evict the re-used tables from L2 / Infinity Cache.
__device__ __forceinline__ uint4 ntload16(const void *p) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

// Bounds-checked little-endian u64 read from global memory: dword loads in the
// body, byte loads for the ragged last dword of the blob (never past `limit`).
__device__ __forceinline__ uint32_t gload32(const uint8_t *base, uint64_t limit, uint64_t a) {
    if (a + 4 <= limit) return *reinterpret_cast<const uint32_t *>(base + a);
    uint32_t w = 0;
    for (int b = 0; b < 4; ++b)
        if (a + b < limit) w |= (uint32_t)base[a + b] << (8 * b);
    return w;
}

__device__ __forceinline__ uint64_t gload64(const uint8_t *base, uint64_t limit, uint64_t pos) {
    const uint64_t a = pos & ~3ULL;
    const uint32_t sh = (uint32_t)(pos & 3) * 8;
    if (a + 12 <= limit) {
        const uint32_t *q = reinterpret_cast<const uint32_t *>(base + a);
        return funnel64(q[0], q[1], q[2], sh);
    }
    return funnel64(gload32(base, limit, a), gload32(base, limit, a + 4), gload32(base, limit, a + 8), sh);
}

// Copies bytes [src_lo, src_lo + nbytes) of global memory into LDS starting at
// dword-aligned `stage`, with 16-byte loads where the source is aligned.  The
// caller guarantees src_lo % 16 == 0 for the staged paths (tile starts are
// multiples of 2048 keys: 2048*L bytes, and the key blob is 16-B aligned).
struct StageRegs {
    uint4 v[4];
};

__device__ __forceinline__ void stage_load(StageRegs &r, const uint8_t *src, uint64_t nbytes, int tid) {
    const uint32_t nvec = (uint32_t)(nbytes >> 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t i = tid + j * P1_THREADS;
        if (i < nvec) {
            r.v[j] = ntload16(src + (uint64_t)i * 16);
        } else if (i == nvec && (nbytes & 15)) {
            // ragged end of the chunk: byte loads, never past nbytes
            uint8_t tmp[16];
            for (int b = 0; b < 16; ++b) tmp[b] = (uint64_t)i * 16 + b < nbytes ? src[(uint64_t)i * 16 + b] : 0;
            r.v[j] = *reinterpret_cast<uint4 *>(tmp);
        }
    }
}

__device__ __forceinline__ void stage_store(const StageRegs &r, uint32_t *stage, uint64_t nbytes, int tid) {
    const uint32_t nvec = (uint32_t)((nbytes + 15) >> 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t i = tid + j * P1_THREADS;
        if (i < nvec) reinterpret_cast<uint4 *>(stage)[i] = r.v[j];
    }
}

// Hash of key `k` of the staged sub-tile (byte offset k*L in LDS).
template <int LFIX>
__device__ __forceinline__ void hash_staged(const uint32_t *stage, uint32_t k, uint32_t key_len,
                                            uint64_t seed, uint64_t &s0, uint64_t &s1) {
    const uint32_t L = LFIX ? LFIX : key_len;
    const uint32_t o = k * L;
    if (LFIX == 13) {
        const uint32_t *q = stage + (o >> 2);
        const uint32_t sh = (o & 3) * 8;
        W64 a0, a1;
        spooky13_u(q[0], q[1], q[2], q[3], sh, seed, a0, a1);
        s0 = u64(a0);
        s1 = u64(a1);
    } else {
        auto rd = [&](uint32_t off) -> uint64_t {
            const uint32_t p = o + off;
            const uint32_t *q = stage + (p >> 2);
            return funnel64(q[0], q[1], q[2], (p & 3) * 8);
        };
        spooky_short(rd, L, seed, s0, s1);
    }
}

// Block-wide exclusive scan of one u32 per thread (512 threads).
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *wsum, int tid, uint32_t &total) {
    const int lane = tid & 63, wid = tid >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < P1_THREADS / 64; ++w) {
        const uint32_t s = wsum[w];
        pre += w < wid ? s : 0;
        tot += s;
    }
    total = tot;
    return pre + x - v;
}

// Block-wide exclusive scan of one u32 per thread (NT threads).
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan_n(uint32_t v, uint32_t *wsum, int tid, uint32_t &total) {
    const int lane = tid & 63, wid = tid >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
        const uint32_t s = wsum[w];
        pre += w < wid ? s : 0;
        tot += s;
    }
    total = tot;
    return pre + x - v;
}

// Pass 1: one workgroup = one tile of 8192 consecutive keys.
template <int SRC, int EPI, int KPS, int LFIX>
__global__ __launch_bounds__(P1_THREADS, 4) void k_pass1(P1Args a) {
    // stage (key bytes of one sub-tile) and sorted (the tile's bucket ids in
    // partition order) are never live together: one 32 KiB buffer serves both.
    constexpr int UNION_WORDS = EPI == EPI_PARTITION ? P1_TILE : (STAGE_BYTES + 64) / 4;
    __shared__ __align__(16) uint32_t stage[UNION_WORDS];
    uint32_t *sorted = stage;
    __shared__ uint32_t bkl[EPI == EPI_PARTITION ? P1_TILE : 1];  // bucket of key kt
    __shared__ uint32_t hist[MAX_PARTS], start[MAX_PARTS], run[MAX_PARTS], base[MAX_PARTS];
    __shared__ uint32_t wsum[P1_THREADS / 64];

    const int tid = threadIdx.x;
    const uint64_t tile0 = (uint64_t)blockIdx.x * P1_TILE;
    if (tile0 >= a.n) return;
    const uint32_t tile_n = (uint32_t)min((uint64_t)P1_TILE, a.n - tile0);
    const uint32_t L = LFIX ? LFIX : a.key_len;

    if (EPI == EPI_PARTITION) {
        for (int i = tid; i < MAX_PARTS; i += P1_THREADS) hist[i] = 0;
    }

    const uint32_t mult = (uint32_t)a.multiplier;  // 2m < 2^32 (checked by the C ABI)
    auto emit = [&](uint32_t kt, uint64_t gk, uint64_t s0, uint64_t s1) {
        if (EPI == EPI_SIG) {
            reinterpret_cast<ulonglong2 *>(a.sig)[gk] = make_ulonglong2(s0, s1);
        } else {
            const uint32_t b = bucket_of_w(w64(s0), mult);
            if (EPI == EPI_ATOMIC) {
                atomicAdd(a.counts + b, 1u);
            } else {
                bkl[kt] = b;
                atomicAdd(&hist[b >> a.bin_shift], 1u);
            }
        }
    };

    if (SRC == SRC_DIRECT13) {
        // 13-byte keys without LDS staging: lane t of a wave loads the
        // dword-aligned 16-byte window holding its key (a wave covers 832
        // contiguous bytes, so the loads coalesce into whole lines); all 16
        // windows of a thread are issued before the first hash, keeping
        // 16 KiB per wave in flight with no barrier until the tile epilogue.
        if (EPI == EPI_PARTITION) __syncthreads();
        const bool careful = (tile0 + P1_TILE) * 13 + 3 > a.blob_bytes;  // last tile: bounds-checked
        if (!careful) {
            u32x4a win[P1_KEYS_PER_THREAD];
#pragma unroll
            for (int j = 0; j < P1_KEYS_PER_THREAD; ++j) {
                const uint64_t byte = (tile0 + tid + j * P1_THREADS) * 13;
                win[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4a *>(a.keys + (byte & ~3ULL)));
            }
#pragma unroll
            for (int j = 0; j < P1_KEYS_PER_THREAD; ++j) {
                const uint32_t kt = tid + j * P1_THREADS;
                const uint32_t sh = ((kt * 13u) & 3u) * 8u;  // tile0*13 is a multiple of 4
                W64 s0, s1;
                spooky13_u(win[j].x, win[j].y, win[j].z, win[j].w, sh, a.seed, s0, s1);
                emit(kt, tile0 + kt, u64(s0), u64(s1));
            }
        } else {
            for (int j = 0; j < P1_KEYS_PER_THREAD; ++j) {
                const uint32_t kt = tid + j * P1_THREADS;
                if (kt < tile_n) {
                    const uint64_t pos = (tile0 + kt) * 13;
                    auto rd = [&](uint32_t off) -> uint64_t { return gload64(a.keys, a.blob_bytes, pos + off); };
                    uint64_t s0, s1;
                    spooky_short(rd, 13, a.seed, s0, s1);
                    emit(kt, tile0 + kt, s0, s1);
                }
            }
        }
    } else if (SRC == SRC_STAGED13 || SRC == SRC_STAGED) {
        // sub-tile = P1_THREADS*KPS keys staged through LDS with 16-B loads,
        // next sub-tile prefetched into registers while this one hashes.
        constexpr int SUB = P1_THREADS * KPS;
        constexpr int NSUB = P1_KEYS_PER_THREAD / KPS;
        const uint64_t tile_bytes0 = tile0 * L;
        StageRegs pre;
        auto sub_bytes = [&](int s) -> uint64_t {
            const uint64_t k0 = (uint64_t)s * SUB;
            if (k0 >= tile_n) return 0;
            return (uint64_t)min((uint32_t)SUB, tile_n - (uint32_t)k0) * L;
        };
        stage_load(pre, a.keys + tile_bytes0, sub_bytes(0), tid);
        if (EPI == EPI_PARTITION) __syncthreads();  // hist zeroed
#pragma unroll
        for (int s = 0; s < NSUB; ++s) {
            const uint64_t nb = sub_bytes(s);
            if (s) __syncthreads();  // all reads of the previous sub-tile done
            stage_store(pre, stage, nb, tid);
            __syncthreads();
            if (s + 1 < NSUB) stage_load(pre, a.keys + tile_bytes0 + (uint64_t)(s + 1) * SUB * L, sub_bytes(s + 1), tid);
#pragma unroll
            for (int q = 0; q < KPS; ++q) {
                const uint32_t k = tid + q * P1_THREADS;  // key within sub-tile
                const uint32_t kt = s * SUB + k;           // key within tile
                if (kt < tile_n) {
                    uint64_t s0, s1;
                    hash_staged<LFIX>(stage, k, L, a.seed, s0, s1);
                    emit(kt, tile0 + kt, s0, s1);
                }
            }
        }
    } else if (SRC == SRC_VARSTAGED) {
        // variable-length keys, LDS-staged: sub-tile s = keys [512s, 512s+512)
        // of the tile; its byte range [off[k0], off[k0+cnt]) (rounded down to
        // 16 B) is copied into LDS with coalesced 16-byte loads, the next
        // sub-tile's range prefetched into registers while this one hashes.
        // A sub-tile longer than the stage (mean key > ~63 B) is hashed from
        // global memory instead (uniform branch).
        constexpr uint64_t STAGE_CAP = (uint64_t)UNION_WORDS * 4 - 16;
        auto range = [&](int s, uint64_t &lo, uint64_t &nb) {
            const uint32_t k0 = (uint32_t)s * P1_THREADS;
            if (k0 >= tile_n) { lo = 0; nb = 0; return; }
            const uint32_t cnt = min((uint32_t)P1_THREADS, tile_n - k0);
            lo = a.offsets[tile0 + k0] & ~15ULL;
            nb = a.offsets[tile0 + k0 + cnt] - lo;
        };
        uint64_t lo, nb, nlo, nnb;
        range(0, lo, nb);
        StageRegs pre;
        if (nb <= STAGE_CAP) stage_load(pre, a.keys + lo, nb, tid);
        if (EPI == EPI_PARTITION) __syncthreads();  // hist zeroed
        for (int s = 0; s < P1_KEYS_PER_THREAD; ++s) {
            if ((uint32_t)s * P1_THREADS >= tile_n) break;
            const bool staged = nb <= STAGE_CAP;
            if (s) __syncthreads();  // all reads of the previous sub-tile done
            if (staged) stage_store(pre, stage, nb, tid);
            __syncthreads();
            range(s + 1, nlo, nnb);
            if (s + 1 < P1_KEYS_PER_THREAD && nnb <= STAGE_CAP) stage_load(pre, a.keys + nlo, nnb, tid);
            const uint32_t kt = s * P1_THREADS + tid;
            if (kt < tile_n) {
                const uint64_t gk = tile0 + kt;
                const uint64_t pos = a.offsets[gk];
                const uint32_t len = (uint32_t)(a.offsets[gk + 1] - pos);
                uint64_t s0, s1;
                if (staged) {
                    const uint32_t o = (uint32_t)(pos - lo);
                    auto rd = [&](uint32_t off) -> uint64_t {
                        const uint32_t p = o + off;
                        const uint32_t *q = stage + (p >> 2);
                        return funnel64(q[0], q[1], q[2], (p & 3) * 8);
                    };
                    spooky_short(rd, len, a.seed, s0, s1);
                } else {
                    auto rd = [&](uint32_t off) -> uint64_t { return gload64(a.keys, a.blob_bytes, pos + off); };
                    spooky_short(rd, len, a.seed, s0, s1);
                }
                emit(kt, gk, s0, s1);
            }
            lo = nlo;
            nb = nnb;
        }
    } else {
        // direct global reads: long fixed keys (L > 52) and variable-length keys
        if (EPI == EPI_PARTITION) __syncthreads();
#pragma unroll
        for (int j = 0; j < P1_KEYS_PER_THREAD; ++j) {
            const uint32_t kt = tid + j * P1_THREADS;
            if (kt < tile_n) {
                const uint64_t gk = tile0 + kt;
                uint64_t pos, len;
                if (SRC == SRC_VAR) {
                    pos = a.offsets[gk];
                    len = a.offsets[gk + 1] - pos;
                } else {
                    pos = gk * L;
                    len = L;
                }
                auto rd = [&](uint32_t off) -> uint64_t { return gload64(a.keys, a.blob_bytes, pos + off); };
                uint64_t s0, s1;
                spooky_short(rd, (uint32_t)len, a.seed, s0, s1);
                emit(kt, gk, s0, s1);
            }
        }
    }

    if (EPI != EPI_PARTITION) return;

    // ---- counting sort of the tile by partition, then run-wise write-out ----
    __syncthreads();
    const uint32_t P = a.nparts;
    const uint32_t copy = a.region0 + (blockIdx.x & (NCOPY - 1));
    uint32_t cnt = tid < (int)P ? hist[tid] : 0, total;
    const uint32_t excl = block_excl_scan(cnt, wsum, tid, total);
    if (tid < (int)P) {
        start[tid] = excl;
        run[tid] = excl;
        base[tid] = cnt ? atomicAdd(a.cursor + copy * P + tid, cnt) : 0;
    }
    __syncthreads();
    for (uint32_t kt = tid; kt < tile_n; kt += P1_THREADS) {
        const uint32_t b = bkl[kt];
        const uint32_t pos = atomicAdd(&run[b >> a.bin_shift], 1u);
        sorted[pos] = b;
    }
    __syncthreads();
    bool ovf = false;
    for (uint32_t j = tid; j < tile_n; j += P1_THREADS) {
        const uint32_t b = sorted[j];
        const uint32_t p = b >> a.bin_shift;
        const uint64_t idx = (uint64_t)base[p] + (j - start[p]);
        if (idx < a.cap) {
            a.ids[((uint64_t)copy * a.nparts + p) * a.cap + idx] = (uint16_t)(b & (PART_BUCKETS - 1));
        } else {
            ovf = true;
        }
    }
    if (ovf) atomicOr(a.overflow, 1u);
}

// Pass 1, 13-byte keys, persistent and software-pipelined (the headline
// kernel).  Each workgroup walks tiles t = blockIdx.x, blockIdx.x + gridDim.x,
// ...; a thread owns keys tid + 512*j (j < 16) of a tile, split in two halves
// of 8 whose 16-byte windows live in register sets X and Y.  While one quarter
// of tile t hashes, the next is in flight; the next tile's first quarters are
// issued as soon as a set is consumed, so HBM reads continue through the hashing and through the
// tile epilogue (counting sort by partition, cursor reservation, run-wise
// write-out into XCD-shared regions).  Bucket ids stay in registers; LDS holds
// only the sorted tile.
// (Two sets of 8 windows spilled at 4 waves/SIMD; quarters of 4 keys in two
// alternating sets of 4 windows fit the 128-VGPR budget.)
constexpr int D13_Q = 4;                          // keys per quarter
constexpr int D13_NQ = P1_KEYS_PER_THREAD / D13_Q;  // quarters per tile

// Kept as the reference point for k_pass1_d13e (BSDB_D13_VARIANT=2): the
// round-1 epilogue, with its loads made unconditional and the epilogue run at
// raised wave priority (the workgroup's critical path).
template <int NT>
__global__ __launch_bounds__(NT, 4) void k_pass1_d13(P1Args a, uint64_t ntiles) {
    constexpr int TILE = NT * P1_KEYS_PER_THREAD;
    __shared__ uint32_t sorted[TILE];
    __shared__ uint32_t hist[MAX_PARTS], run[MAX_PARTS];
    __shared__ uint32_t off32[MAX_PARTS];
    __shared__ uint32_t wsum[2 * NT / 64];
    __shared__ uint32_t tile_ovf;
    const int tid = threadIdx.x;
    const uint32_t P = a.nparts;
    if (tid == 0) tile_ovf = 0;
    const uint32_t mult = (uint32_t)a.multiplier;
    const uint64_t G = gridDim.x;
    for (int i = tid; i < MAX_PARTS; i += NT) hist[i] = 0;

    uint64_t t = blockIdx.x;
    if (t >= ntiles) return;
    // every tile here is full and readable 3 bytes past its last key: the host
    // sends the ragged last tile to k_pass1<SRC_DIRECT13> (bounds-checked)
    // two register sets of D13_Q windows, alternating over the quarters
    u32x4a X[D13_Q], Y[D13_Q];
    // past the last tile the loads re-read tile blockIdx.x (unconditional
    // loads keep the compiler's waitcnt bookkeeping exact)
    const uint64_t t_first = blockIdx.x;
    auto load_q = [&](u32x4a(&R)[D13_Q], uint64_t tt, int q) {
        const uint64_t ts = tt < ntiles ? tt : t_first;
#pragma unroll
        for (int j = 0; j < D13_Q; ++j) {
            const uint64_t byte = (ts * TILE + tid + (q * D13_Q + j) * NT) * 13;
            R[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4a *>(a.keys + (byte & ~3ULL)));
        }
    };
    load_q(X, t, 0);
    load_q(Y, t, 1);
    __syncthreads();  // hist zeroed

    for (; t < ntiles; t += G) {
        uint32_t bk[P1_KEYS_PER_THREAD];
        uint32_t rk[P1_KEYS_PER_THREAD / 2];  // rank within (tile, partition), two u16 per register
        auto hash_q = [&](const u32x4a(&R)[D13_Q], int q) {
#pragma unroll
            for (int j = 0; j < D13_Q; ++j) {
                const uint32_t kt = tid + (q * D13_Q + j) * NT;
                const uint32_t sh = ((kt * 13u) & 3u) * 8u;  // tile0*13 is a multiple of 4
                W64 s0, s1;
                spooky13_u(R[j].x, R[j].y, R[j].z, R[j].w, sh, a.seed, s0, s1);
                const uint32_t b = bucket_of_w(s0, mult);
                const int jj = q * D13_Q + j;
                bk[jj] = b;
                // the count's old value is this key's rank in its partition run
                const uint32_t r = atomicAdd(&hist[b >> a.bin_shift], 1u);
                if (jj & 1) rk[jj >> 1] |= r << 16; else rk[jj >> 1] = r;
            }
        };
        hash_q(X, 0);
        load_q(X, t, 2);
        hash_q(Y, 1);
        load_q(Y, t, 3);
        hash_q(X, 2);
        load_q(X, t + G, 0);
        hash_q(Y, 3);
        load_q(Y, t + G, 1);
        __builtin_amdgcn_s_setprio(2);  // the epilogue is the workgroup's critical path
        __syncthreads();  // all hist adds of this tile done
        // Regions are shared by the workgroups of one XCD (copy = t % 8: tiles
        // are dealt round-robin, so copy c is written from one XCD's L2, where
        // consecutive reservations by different workgroups complete 128-byte
        // lines quickly).  The returning cursor atomic overlaps the LDS scatter.
        const uint32_t copy = (uint32_t)(t & (NCOPY - 1));
        // element offsets below are relative to this tile's region set (P*cap < 2^32)
        uint16_t *const tile_base = a.ids + (uint64_t)copy * P * a.cap;
        // partitions p = tid and p = tid + NT (P <= 2*NT)
        const uint32_t p0 = tid, p1 = tid + NT;
        const uint32_t c0 = p0 < P ? hist[p0] : 0, c1 = p1 < P ? hist[p1] : 0;
        uint32_t total;
        const uint32_t e0 = block_excl_scan_n<NT>(c0 + c1, wsum, tid, total);
        const uint32_t e1 = e0 + c0;
        uint32_t b0 = 0, b1 = 0;
        if (p0 < P) {
            run[p0] = e0;  // partition start in the sorted tile (read-only below)
            hist[p0] = 0;  // ready for the next tile
            if (c0) b0 = atomicAdd(a.cursor + copy * P + p0, c0);
        }
        if (p1 < P) {
            run[p1] = e1;
            hist[p1] = 0;
            if (c1) b1 = atomicAdd(a.cursor + copy * P + p1, c1);
        }
        __syncthreads();
        // scatter: slot = start[p] + rank (plain LDS reads, broadcast on equal p)
#pragma unroll
        for (int j = 0; j < P1_KEYS_PER_THREAD; ++j) {
            const uint32_t r = (rk[j >> 1] >> ((j & 1) * 16)) & 0xFFFFu;
            sorted[run[bk[j] >> a.bin_shift] + r] = bk[j];
        }
        if (p0 < P) {
            if ((uint64_t)b0 + c0 > a.cap) tile_ovf = 1;
            // element offset of sorted slot 0 for partition p (ids buffer < 2^32
            // elements: checked by the host plan)
            off32[p0] = (uint32_t)((uint64_t)p0 * a.cap + b0 - e0);
        }
        if (p1 < P) {
            if ((uint64_t)b1 + c1 > a.cap) tile_ovf = 1;
            off32[p1] = (uint32_t)((uint64_t)p1 * a.cap + b1 - e1);
        }
        __syncthreads();
        if (!tile_ovf) {
            // batched: 16 sorted reads, 16 offset reads, 16 two-byte stores
            uint32_t sb[P1_KEYS_PER_THREAD];
#pragma unroll
            for (int j = 0; j < P1_KEYS_PER_THREAD; ++j) sb[j] = sorted[tid + j * NT];
            uint32_t so[P1_KEYS_PER_THREAD];
#pragma unroll
            for (int j = 0; j < P1_KEYS_PER_THREAD; ++j) so[j] = off32[sb[j] >> a.bin_shift];
#pragma unroll
            for (int j = 0; j < P1_KEYS_PER_THREAD; ++j)
                tile_base[(uint64_t)(so[j] + tid + j * NT)] = (uint16_t)(sb[j] & (PART_BUCKETS - 1));
        } else if (tid == 0) {
            atomicOr(a.overflow, 1u);
        }
        __syncthreads();  // sorted / run / off64 reused by the next tile
        __builtin_amdgcn_s_setprio(0);
    }
}

// Pass 1, 13-byte keys -- the production kernel (k_pass1_d13e): binned, with
// a 16-byte write-out.  One 1024-thread workgroup per CU, 16384-key tiles,
// ONE barrier per tile.
//  * Hash: a key's 2-byte partition-local id goes from the hash straight into
//    its partition's LDS bin (rank = the bin counter's old value); no bucket
//    id or rank is held in registers, so the four quarters of a tile live in
//    four register sets and the next tile's quarter q is loaded as soon as
//    this tile's quarter q is hashed (three quarters of prefetch).
//  * Bins are double-buffered.  After the tile's barrier the owner lane of
//    partition p (lane p/16 of wave p%16) takes its count c and reserves the
//    bin's whole 8-id chunks (c & ~7) in the XCD-shared region of copy t % 8
//    with one cursor atomic; runs therefore start 16-byte aligned.  The
//    remainder (c & 7 ids) is not padded: the owner moves it to the start of
//    the same bin once its chunks are out (during the next tile) and re-arms
//    the counter at it, so the tile after next ranks on top of it.  Only the
//    workgroup's last two remainders per partition are padded (0xFFFF, which
//    pass 2 adds as 0), in one run at the end: pads fell from ~6 % of the
//    ids to ~0.1 %.
//  * During the next tile the wave streams its partitions' bins out as
//    16-byte chunks (ds_read_b128 -> global_store_dwordx4), chunks of all its
//    partitions packed across lanes: ~3 store instructions per wave per tile
//    instead of one 2-byte store per id.
// A bin holds 128 ids (tile share 61 +- 8); a run that would not fit padded
// (c > 120) or a full region raises the overflow flag and the chunk is
// recounted with direct atomics.
constexpr int D13E_NT = 1024;
constexpr int D13E_NW = D13E_NT / 64;
constexpr int D13E_TILE = D13E_NT * P1_KEYS_PER_THREAD;  // 16384
constexpr int D13E_BIN_IDS = 36864;  // ids per bin buffer: nparts * capb (72 KiB, two buffers)
constexpr int D13E_MAXP = 288;       // bins (capb >= 128 ids: tile share 57 +- 7.5 at 288 bins)
constexpr uint16_t ID_PAD = 0xFFFF;                       // not a local id (ids are < 2^15)

// VARIANT 0 is production.  Profiling only (results invalid): 1 = hash and
// bins, no cursor atomics and no write-out; 4 = per-wave phase cycles
// (s_memtime) written over counts[8*wave ..] (tools/stamp_probe_e.py);
// 12 = everything but the hash: the same loads, bins, cursor atomics and
// write-out with a 2-instruction stand-in bucket (uniform over [0, m) for
// random key bytes) -- what pass 1's memory traffic alone costs.
// L: the key length, 13 or an aligned 8 / 12 / 16 (the same design; the
// 16-byte window of a key then starts at the key itself).
template <int VARIANT, bool SEED0 = false, int L = 13>
__global__ __launch_bounds__(D13E_NT, 1) void k_pass1_d13e(P1Args a, uint64_t ntiles) {
    static_assert(L == 13 || L == 8 || L == 12 || L == 16, "key lengths of the windowed kernel");
    // SEED0: the seed is 0 (every BSDBWriter build, CBHS:209): the hash's
    // seed terms fold at compile time
    const uint64_t seed = SEED0 ? 0ull : a.seed;
    constexpr int NT = D13E_NT, NW = D13E_NW, TILE = D13E_TILE;
    __shared__ __align__(16) uint16_t bins[2][D13E_BIN_IDS];
    __shared__ uint32_t cnt[2][D13E_MAXP];
    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63;
    const uint32_t P = a.nparts;  // bins: bucket >> bin_shift
    const uint32_t CAPB = a.capb;  // P * CAPB <= D13E_BIN_IDS (host plan); mean fill 16384/P, CAPB >= 2.25x that
    const uint32_t bsh = a.bin_shift;
    const uint32_t mult = (uint32_t)a.multiplier;
    const uint64_t G = gridDim.x;
    for (int i = tid; i < 2 * D13E_MAXP; i += NT) (&cnt[0][0])[i] = 0;
    const uint64_t t0 = blockIdx.x;
    if (t0 >= ntiles) return;
    // wave w owns the contiguous partitions [w*PPW, w*PPW + PPW): lane l < PPW
    // owns w*PPW + l, so a wave's cursor atomics hit consecutive words
    const uint32_t PPW = (P + NW - 1) / NW;
    const bool owner = (uint32_t)l < PPW && (uint32_t)w * PPW + l < P;
    const uint32_t my_p = owner ? (uint32_t)w * PPW + l : P;  // P = none

    u32x4a S[4][D13_Q];
    // Key kt of a tile starts at byte L * kt of it; tile, quarter and key
    // slot offsets (multiples of L * NT, e.g. 13 * 1024 = 13312) are multiples of 4, so a
    // lane's 4-byte-aligned window offset and its byte shift are the same
    // for every key it loads: the address is a uniform base (scalar
    // arithmetic) + one 32-bit lane offset, no per-key VALU.
    const uint32_t lane_off = ((uint32_t)tid * L) & ~3u;
    const uint32_t sh = (((uint32_t)tid * L) & 3u) * 8u;  // (0 for L = 8, 12, 16)
    static_assert((NT * L) % 4 == 0 && ((uint64_t)TILE * L) % 4 == 0, "window alignment per lane");
    // unconditional loads (past the last tile they re-read tile t0): keeps
    // the compiler's waitcnt bookkeeping free of merged paths
    // Buffer loads through a per-tile descriptor (built by scalar code): the
    // lane offset is the voffset, the key slot's offset the soffset, so a
    // load costs no VALU (the flat form spent a 64-bit add per load).
    // aux 2 = nt (streamed once, as __builtin_nontemporal_load).
    auto load_q = [&](int q, uint64_t tt) {
        const uint64_t ts = tt < ntiles ? tt : t0;
        const uint8_t *tb = a.keys + ts * ((uint64_t)TILE * L);
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(tb), 0, TILE * L + 16, 0x00020000);
#pragma unroll
        for (int j = 0; j < D13_Q; ++j) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, lane_off, (q * D13_Q + j) * NT * L, 2);
            S[q][j] = u32x4a{v[0], v[1], v[2], v[3]};
        }
    };
    bool ovf = false;
    // the quarter's D13_Q keys hashed first, then their rank atomics issued
    // together and their ids stored: one LDS round trip per quarter
    auto hash_q = [&](int q, uint32_t cur) {
        uint32_t b[D13_Q], r[D13_Q];
#pragma unroll
        for (int j = 0; j < D13_Q; ++j) {
            if constexpr (VARIANT == 12)
                b[j] = __umulhi(S[q][j].x ^ S[q][j].z, mult >> 1);
            else if constexpr (L == 13)
                b[j] = spooky13_bucket(S[q][j].x, S[q][j].y, S[q][j].z, S[q][j].w, sh, seed, mult);
            else
                b[j] = spooky_fix_bucket<L>(S[q][j].x, S[q][j].y, S[q][j].z, S[q][j].w, seed, mult);
        }
#pragma unroll
        for (int j = 0; j < D13_Q; ++j) r[j] = atomicAdd(&cnt[cur][b[j] >> bsh], 1u);
#pragma unroll
        for (int j = 0; j < D13_Q; ++j) {
            // branch-free: an overflowing bin (flagged below) reuses its last slot
            const uint32_t slot = __umul24(b[j] >> bsh, CAPB) + min(r[j], CAPB - 1u);  // (v_mad_u32_u24 + v_min)
            __builtin_assume(slot < (uint32_t)D13E_BIN_IDS);
            bins[cur][slot] = (uint16_t)(b[j] & (PART_BUCKETS - 1));
        }
    };
    // owner state of the previous tile: whole-chunk count, remainder and
    // cursor base of my_p
    uint32_t c8_prev = 0, rm_prev = 0, b_prev = 0, copy_prev = 0;
    auto write_out = [&](uint32_t prev) {
        // chunks (8 ids) of this wave's partitions, packed across lanes:
        // owner lane j covers chunk indices [st_j, st_j + nch_j)
        // b_prev is first touched here, a whole tile after its atomic (a use
        // right after the atomic would also wait for the prefetch behind it)
        const bool fits = (uint64_t)b_prev + c8_prev <= a.cap;
        ovf |= my_p < P && !fits;
        const uint32_t nch = (my_p < P && fits) ? c8_prev / 8 : 0;
        uint32_t x = nch;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if (l >= d) x += y;
        }
        const uint32_t st = x - nch;
        const uint32_t total = __builtin_amdgcn_readlane(x, 63);
        uint16_t *const rbase = a.ids + (uint64_t)copy_prev * P * a.cap;  // P*cap < 2^32 (host plan)
        for (uint32_t i0 = 0; i0 < total; i0 += 64) {
            const uint32_t i = i0 + l;
            // owner lane j = last lane (of the first 32) with st_j <= i
            int j = 0;
#pragma unroll
            for (int step = 16; step >= 1; step >>= 1) {
                const uint32_t s_try = __shfl(st, j + step, 64);
                if (s_try <= i) j += step;
            }
            const uint32_t bj = __shfl(b_prev, j, 64), sj = __shfl(st, j, 64);
            const uint32_t k = i - sj;
            const uint32_t p = (uint32_t)w * PPW + j;
            if (i < total) {
                const uint4 v = *reinterpret_cast<const uint4 *>(&bins[prev][p * CAPB + 8 * k]);
                *reinterpret_cast<uint4 *>(rbase + (uint64_t)p * a.cap + bj + 8 * k) = v;
            }
        }
        // the remainder to the bin's start, for the tile after next (after
        // this wave's chunk reads in program order; that tile hashes after
        // the coming barrier)
        if (my_p < P && c8_prev)
            for (uint32_t e = 0; e < rm_prev; ++e) bins[prev][my_p * CAPB + e] = bins[prev][my_p * CAPB + c8_prev + e];
    };

#pragma unroll
    for (int q = 0; q < 4; ++q) load_q(q, t0);
    __syncthreads();  // cnt zeroed
    uint32_t cur = 0;
    bool have_prev = false;
    constexpr bool STAMP = VARIANT == 4;  // diagnostic: phase cycles over counts[]
    uint64_t st_h = 0, st_w = 0, st_b = 0, st_o = 0, ts = 0, st_t0 = 0;
    uint32_t st_n = 0;
    auto stamp = [&](uint64_t &acc) {
        if (STAMP) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            acc += now - ts;
            ts = now;
        }
    };
    if (STAMP) st_t0 = ts = __builtin_amdgcn_s_memtime();
    for (uint64_t t = t0; t < ntiles; t += G, cur ^= 1) {
        hash_q(0, cur);
        load_q(0, t + G);
        hash_q(1, cur);
        load_q(1, t + G);
        hash_q(2, cur);
        load_q(2, t + G);
        hash_q(3, cur);
        stamp(st_h);
        if (have_prev && VARIANT != 1) write_out(cur ^ 1);
        load_q(3, t + G);
        stamp(st_w);
        __syncthreads();  // bins[cur] complete; bins[cur ^ 1] written out
        stamp(st_b);
        ++st_n;
        // owners: count, reserve the whole chunks, re-arm at the remainder
        const uint32_t copy = (uint32_t)(t & (a.ncopy - 1));
        c8_prev = 0;
        rm_prev = 0;
        b_prev = 0;
        if (my_p < P) {
            const uint32_t c = cnt[cur][my_p];
            ovf |= c > CAPB;
            const uint32_t cc = c > CAPB ? 0 : c;  // (an overflow is recounted: nothing kept)
            c8_prev = cc & ~7u;
            rm_prev = cc & 7u;
            cnt[cur][my_p] = rm_prev;  // the tile after next ranks after the carried ids
        }
        // Every lane issues the atomic -- a lane without a partition adds 0
        // to a word of this workgroup's own scratch -- so the instruction is
        // unconditional and the waitcnt pass counts it exactly (the
        // write-out's wait for it then covers nothing younger).  Lanes of one
        // instruction must not share a word: same-word lanes are serialised
        // at the memory side (measured 6x slower).
        if (VARIANT != 1)
            b_prev = atomicAdd(my_p < P ? a.cursor + copy * P + my_p : a.scratch + P1_SCRATCH_WG + blockIdx.x * 1024 + tid,
                               c8_prev);
        copy_prev = copy;
        have_prev = true;
        stamp(st_o);
    }
    if (STAMP && l == 0) {
        const uint64_t wg = (uint64_t)blockIdx.x * NW + w;
        a.counts[8 * wg + 0] = (uint32_t)(st_h >> 4);
        a.counts[8 * wg + 1] = (uint32_t)(st_w >> 4);
        a.counts[8 * wg + 2] = (uint32_t)(st_b >> 4);
        a.counts[8 * wg + 3] = (uint32_t)(st_o >> 4);
        a.counts[8 * wg + 4] = (uint32_t)((__builtin_amdgcn_s_memtime() - st_t0) >> 4);
        a.counts[8 * wg + 5] = st_n;
    }
    if (have_prev && VARIANT != 1) write_out(cur ^ 1);
    // the last two remainders of my_p: the one carried to the start of
    // bins[cur] (its tile's successor never came) and the last tile's, moved
    // by write_out to the start of bins[cur ^ 1]: one run padded to 8
    if (have_prev && VARIANT != 1 && my_p < P) {
        uint16_t *const bc = &bins[cur][my_p * CAPB];
        const uint32_t r0 = cnt[cur][my_p], r1 = rm_prev;  // (<= 7 each)
        for (uint32_t e = 0; e < r1; ++e) bc[r0 + e] = bins[cur ^ 1][my_p * CAPB + e];
        const uint32_t c8 = (r0 + r1 + 7) & ~7u;
        for (uint32_t e = r0 + r1; e < c8; ++e) bc[e] = ID_PAD;
        if (c8) {
            const uint32_t base = atomicAdd(a.cursor + copy_prev * P + my_p, c8);
            if ((uint64_t)base + c8 <= a.cap) {
                uint16_t *const dst = a.ids + (uint64_t)copy_prev * P * a.cap + (uint64_t)my_p * a.cap + base;
                for (uint32_t k = 0; k < c8 / 8; ++k)
                    *reinterpret_cast<uint4 *>(dst + 8 * k) = *reinterpret_cast<const uint4 *>(bc + 8 * k);
            } else {
                ovf = true;
            }
        }
    }
    if (ovf) atomicOr(a.overflow, 1u);
}

// Pass 1, variable-length keys -- k_pass1_vare: the binned design of
// k_pass1_d13e behind a per-wave LDS-staged front end.  TWO 512-thread
// workgroups per CU, each with its own single-buffered bins, 8192-key tiles:
// while one workgroup waits at a tile barrier (its waves are unevenly served
// by the SIMDs' age-ordered VALU arbitration) or for its cursor atomics, the
// other keeps the SIMDs busy.
//  * A wave takes its keys in groups of 128 consecutive keys, two adjacent
//    keys per lane (group g of tile t: keys t*8192 + g*1024 + w*128 + 2*lane
//    + {0, 1}); hashing two keys at once gives the hash chains ILP.
//  * A group's bytes are one contiguous range of the blob (~2.3 KiB at the C5
//    mean of 17.7 B): the wave copies it with 16-byte loads, 3 per lane, into
//    its own LDS stage (no workgroup barrier); each lane then reads the 17
//    dwords a key of <= 64 B can touch and hashes on registers.  A group's
//    range and offsets are loaded two groups ahead; the range bounds of a
//    tile's groups a tile ahead, so no load waits on another.
//  * A range over 3 KiB is completed with synchronous loads; one over the
//    5 KiB stage (mean key > 39 B) is hashed straight from global memory, as
//    are keys over 64 B from the stage.
//  * After the tile's barrier each bin's owner lane pads it to 8 ids,
//    reserves its run in the XCD copy with one cursor atomic and its wave
//    writes its bins out in 16-byte chunks (k_pass1_d13e's write-out); a
//    second barrier frees the bins.  <= 144 bins of >= 2.25x their mean fill.
constexpr int VARE_NT = 512;
constexpr int VARE_NW = VARE_NT / 64;
constexpr int VARE_NG = 8;                         // groups of 128 keys per wave per tile
constexpr int VARE_TILE = VARE_NT * 2 * VARE_NG;   // 8192 keys
constexpr int VARE_BIN_IDS = 18432;                // ids in the bins (36 KiB)
constexpr int VARE_MAXP = 144;
constexpr uint32_t VARE_PRE_VECS = 192;            // 16-B vectors per group prefetched (3 per lane)
constexpr uint32_t VARE_STAGE_VECS = 288;          // 16-B vectors per wave stage (4.5 KiB)
constexpr int VARE_STAGE_WORDS = VARE_STAGE_VECS * 4 + 20;  // + slack for the 17-dword key reads
constexpr int VARE_PERM_WORDS = 128;               // per wave: a group's keys sorted short-first

__device__ __forceinline__ uint64_t readlane64(uint64_t x, int l) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(x >> 32), l) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((uint32_t)x, l);
}

// VARIANT 0 is production.  Profiling only (results invalid): 1 = no cursor
// atomics and no write-out; 4 = phase cycles (s_memtime) over counts[8*wave
// ..].
// k_pass1_vare's general-length paths (keys over 64 B, groups over the stage),
// out of line: the unrolled hot loop then carries one copy of each.
__device__ __forceinline__ uint64_t vare_sig0_lds(const uint32_t *stage, uint32_t o, uint32_t len,
                                                            uint64_t seed) {
    const uint32_t b = o >> 2, sh = (o & 3) * 8;
    auto rd = [&](uint32_t off) -> uint64_t {
        const uint32_t i = b + (off >> 2);
        return funnel64(stage[i], stage[i + 1], stage[i + 2], sh);
    };
    return spooky_short_sig0_u(rd, len, seed);
}
// a range over the stage: dword loads from global memory, clamped to the
// range's last dword (its lines are readable)
__device__ __forceinline__ uint64_t vare_sig0_global(const uint32_t *src, uint64_t nwords, uint64_t o,
                                                               uint32_t len, uint64_t seed) {
    const uint64_t last = nwords - 1, b = o >> 2;
    const uint32_t sh = (uint32_t)(o & 3) * 8;
    auto rd = [&](uint32_t off) -> uint64_t {
        const uint64_t i = b + (off >> 2);
        return funnel64(src[min(i, last)], src[min(i + 1, last)], src[min(i + 2, last)], sh);
    };
    return spooky_short_sig0_u(rd, len, seed);
}

// FIXED: keys of a.key_len bytes each, no offsets array (key k at k * L):
// the same kernel serves every fixed length but 13 (k_pass1_d13e).
template <int VARIANT, bool FIXED, bool SEED0 = false>
__global__ __launch_bounds__(VARE_NT, 4) void k_pass1_vare(P1Args a, uint64_t ntiles) {
    const uint64_t seed = SEED0 ? 0ull : a.seed;  // (as k_pass1_d13e)
    constexpr int NT = VARE_NT, NW = VARE_NW, TILE = VARE_TILE, NG = VARE_NG;
    __shared__ __align__(16) uint16_t bins[VARE_BIN_IDS];
    __shared__ uint32_t cnt[2][VARE_MAXP];  // rank counters, by tile parity
    __shared__ __align__(16) uint32_t stage_all[NW * VARE_STAGE_WORDS];
    __shared__ uint32_t perm_all[NW * VARE_PERM_WORDS];
    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63;
    uint32_t *const stage = stage_all + w * VARE_STAGE_WORDS;
    uint32_t *const perm = perm_all + w * VARE_PERM_WORDS;
    const uint32_t P = a.nparts;
    const uint32_t CAPB = a.capb;
    const uint32_t bsh = a.bin_shift;
    const uint32_t mult = (uint32_t)a.multiplier;
    const uint64_t G = gridDim.x;
    const uintptr_t blob = (uintptr_t)a.keys;
    for (int i = tid; i < 2 * VARE_MAXP; i += NT) (&cnt[0][0])[i] = 0;
    uint32_t cb = 0;  // counters of the tile being hashed
    const uint64_t t0 = blockIdx.x;
    if (t0 >= ntiles) return;
    const uint32_t PPW = (P + NW - 1) / NW;  // <= 18
    const bool owner = (uint32_t)l < PPW && (uint32_t)w * PPW + l < P;
    const uint32_t my_p = owner ? (uint32_t)w * PPW + l : P;
    constexpr bool STAMP = VARIANT == 4;
    uint64_t st_acc[6] = {0, 0, 0, 0, 0, 0}, st_last = 0, st_t0 = 0;
    auto stamp = [&](int ph) __attribute__((always_inline)) {
        if (STAMP) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            st_acc[ph] += now - st_last;
            st_last = now;
        }
    };

    // Range bounds of this wave's NG groups of a tile: lane 2g holds
    // off[first key of group g], lane 2g+1 off[its last key + 1].  Past the
    // last tile, tile t0 again (unconditional loads keep the waitcnt pass exact).
    auto load_bounds = [&](uint64_t tt) __attribute__((always_inline)) {
        const uint64_t ts = tt < ntiles ? tt : t0;
        const uint32_t i = (uint32_t)l < 2 * NG ? (uint32_t)l : 2 * NG - 1;
        const uint64_t k = ts * TILE + (i >> 1) * (NT * 2) + (uint64_t)w * 128 + (i & 1) * 128;
        if (FIXED) return k * a.key_len;
        return __builtin_nontemporal_load(a.offsets + k);
    };
    // B: a group's byte range (3 vectors per lane) and the lane's offsets
    // off[k], off[k+1], off[k+2] (k = its first key), ring of 2
    u32x4 V[2][3];
    u64x2 O01[2];
    uint64_t O2[2], Blo[2];
    uint32_t Bn[2];
    auto issue_B = [&](int r, uint64_t bnd, uint32_t gi, uint64_t tt) __attribute__((always_inline)) {
        const uint64_t first = readlane64(bnd, 2 * gi);
        const uint64_t last = readlane64(bnd, 2 * gi + 1);
        const uintptr_t lo = (blob + first) & ~(uintptr_t)15;
        const uint64_t nv = (blob + last - lo + 15) >> 4;  // 0: an all-empty group
        const uint32_t nvec = nv > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)nv;
        // an empty group reads the offsets array instead (always readable);
        // pointers derived from the kernel arguments, not from integers, so
        // the loads stay global_load (a flat load makes every wait a full drain)
        const uint8_t *src = nvec || FIXED ? a.keys + (lo - blob) : reinterpret_cast<const uint8_t *>(a.offsets);
        const uint32_t nl = nvec ? nvec - 1 : 0;
#pragma unroll
        for (int i = 0; i < 3; ++i)
            V[r][i] = __builtin_nontemporal_load(
                reinterpret_cast<const u32x4 *>(src + 16 * (uint64_t)min((uint32_t)(64 * i + l), nl)));
        const uint64_t ts = tt < ntiles ? tt : t0;
        const uint64_t k = ts * TILE + (uint64_t)gi * (NT * 2) + (uint64_t)w * 128 + 2 * l;
        if (FIXED) {
            const uint64_t L = a.key_len;
            O01[r] = u64x2{k * L, (k + 1) * L};
            O2[r] = (k + 2) * L;
        } else {
            O01[r] = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(a.offsets + k));
            O2[r] = __builtin_nontemporal_load(a.offsets + k + 2);
        }
        Blo[r] = lo;
        Bn[r] = nvec;
    };
    // the group's range -> this wave's stage (lanes past the range store
    // copies of its last vector into slots no key reads)
    auto stage_group = [&](int r) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 3; ++i) reinterpret_cast<u32x4 *>(stage)[64 * i + l] = V[r][i];
        const uint32_t nvec = Bn[r];
        if (nvec > VARE_PRE_VECS && nvec <= VARE_STAGE_VECS) {
            for (uint32_t v = VARE_PRE_VECS + l; v < nvec; v += 64)
                reinterpret_cast<u32x4 *>(stage)[v] =
                    __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(a.keys + (Blo[r] - blob) + 16 * (uint64_t)v));
        }
    };
    // signature word 0 of the key at blob offset pos (the general path)
    auto sig0_of = [&](uint64_t pos, uint32_t len, uintptr_t lo, uint32_t nvec, bool staged) __attribute__((always_inline)) {
        const uint64_t o = blob + pos - lo;
        if (staged) return vare_sig0_lds(stage, (uint32_t)o, len, seed);
        return vare_sig0_global(reinterpret_cast<const uint32_t *>(a.keys + (lo - blob)), 4 * (uint64_t)nvec, o, len, seed);
    };
    // bin inserts, software-pipelined: the rank atomics of a group are issued
    // after its hash and the ids stored during the next group (after its key
    // reads), so the atomics' round trip is not waited for in the group
    uint32_t pend_p[2] = {0, 0}, pend_rk[2] = {0, 0};
    uint16_t pend_id[2] = {0, 0};
    bool pend = false;
    auto insert = [&](int k, uint64_t s0) __attribute__((always_inline)) {
        const uint32_t bk = bucket_of_w(w64(s0), mult);
        const uint32_t p = bk >> bsh;
        pend_rk[k] = atomicAdd(&cnt[cb][p], 1u);  // first used by flush_inserts
        pend_p[k] = p;
        pend_id[k] = (uint16_t)(bk & (PART_BUCKETS - 1));
    };
    auto flush_inserts = [&]() __attribute__((always_inline)) {
        if (pend) {
#pragma unroll
            for (int k = 0; k < 2; ++k)
                bins[__umul24(pend_p[k], CAPB) + min(pend_rk[k], CAPB - 1u)] = pend_id[k];
        }
        pend = false;
    };
    // Hash of one key of a staged group per lane, o = its offset in the stage.
    // The hash branches on the length (ShortMix for >= 16 B, twice for >= 48
    // B); a branch runs whenever ANY lane takes it, so the caller sorts a
    // group's keys short-first: chain 0 then holds only keys < 16 B (no mix,
    // 5 dwords) unless the group has fewer than 64 of them.
    // VARIANT 5 (profiling, results invalid): every lane reads a conflict-free
    // address instead of its key's.  VARIANT 6: 8-byte aligned ds_read_b64
    // reads, the odd-dword start selected in registers.
    auto read_key = [&](uint32_t b, auto nc, uint32_t *d) __attribute__((always_inline)) {
        constexpr int N = decltype(nc)::value;
        if (VARIANT == 6) {
            const uint64_t *q = reinterpret_cast<const uint64_t *>(stage) + (b >> 1);
            const bool odd = b & 1;
            uint32_t x[N + 1 + (N & 1)];
#pragma unroll
            for (int i = 0; i < (N + 2) / 2; ++i) {
                const uint64_t v = q[i];
                x[2 * i] = (uint32_t)v;
                x[2 * i + 1] = (uint32_t)(v >> 32);
            }
#pragma unroll
            for (int i = 0; i < N; ++i) d[i] = odd ? x[i + 1] : x[i];
        } else {
            const uint32_t bb = VARIANT == 5 ? (uint32_t)l * 17 : b;
#pragma unroll
            for (int i = 0; i < N; ++i) d[i] = stage[bb + i];
        }
    };
    auto sig0_staged = [&](uint32_t o, uint32_t len) __attribute__((always_inline)) {
        const uint32_t b = o >> 2, sh = (o & 3) * 8;
        uint64_t s0;
        if (__builtin_amdgcn_ballot_w64(len >= 16) == 0) {  // wave-uniform
            uint32_t d[5];
            read_key(b, std::integral_constant<int, 5>{}, d);
            s0 = spooky_lt16_sig0(d, sh, len, seed);
        } else if (len <= 64) {
            uint32_t d[17];
            read_key(b, std::integral_constant<int, 17>{}, d);
            s0 = spooky_le64_sig0(d, sh, len, seed);
        } else {
            s0 = vare_sig0_lds(stage, o, len, seed);
        }
        return s0;
    };
    auto hash_group = [&](uint64_t pos, uint32_t la, uint32_t lb, uintptr_t lo, uint32_t nvec)
                          __attribute__((always_inline)) {
        const bool staged = nvec <= VARE_STAGE_VECS;  // wave-uniform
        uint64_t sa, sb;
        if (staged) {
            // sort the group's 128 keys (key 2l+k = lane l's key k) short
            // (< 16 B) first, by counting: q = rank among its class
            const uint32_t oa = (uint32_t)(blob + pos - lo), ob = oa + la;
            const bool s0 = la < 16, s1 = lb < 16;
            const uint64_t m0 = __builtin_amdgcn_ballot_w64(s0), m1 = __builtin_amdgcn_ballot_w64(s1);
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m0, 0u)) +
                                   __builtin_amdgcn_mbcnt_hi((uint32_t)(m1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m1, 0u));
            const uint32_t ns = (uint32_t)__builtin_popcountll(m0) + (uint32_t)__builtin_popcountll(m1);
            const uint32_t r0 = below, r1 = below + (s0 ? 1u : 0u);  // short ranks
            const uint32_t q0 = s0 ? r0 : ns + 2 * l - r0, q1 = s1 ? r1 : ns + 2 * l + 1 - r1;
            // (offsets < 4.6 KiB and lengths < 64 KiB: 16 bits each)
            perm[q0] = oa | (la << 16);
            perm[q1] = ob | (lb << 16);
            __builtin_amdgcn_wave_barrier();
            const uint32_t ka = perm[l], kb = perm[64 + l];
            flush_inserts();  // the previous group's ids
            sa = sig0_staged(ka & 0xFFFF, ka >> 16);
            sb = sig0_staged(kb & 0xFFFF, kb >> 16);
        } else {
            flush_inserts();
            sa = sig0_of(pos, la, lo, nvec, false);
            sb = sig0_of(pos + la, lb, lo, nvec, false);
        }
        insert(0, sa);
        insert(1, sb);
        pend = true;
    };

    bool ovf = false;
    // this wave's bins -> its region of copy `copy`, chunks of 8 ids packed
    // across lanes, one 16-byte store each (k_pass1_d13e's write-out)
    auto write_out = [&](uint32_t c8, uint32_t base, uint32_t copy) __attribute__((always_inline)) {
        const bool fits = (uint64_t)base + c8 <= a.cap;
        ovf |= my_p < P && !fits;
        const uint32_t nch = (my_p < P && fits) ? c8 / 8 : 0;
        uint32_t x = nch;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if (l >= d) x += y;
        }
        const uint32_t st = x - nch;
        const uint32_t total = __builtin_amdgcn_readlane(x, 63);
        uint16_t *const rbase = a.ids + (uint64_t)copy * P * a.cap;
        for (uint32_t i0 = 0; i0 < total; i0 += 64) {
            const uint32_t i = i0 + l;
            int j = 0;
#pragma unroll
            for (int step = 16; step >= 1; step >>= 1) {  // PPW <= 18 < 32
                const uint32_t s_try = __shfl(st, j + step, 64);
                if (s_try <= i) j += step;
            }
            const uint32_t bj = __shfl(base, j, 64), sj = __shfl(st, j, 64);
            const uint32_t k = i - sj;
            const uint32_t p = (uint32_t)w * PPW + j;
            if (i < total) {
                const uint4 v = *reinterpret_cast<const uint4 *>(&bins[p * CAPB + 8 * k]);
                *reinterpret_cast<uint4 *>(rbase + (uint64_t)p * a.cap + bj + 8 * k) = v;
            }
        }
    };

    // step j of tile tt: stage group j, issue group j+2's range and offsets
    // (from the next tile's bounds past the last group), hash group j.
    // Unrolled by construction: in a rolled loop the register allocator
    // rotates the ring with copies, and a copy of a loading register waits
    // for the load.
    uint64_t bnd_cur = 0, bnd_next = 0;
    auto step = [&](auto jc, uint64_t tt) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
        constexpr int r = j & 1;
        stamp(5);
        stage_group(r);
        stamp(0);
        const uint64_t pos = O01[r].x, lo = Blo[r];
        const uint32_t la = (uint32_t)(O01[r].y - O01[r].x), lb = (uint32_t)(O2[r] - O01[r].y), nvec = Bn[r];
        if (j + 2 < NG) issue_B(r, bnd_cur, j + 2, tt);
        else issue_B(r, bnd_next, j + 2 - NG, tt + G);
        stamp(1);
        __builtin_amdgcn_wave_barrier();
        hash_group(pos, la, lb, lo, nvec);
        __builtin_amdgcn_wave_barrier();  // this stage is refilled by the next group
        stamp(2);
    };

    if (STAMP) st_t0 = st_last = __builtin_amdgcn_s_memtime();
    bnd_cur = load_bounds(t0);
    issue_B(0, bnd_cur, 0, t0);
    issue_B(1, bnd_cur, 1, t0);
    __syncthreads();  // cnt zeroed
    bnd_next = load_bounds(t0 + G);
    step(std::integral_constant<int, 0>{}, t0);
    for (uint64_t t = t0; t < ntiles; t += G) {
        step(std::integral_constant<int, 1>{}, t);
        step(std::integral_constant<int, 2>{}, t);
        step(std::integral_constant<int, 3>{}, t);
        step(std::integral_constant<int, 4>{}, t);
        step(std::integral_constant<int, 5>{}, t);
        step(std::integral_constant<int, 6>{}, t);
        step(std::integral_constant<int, 7>{}, t);
        static_assert(NG == 8, "step calls");
        flush_inserts();
        __syncthreads();  // bins complete
        stamp(3);
        // owners: count, pad to a multiple of 8, re-arm, reserve; every lane
        // issues the atomic (a lane without a bin adds 0 to a scratch word of
        // its own: same-word lanes are serialised at the memory side)
        const uint32_t copy = (uint32_t)(t & (a.ncopy - 1));
        uint32_t c8 = 0;
        if (my_p < P) {
            const uint32_t c = cnt[cb][my_p];
            cnt[cb][my_p] = 0;
            ovf |= c > CAPB;
            c8 = c > CAPB ? 0 : (c + 7) & ~7u;
            for (uint32_t e = c; e < c8; ++e) bins[my_p * CAPB + e] = ID_PAD;
        }
        uint32_t base = 0;
        if (VARIANT != 1)
            base = atomicAdd(my_p < P ? a.cursor + copy * P + my_p : a.scratch + P1_SCRATCH_WG + blockIdx.x * 1024 + tid, c8);
        // while the atomics fly: step 0 of the next tile, up to its rank
        // atomics (other counters; its ids reach the bins after the barrier
        // below).  Past the last tile it hashes tile t0 again, to no effect.
        cb ^= 1;
        bnd_cur = bnd_next;
        bnd_next = load_bounds(t + 2 * G);
        step(std::integral_constant<int, 0>{}, t + G);
        stamp(2);
        if (VARIANT != 1) write_out(c8, base, copy);
        stamp(4);
        __syncthreads();  // bins written out and counters re-armed
        stamp(3);
    }
    if (STAMP && l == 0) {
        const uint64_t wg = (uint64_t)blockIdx.x * NW + w;
        for (int i = 0; i < 6; ++i) a.counts[8 * wg + i] = (uint32_t)(st_acc[i] >> 4);
        a.counts[8 * wg + 6] = (uint32_t)((__builtin_amdgcn_s_memtime() - st_t0) >> 4);
    }
    if (ovf) atomicOr(a.overflow, 1u);
}

// Fallback when pass 1 overflowed a region (adversarial key sets): recount the
// whole launch with direct atomics.  Exits immediately in the normal case.
template <int SRC, int LFIX>
__global__ __launch_bounds__(P1_THREADS) void k_overflow_fallback(P1Args a) {
    if (*a.overflow == 0) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(a.overflow + 2, 1u);  // bsdb_fallback_count
    const uint64_t stride = (uint64_t)gridDim.x * P1_THREADS;
    for (uint64_t gk = (uint64_t)blockIdx.x * P1_THREADS + threadIdx.x; gk < a.n; gk += stride) {
        uint64_t pos, len;
        if (SRC == SRC_VAR) {
            pos = a.offsets[gk];
            len = a.offsets[gk + 1] - pos;
        } else {
            pos = gk * a.key_len;
            len = a.key_len;
        }
        auto rd = [&](uint32_t off) -> uint64_t { return gload64(a.keys, a.blob_bytes, pos + off); };
        uint64_t s0, s1;
        spooky_short(rd, (uint32_t)len, a.seed, s0, s1);
        atomicAdd(a.counts + bucket_of(s0, a.multiplier), 1u);
    }
}

// ---- A6: exclusive prefix sum counts[m] (u32) -> E[m+1] (u64) ------------
constexpr int SCAN_THREADS = 1024;
constexpr int SCAN_PER_THREAD = 8;
constexpr int SCAN_BLOCK = SCAN_THREADS * SCAN_PER_THREAD;

__device__ __forceinline__ uint64_t block_excl_scan64(uint64_t v, uint64_t *wsum, int tid, uint64_t &total) {
    const int lane = tid & 63, wid = tid >> 6;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
    for (int w = 0; w < SCAN_THREADS / 64; ++w) {
        const uint64_t s = wsum[w];
        pre += w < wid ? s : 0;
        tot += s;
    }
    total = tot;
    __syncthreads();
    return pre + x - v;
}

__global__ __launch_bounds__(SCAN_THREADS) void k_scan_partial(const uint32_t *counts, uint64_t m, uint64_t *part) {
    __shared__ uint64_t wsum[SCAN_THREADS / 64];
    const uint64_t i0 = (uint64_t)blockIdx.x * SCAN_BLOCK + (uint64_t)threadIdx.x * SCAN_PER_THREAD;
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < SCAN_PER_THREAD; ++j) s += i0 + j < m ? counts[i0 + j] : 0;
    uint64_t tot;
    block_excl_scan64(s, wsum, threadIdx.x, tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ __launch_bounds__(SCAN_THREADS) void k_scan_top(uint64_t *part, uint64_t nparts) {
    __shared__ uint64_t wsum[SCAN_THREADS / 64];
    uint64_t carry = 0;
    for (uint64_t b = 0; b < nparts; b += SCAN_THREADS) {
        const uint64_t i = b + threadIdx.x;
        const uint64_t v = i < nparts ? part[i] : 0;
        uint64_t tot;
        const uint64_t e = block_excl_scan64(v, wsum, threadIdx.x, tot);
        if (i < nparts) part[i] = carry + e;
        carry += tot;
    }
}

__global__ __launch_bounds__(SCAN_THREADS) void k_scan_final(const uint32_t *counts, uint64_t m,
                                                             const uint64_t *part, uint64_t *E) {
    __shared__ uint64_t wsum[SCAN_THREADS / 64];
    const uint64_t i0 = (uint64_t)blockIdx.x * SCAN_BLOCK + (uint64_t)threadIdx.x * SCAN_PER_THREAD;
    uint32_t c[SCAN_PER_THREAD];
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < SCAN_PER_THREAD; ++j) {
        c[j] = i0 + j < m ? counts[i0 + j] : 0;
        s += c[j];
    }
    uint64_t tot;
    uint64_t run = part[blockIdx.x] + block_excl_scan64(s, wsum, threadIdx.x, tot);
    if (i0 == 0) E[0] = 0;
#pragma unroll
    for (int j = 0; j < SCAN_PER_THREAD; ++j) {
        run += c[j];
        if (i0 + j < m) E[i0 + j + 1] = run;
    }
}

// Pass 2, persistent and balanced.  A launch's id stream is the concatenation,
// partition-major, of its (partition, region) segments: items k = p*R + r,
// with regions 0..nmain-1 (capacity cap) followed by tail regions
// (capacity cap_tail).  k_pass2_plan prefix-sums the segment fills; each of
// the G workgroups of k_pass2b then histograms exactly its share
// [total*i/G, total*(i+1)/G) of the stream in a 128 KiB LDS table and
// flushes the table (coalesced atomics) only when its share crosses into the
// next partition: ~2 flushes per workgroup instead of one per (partition,
// slice), no tail of idle workgroups, and 4 x 16 B of ids in flight per lane.
struct P2Layout {
    const uint16_t *ids;
    const uint32_t *cursor;    // fills [R][P] (P = region bins)
    const uint32_t *overflow;
    uint64_t cap, cap_tail;    // ids per segment of a main / tail region
    uint32_t nparts, nmain, ntail;
    uint32_t bshift;           // bins per pass-2 partition = 2^bshift (bin = bucket >> (15 - bshift))
    uint64_t num_buckets;
    uint32_t *counts;
};

__device__ __forceinline__ uint64_t p2_seg_base(const P2Layout &L, uint32_t p, uint32_t r) {
    return r < L.nmain ? ((uint64_t)r * L.nparts + p) * L.cap
                       : (uint64_t)L.nmain * L.nparts * L.cap + ((uint64_t)(r - L.nmain) * L.nparts + p) * L.cap_tail;
}

constexpr int P2_ITEMS_PER_THREAD = 8;

// pref[k] = ids before item k (exclusive), pref[NI] = total.  One workgroup,
// items in rounds of SCAN_THREADS * P2_ITEMS_PER_THREAD.
__global__ __launch_bounds__(SCAN_THREADS) void k_pass2_plan(P2Layout L, uint64_t *pref) {
    __shared__ uint64_t wsum[SCAN_THREADS / 64];
    const uint32_t R = L.nmain + L.ntail, NI = L.nparts * R;
    const int tid = threadIdx.x;
    uint64_t carry = 0;
    for (uint32_t base = 0; base < NI; base += SCAN_THREADS * P2_ITEMS_PER_THREAD) {
        uint64_t f[P2_ITEMS_PER_THREAD], s = 0;
#pragma unroll
        for (int j = 0; j < P2_ITEMS_PER_THREAD; ++j) {
            const uint32_t k = base + tid * P2_ITEMS_PER_THREAD + j;
            f[j] = 0;
            if (k < NI) {
                const uint32_t p = k / R, r = k % R;
                f[j] = min((uint64_t)L.cursor[(uint64_t)r * L.nparts + p], r < L.nmain ? L.cap : L.cap_tail);
            }
            s += f[j];
        }
        uint64_t tot;
        uint64_t run = carry + block_excl_scan64(s, wsum, tid, tot);  // ends with a barrier
#pragma unroll
        for (int j = 0; j < P2_ITEMS_PER_THREAD; ++j) {
            const uint32_t k = base + tid * P2_ITEMS_PER_THREAD + j;
            if (k < NI) pref[k] = run;
            run += f[j];
        }
        carry += tot;
    }
    if (tid == 0) pref[NI] = carry;
}

__global__ __launch_bounds__(P2_THREADS, 1) void k_pass2b(P2Layout L, const uint64_t *pref) {
    __shared__ uint32_t hist[PART_BUCKETS + 64];  // + per-lane sinks for pads
    __shared__ uint32_t k_start;
    if (*L.overflow) return;
    const int tid = threadIdx.x;
    const uint32_t R = L.nmain + L.ntail, NI = L.nparts * R;
    const uint64_t G = gridDim.x, total = pref[NI];
    const uint64_t lo = total * blockIdx.x / G, hi = total * (blockIdx.x + 1) / G;
    if (lo >= hi) return;
    if (tid == 0) {
        // first item with pref[k] <= lo < pref[k+1]
        uint32_t a = 0, b = NI;  // invariant: pref[a] <= lo < pref[b]
        while (b - a > 1) {
            const uint32_t c = (a + b) / 2;
            if (pref[c] <= lo) a = c; else b = c;
        }
        k_start = a;
    }
    for (int i = tid; i < PART_BUCKETS; i += P2_THREADS) hist[i] = 0;
    __syncthreads();
    auto flush = [&](uint32_t p) {
        __syncthreads();
        const uint64_t b0 = (uint64_t)p << PART_SHIFT;
        const uint32_t nb = (uint32_t)min((uint64_t)PART_BUCKETS, L.num_buckets - b0);
        for (uint32_t i = tid; i < PART_BUCKETS; i += P2_THREADS) {
            const uint32_t h = hist[i];
            if (h && i < nb) atomicAdd(L.counts + b0 + i, h);
            hist[i] = 0;
        }
        __syncthreads();
    };
    const uint32_t sink = PART_BUCKETS + (tid & 63);
    static_assert(PART_BUCKETS + 64 <= 0xFFFF, "pads sort above the sinks");
    int64_t cur_p = -1;
    for (uint32_t k = k_start; k < NI; ++k) {
        const uint64_t pk = pref[k], pk1 = pref[k + 1];
        if (pk >= hi) break;
        const uint64_t a = max(lo, pk) - pk, b = min(hi, pk1) - pk;
        if (a >= b) continue;
        const uint32_t p = k / R, r = k % R;  // bin p of pass-2 partition p >> bshift
        if ((int64_t)(p >> L.bshift) != cur_p) {
            if (cur_p >= 0) flush((uint32_t)cur_p);
            cur_p = p >> L.bshift;
        }
        // segment base is a multiple of 64 ids: 16-byte vectors from a8 on
        const uint16_t *src = L.ids + p2_seg_base(L, p, r);
        const uint64_t a8 = min(b, (a + 7) & ~7ULL), b8 = max(a8, b & ~7ULL);
        // an id with the top bit set is a pad (ID_PAD): it goes to a per-lane
        // sink word (pads of one wave on one word would serialise)
        // (pads are 0xFFFF > every sink index > every id: one v_min, which the
        // compiler folds with the 16-bit extraction into an SDWA operand)
        auto add_id = [&](uint32_t id) { atomicAdd(&hist[min(id, sink)], 1u); };
        if (a + tid < a8) add_id(src[a + tid]);
        if (b8 + tid < b) add_id(src[b8 + tid]);
        const uint4 *v = reinterpret_cast<const uint4 *>(src);
        uint64_t i = a8 / 8 + tid;
        const uint64_t v1 = b8 / 8;
        for (; i + 3 * P2_THREADS < v1; i += 4 * P2_THREADS) {
            uint4 w[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) w[u] = ntload16(v + i + u * P2_THREADS);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                add_id(w[u].x & 0xFFFF); add_id(w[u].x >> 16);
                add_id(w[u].y & 0xFFFF); add_id(w[u].y >> 16);
                add_id(w[u].z & 0xFFFF); add_id(w[u].z >> 16);
                add_id(w[u].w & 0xFFFF); add_id(w[u].w >> 16);
            }
        }
        for (; i < v1; i += P2_THREADS) {
            const uint4 w = ntload16(v + i);
            add_id(w.x & 0xFFFF); add_id(w.x >> 16);
            add_id(w.y & 0xFFFF); add_id(w.y >> 16);
            add_id(w.z & 0xFFFF); add_id(w.z >> 16);
            add_id(w.w & 0xFFFF); add_id(w.w >> 16);
        }
    }
    if (cur_p >= 0) flush((uint32_t)cur_p);
}

// key i has length 8 + r, r drawn Zipf(s=1.1)
// over the 57 lengths 8..64 (rank 1 = length 8) by inverse CDF on
// u = splitmix64(i ^ 0xB5DB0005); bytes 0-7 = i big-endian (BaseTest.java:16-24),
// tail word w (bytes 8+8w..) = splitmix64(((i << 3) + w) ^ 0xB5DB0005A5A5A5A5)
// little-endian.  Thresholds = floor(CDF(r) * 2^64), r = 1..56.
__constant__ uint64_t ZIPF_CDF[56] = {0x415ff50621eab000ULL, 0x5fdf8ea4661c1800ULL, 0x7365cc48cd422800ULL, 0x81a02c160ca0d800ULL, 0x8cc1c51827e0f000ULL, 0x95dd881c0eabb000ULL, 0x9d8d9c8bd387d800ULL, 0xa430d6d3c06da800ULL, 0xaa0593efa19cb800ULL, 0xaf36f652f272a000ULL, 0xb3e4079390b42800ULL, 0xb823d5bdeb558000ULL, 0xbc07f52bb16ae800ULL, 0xbf9e197287e21000ULL, 0xc2f123c939aa0800ULL, 0xc609db869ad6f800ULL, 0xc8ef6f73a3a9d800ULL, 0xcba7d2952de20000ULL, 0xce38001f766e2000ULL, 0xd0a42e21797a3800ULL, 0xd2eff3ea03b6c000ULL, 0xd51e678ba501e800ULL, 0xd73234d900b38000ULL, 0xd92daf816c491000ULL, 0xdb12e17da86ff800ULL, 0xdce396a9b5e6c000ULL, 0xdea1662ec6fe5800ULL, 0xe04dba370d317800ULL, 0xe1e9d64761753000ULL, 0xe376dc8509ffe800ULL, 0xe4f5d21dcfad2800ULL, 0xe667a2fc93d9d000ULL, 0xe7cd24eb876f7000ULL, 0xe9271a3e3b92e800ULL, 0xea76341874c6f000ULL, 0xebbb14628b26f800ULL, 0xecf64f78eaa7d000ULL, 0xee286da1bdeba000ULL, 0xef51ec51cc50e000ULL, 0xf0733f47f9ee2000ULL, 0xf18cd1858f189800ULL, 0xf29f062863636800ULL, 0xf3aa392b30515800ULL, 0xf4aec00f9fea5000ULL, 0xf5acea751b007800ULL, 0xf6a5029ee3f44800ULL, 0xf7974deba8448800ULL, 0xf8840d40614fb000ULL, 0xf96b7d68184c6800ULL, 0xfa4dd769e82e0000ULL, 0xfb2b50d667f27000ULL, 0xfc041c0d7f209800ULL, 0xfcd8687d83bcc000ULL, 0xfda862dc63a64800ULL, 0xfe74355b824d6000ULL, 0xff3c07d6de49e800ULL};

__device__ __forceinline__ uint32_t varkey_len(uint64_t i) {
    const uint64_t u = splitmix64(i ^ 0xB5DB0005ULL);
    uint32_t r = 0;
#pragma unroll 8
    for (int t = 0; t < 56; ++t) r += u >= ZIPF_CDF[t];
    return 8 + r;
}

__global__ __launch_bounds__(256) void k_gen_var_len(uint64_t first, uint64_t n, uint32_t *len) {
    for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (uint64_t)gridDim.x * 256)
        len[k] = varkey_len(first + k);
}

__global__ __launch_bounds__(256) void k_gen_var_fill(uint64_t first, uint64_t n, const uint64_t *off, uint8_t *blob) {
    for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (uint64_t)gridDim.x * 256) {
        const uint64_t i = first + k, p = off[k];
        const uint32_t len = (uint32_t)(off[k + 1] - p);
        for (int b = 0; b < 8; ++b) blob[p + b] = (uint8_t)(i >> (56 - 8 * b));
        for (uint32_t j = 8; j < len; j += 8) {
            const uint64_t w = splitmix64(((i << 3) + ((j - 8) >> 3)) ^ 0xB5DB0005A5A5A5A5ULL);
            for (uint32_t b = 0; b < 8 && j + b < len; ++b) blob[p + j + b] = (uint8_t)(w >> (8 * b));
        }
    }
}

// ---- synthetic 13-byte keys (bench input) ------------
// Grid-stride over blocks of 256 keys: a dispatch holds < 2^32 work-items, so
// a 13 B-key set (the README shape) cannot be one thread per key.
__global__ __launch_bounds__(256) void k_gen_keys13(uint64_t first, uint64_t n, uint8_t *out) {
    __shared__ __align__(16) uint8_t buf[256 * 13];
    const uint64_t nblk = (n + 255) / 256;
    for (uint64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
        const uint64_t k0 = blk * 256;
        const uint64_t k = k0 + threadIdx.x;
        __syncthreads();
        if (k < n) {
            const uint64_t i = first + k;
            const uint64_t w0 = splitmix64(i ^ 0xB5DB0001ULL);
            const uint64_t w1 = (i ^ (splitmix64(i + 1) >> 24)) & 0xFFFFFFFFFFULL;
            uint8_t *d = buf + threadIdx.x * 13;
            for (int b = 0; b < 8; ++b) d[b] = (uint8_t)(w0 >> (8 * b));
            for (int b = 0; b < 5; ++b) d[8 + b] = (uint8_t)(w1 >> (8 * b));
        }
        __syncthreads();
        // k0*13 = blk*3328 is dword aligned: dword stores, byte tail
        const uint32_t nbytes = (uint32_t)min((uint64_t)256, n - k0) * 13;
        uint32_t *o32 = reinterpret_cast<uint32_t *>(out + k0 * 13);
        const uint32_t *b32 = reinterpret_cast<const uint32_t *>(buf);
        for (uint32_t w = threadIdx.x; w < nbytes / 4; w += 256) o32[w] = b32[w];
        for (uint32_t b = (nbytes & ~3u) + threadIdx.x; b < nbytes; b += 256) out[k0 * 13 + b] = buf[b];
    }
}

}  // namespace bsdb
