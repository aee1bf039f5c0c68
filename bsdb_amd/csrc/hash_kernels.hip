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
// stream.  So pass 1 hashes a tile of 8192 keys, counting-sorts the tile's
// bucket ids by partition (32768 buckets each) in LDS and writes 2-byte
// partition-local ids in runs; pass 2 histograms one partition at a time in a
// 128 KiB LDS table and flushes it with coalesced atomics.  Extra traffic is
// 4 B/key on top of the key bytes.  See DESIGN.md.
#include <hip/hip_runtime.h>
#include <stdint.h>

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
                atomicAdd(&hist[b >> PART_SHIFT], 1u);
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
        const uint32_t pos = atomicAdd(&run[b >> PART_SHIFT], 1u);
        sorted[pos] = b;
    }
    __syncthreads();
    bool ovf = false;
    for (uint32_t j = tid; j < tile_n; j += P1_THREADS) {
        const uint32_t b = sorted[j];
        const uint32_t p = b >> PART_SHIFT;
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

// VARIANT 0 is production.  Profiling variants (results invalid), pass-1 ms
// per 2^31 keys at the C4 bucket count: 1 = hash only,
// no tile epilogue (5.0 vs 7.0); 5 = scan + cursor atomics + barriers, no
// scatter / write-out (6.4); 7 = no write-out (7.07); 6 = adds as
// v_add_co/v_addc pairs (+3.5 %).  Private per-workgroup regions (no cursor
// atomics) measured 8.37: a tile leaves ~60 B per partition, so private lines
// are written partially, while the XCD-shared regions complete lines in L2.
template <int VARIANT, int NT>
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
    const W64 seedw = w64(a.seed);
    const uint64_t G = gridDim.x;
    // EXACT (VARIANT >= 19): every vector-memory operation of the loop is
    // unconditional and each wave only ever waits for its OLDEST outstanding
    // operations (s_waitcnt vmcnt counts loads, stores and atomics together,
    // in issue order): the cursor atomics are issued before the next tile's
    // prefetch, the id stores before the loop head's wait for it.
    constexpr bool EXACT = VARIANT >= 19;
    constexpr bool PRIO = VARIANT == 12 || VARIANT == 19;
    bool ovf_any = false;
    for (int i = tid; i < MAX_PARTS; i += NT) hist[i] = 0;

    uint64_t t = blockIdx.x;
    if (t >= ntiles) return;
    // every tile here is full and readable 3 bytes past its last key: the host
    // sends the ragged last tile to k_pass1<SRC_DIRECT13> (bounds-checked)
    // two register sets of D13_Q windows, alternating over the quarters
    u32x4a X[D13_Q], Y[D13_Q];
    // Past the last tile the loads re-read tile blockIdx.x instead of being
    // skipped: a conditional load would make the waitcnt pass merge the two
    // paths and wait for the fresh prefetch before hashing the current quarter.
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
    if (EXACT) {
        // the loop head is entered with the previous tile's 16 id stores
        // behind the prefetch; give the first entry the same shape so the
        // waitcnt pass needs no conservative merge there
        uint16_t *const dummy = reinterpret_cast<uint16_t *>(a.scratch + 2048);
#pragma unroll
        for (int j = 0; j < P1_KEYS_PER_THREAD; ++j) dummy[j * NT + tid] = 0;
    }
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
                if (VARIANT == 6)
                    spooky13_w(R[j].x, R[j].y, R[j].z, R[j].w, sh, seedw, s0, s1);
                else
                    spooky13_u(R[j].x, R[j].y, R[j].z, R[j].w, sh, a.seed, s0, s1);
                const uint32_t b = bucket_of_w(s0, mult);
                const int jj = q * D13_Q + j;
                bk[jj] = b;
                // the count's old value is this key's rank in its partition run
                const uint32_t r = atomicAdd(&hist[b >> PART_SHIFT], 1u);
                if (jj & 1) rk[jj >> 1] |= r << 16; else rk[jj >> 1] = r;
            }
        };
        hash_q(X, 0);
        load_q(X, t, 2);
        hash_q(Y, 1);
        load_q(Y, t, 3);
        hash_q(X, 2);
        if (!EXACT) load_q(X, t + G, 0);
        hash_q(Y, 3);
        if (!EXACT) load_q(Y, t + G, 1);
        if (VARIANT == 1) {
            uint32_t x = 0;
#pragma unroll
            for (int j = 0; j < P1_KEYS_PER_THREAD; ++j) x ^= bk[j];
            if (x == 0xFFFFFFFFu) a.overflow[1] = x;  // keep the hashes live
            continue;
        }
        if (PRIO) __builtin_amdgcn_s_setprio(2);  // epilogue = the workgroup's critical path
        __syncthreads();  // all hist adds of this tile done
        // Regions are shared by the workgroups of one XCD (copy = t % 8: tiles
        // are dealt round-robin, so copy c is written from one XCD's L2, where
        // consecutive reservations by different workgroups complete 128-byte
        // lines quickly).  The returning cursor atomic overlaps the LDS scatter.
        const uint32_t copy = (uint32_t)(t & (NCOPY - 1));
        // element offsets below are relative to this tile's region set
        // (P*cap < 2^32: checked by the host plan)
        uint16_t *const tile_base = a.ids + (uint64_t)copy * P * a.cap;
        // partitions p = tid and p = tid + NT (P <= 2*NT)
        const uint32_t p0 = tid, p1 = tid + NT;
        const uint32_t c0 = p0 < P ? hist[p0] : 0, c1 = p1 < P ? hist[p1] : 0;
        uint32_t total;
        const uint32_t e0 = block_excl_scan_n<NT>(c0 + c1, wsum, tid, total);
        const uint32_t e1 = e0 + c0;
        uint32_t b0 = 0, b1 = 0;
        if (EXACT) {
            // every lane adds (0 to a scratch word when it has no partition)
            uint32_t *const wgs = a.scratch + P1_SCRATCH_WG + blockIdx.x * 1024;  // this workgroup's own words
            b0 = atomicAdd(p0 < P ? a.cursor + copy * P + p0 : wgs + p0, c0);
            b1 = atomicAdd(p1 < P ? a.cursor + copy * P + p1 : wgs + (p1 & 1023), c1);
            load_q(X, t + G, 0);
            load_q(Y, t + G, 1);
        }
        if (p0 < P) {
            run[p0] = e0;  // partition start in the sorted tile (read-only below)
            hist[p0] = 0;  // ready for the next tile
            if (!EXACT && c0) b0 = atomicAdd(a.cursor + copy * P + p0, c0);
        }
        if (p1 < P) {
            run[p1] = e1;
            hist[p1] = 0;
            if (!EXACT && c1) b1 = atomicAdd(a.cursor + copy * P + p1, c1);
        }
        __syncthreads();
        // scatter: slot = start[p] + rank (plain LDS reads, broadcast on equal p)
#pragma unroll
        for (int j = 0; j < P1_KEYS_PER_THREAD; ++j) {
            const uint32_t r = (rk[j >> 1] >> ((j & 1) * 16)) & 0xFFFFu;
            if (VARIANT != 5) sorted[run[bk[j] >> PART_SHIFT] + r] = bk[j];
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
        if (EXACT) {
            // unconditional stores: an overflowing tile writes element 0 of its
            // region set (garbage, the chunk is recounted) instead of past cap
            const bool ovf = tile_ovf;
            ovf_any |= ovf;
            uint32_t sb[P1_KEYS_PER_THREAD];
#pragma unroll
            for (int j = 0; j < P1_KEYS_PER_THREAD; ++j) sb[j] = sorted[tid + j * NT];
            uint32_t so[P1_KEYS_PER_THREAD];
#pragma unroll
            for (int j = 0; j < P1_KEYS_PER_THREAD; ++j) so[j] = off32[sb[j] >> PART_SHIFT];
#pragma unroll
            for (int j = 0; j < P1_KEYS_PER_THREAD; ++j)
                tile_base[ovf ? 0 : (uint64_t)(so[j] + tid + j * NT)] = (uint16_t)(sb[j] & (PART_BUCKETS - 1));
        } else if (VARIANT == 5 || VARIANT == 7) {
        } else if (!tile_ovf) {
            // batched: 16 sorted reads, 16 offset reads, 16 two-byte stores
            uint32_t sb[P1_KEYS_PER_THREAD];
#pragma unroll
            for (int j = 0; j < P1_KEYS_PER_THREAD; ++j) sb[j] = sorted[tid + j * NT];
            uint32_t so[P1_KEYS_PER_THREAD];
#pragma unroll
            for (int j = 0; j < P1_KEYS_PER_THREAD; ++j) so[j] = off32[sb[j] >> PART_SHIFT];
#pragma unroll
            for (int j = 0; j < P1_KEYS_PER_THREAD; ++j)
                tile_base[(uint64_t)(so[j] + tid + j * NT)] = (uint16_t)(sb[j] & (PART_BUCKETS - 1));
        } else if (tid == 0) {
            atomicOr(a.overflow, 1u);
        }
        __syncthreads();  // sorted / run / off64 reused by the next tile
        if (PRIO) __builtin_amdgcn_s_setprio(0);
    }
    if (EXACT && ovf_any && tid == 0) atomicOr(a.overflow, 1u);
}

// Pass 1, 13-byte keys, two barriers per tile (k_pass1_d13b).  Same front end
// and XCD-shared regions as k_pass1_d13; the tile epilogue is re-timed so no
// wave waits on a returning memory operation or on a partner's scan:
//   A  barrier: hist[cur] complete
//      every wave scans the (<= 512) partition counts itself into its own
//      copy runw[w] (no barrier), scatters its keys into `sorted`, and thread
//      p issues the cursor atomic of partition p;
//      then the next tile's first quarter is hashed (into hist[nxt]) while
//      the atomics return; thread p writes off32[p];
//   C  barrier: sorted / off32 complete
//      write-out (runs of 2-byte ids into the XCD-shared regions), then
//      hist[cur] is zeroed for the tile after next.
// `sorted`, `off32` need no double buffer: the next scatter / off32 write is
// behind the next A barrier, which every wave reaches after its write-out.
// hist is double-buffered: the next tile's first quarter counts into hist[nxt]
// while slower waves may still be scanning hist[cur].
// STAMP (diagnostic builds only, results invalid): per-wave s_memtime sums of
// the cycles spent in barrier A, in barrier C and in the whole loop, written
// over counts[4*wave ..] at exit.
template <int NT, int KQ, int WPS, int STAMP = 0, int PRIO = 0>
__global__ __launch_bounds__(NT, WPS) void k_pass1_d13b(P1Args a, uint64_t ntiles) {
    constexpr int TILE = NT * P1_KEYS_PER_THREAD;
    constexpr int NQ = P1_KEYS_PER_THREAD / KQ;  // quarters per tile (even)
    static_assert(NQ % 2 == 0, "two alternating register sets");
    constexpr int NW = NT / 64;
    __shared__ uint32_t sorted[TILE];
    __shared__ __align__(16) uint32_t hist[2][MAX_PARTS];
    __shared__ __align__(16) uint32_t runw[NW][MAX_PARTS];
    __shared__ uint32_t off32[MAX_PARTS];
    __shared__ uint32_t tile_ovf;
    const int tid = threadIdx.x;
    const int w = tid >> 6, l = tid & 63;
    const uint32_t P = a.nparts;
    const uint32_t mult = (uint32_t)a.multiplier;
    const uint64_t G = gridDim.x;
    if (tid == 0) tile_ovf = 0;
    for (int i = tid; i < 2 * MAX_PARTS; i += NT) (&hist[0][0])[i] = 0;

    uint64_t t = blockIdx.x;
    if (t >= ntiles) return;
    // every tile here is full and readable 3 bytes past its last key: the host
    // sends the ragged end to k_pass1<SRC_DIRECT13> (bounds-checked)
    u32x4a X[KQ], Y[KQ];
    const uint64_t t_first = blockIdx.x;  // see k_pass1_d13c: unconditional loads
    auto load_q = [&](u32x4a(&R)[KQ], uint64_t tt, int q) {
        const uint64_t ts = tt < ntiles ? tt : t_first;
#pragma unroll
        for (int j = 0; j < KQ; ++j) {
            const uint64_t byte = (ts * TILE + tid + (q * KQ + j) * NT) * 13;
            R[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4a *>(a.keys + (byte & ~3ULL)));
        }
    };
    uint32_t bk[P1_KEYS_PER_THREAD];
    uint32_t rk[P1_KEYS_PER_THREAD / 2];  // rank within (tile, partition), two u16 per register
    auto hash_q = [&](const u32x4a(&R)[KQ], int q, uint32_t *h) {
#pragma unroll
        for (int j = 0; j < KQ; ++j) {
            const uint32_t kt = tid + (q * KQ + j) * NT;
            const uint32_t sh = ((kt * 13u) & 3u) * 8u;  // tile0*13 is a multiple of 4
            W64 s0, s1;
            spooky13_u(R[j].x, R[j].y, R[j].z, R[j].w, sh, a.seed, s0, s1);
            const uint32_t b = bucket_of_w(s0, mult);
            const int jj = q * KQ + j;
            bk[jj] = b;
            // the count's old value is this key's rank in its partition run
            const uint32_t r = atomicAdd(&h[b >> PART_SHIFT], 1u);
            if (jj & 1) rk[jj >> 1] |= r << 16; else rk[jj >> 1] = r;
        }
    };
    load_q(X, t, 0);
    load_q(Y, t, 1);
    __syncthreads();  // hist zeroed
    uint32_t cur = 0;
    uint64_t st_a = 0, st_c = 0;
    uint32_t st_n = 0;
    const uint64_t st_t0 = STAMP ? __builtin_amdgcn_s_memtime() : 0;
    hash_q(X, 0, hist[cur]);
    if (NQ > 2) load_q(X, t, 2); else load_q(X, t + G, 0);

    for (; t < ntiles; t += G, cur ^= 1) {
        // quarter q hashes from set q%2, then that set loads quarter q+2
        // (of this tile, or of the next one)
#pragma unroll
        for (int q = 1; q < NQ; ++q) {
            if (q & 1) {
                hash_q(Y, q, hist[cur]);
                if (q + 2 < NQ) load_q(Y, t, q + 2); else load_q(Y, t + G, q + 2 - NQ);
            } else {
                hash_q(X, q, hist[cur]);
                if (q + 2 < NQ) load_q(X, t, q + 2); else load_q(X, t + G, q + 2 - NQ);
            }
        }
        uint64_t ts0 = STAMP ? __builtin_amdgcn_s_memtime() : 0;
        __syncthreads();  // A: hist[cur] complete
        if (STAMP) {
            const uint64_t ts1 = __builtin_amdgcn_s_memtime();
            st_a += ts1 - ts0;
        }
        if (PRIO) __builtin_amdgcn_s_setprio(2);
        // cursor reservation of partitions p0 = tid, p1 = tid + NT in the
        // XCD-shared regions of copy t % 8 (tiles are dealt round-robin, so a
        // copy is written from one XCD's L2), issued first to give the
        // atomics the most time
        const uint32_t copy = (uint32_t)(t & (NCOPY - 1));
        const uint32_t p0 = tid, p1 = tid + NT;
        uint32_t c0 = 0, c1 = 0, b0 = 0, b1 = 0;
        if (p0 < P) {
            c0 = hist[cur][p0];
            if (c0) b0 = atomicAdd(a.cursor + copy * P + p0, c0);
        }
        if (p1 < P) {
            c1 = hist[cur][p1];
            if (c1) b1 = atomicAdd(a.cursor + copy * P + p1, c1);
        }
        // per-wave exclusive scan of the partition counts: lane l owns
        // partitions 8l .. 8l+7 (entries >= P are zero)
        {
            const uint4 h0 = *reinterpret_cast<const uint4 *>(&hist[cur][8 * l]);
            const uint4 h1 = *reinterpret_cast<const uint4 *>(&hist[cur][8 * l + 4]);
            uint32_t e[8] = {0, h0.x, h0.x + h0.y, h0.x + h0.y + h0.z, 0, 0, 0, 0};
            e[4] = e[3] + h0.w;
            e[5] = e[4] + h1.x;
            e[6] = e[5] + h1.y;
            e[7] = e[6] + h1.z;
            const uint32_t tot = e[7] + h1.w;
            uint32_t x = tot;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(x, d, 64);
                if (l >= d) x += y;
            }
            const uint32_t base = x - tot;
            *reinterpret_cast<uint4 *>(&runw[w][8 * l]) = make_uint4(base + e[0], base + e[1], base + e[2], base + e[3]);
            *reinterpret_cast<uint4 *>(&runw[w][8 * l + 4]) = make_uint4(base + e[4], base + e[5], base + e[6], base + e[7]);
        }
        // scatter: slot = run[p] + rank (this wave's own copy of run; LDS
        // operations of one wave complete in order)
#pragma unroll
        for (int j = 0; j < P1_KEYS_PER_THREAD; ++j) {
            const uint32_t r = (rk[j >> 1] >> ((j & 1) * 16)) & 0xFFFFu;
            sorted[runw[w][bk[j] >> PART_SHIFT] + r] = bk[j];
        }
        // the next tile's first quarter hashes while the atomics return
        if (PRIO) __builtin_amdgcn_s_setprio(0);
        if (t + G < ntiles) {
            hash_q(X, 0, hist[cur ^ 1]);
            if (NQ > 2) load_q(X, t + G, 2); else load_q(X, t + 2 * G, 0);
        }
        if (p0 < P) {
            if ((uint64_t)b0 + c0 > a.cap) tile_ovf = 1;
            // element offset, relative to this copy's region set, of sorted slot 0
            off32[p0] = (uint32_t)((uint64_t)p0 * a.cap + b0 - runw[w][p0]);
        }
        if (p1 < P) {
            if ((uint64_t)b1 + c1 > a.cap) tile_ovf = 1;
            off32[p1] = (uint32_t)((uint64_t)p1 * a.cap + b1 - runw[w][p1]);
        }
        ts0 = STAMP ? __builtin_amdgcn_s_memtime() : 0;
        if (PRIO) __builtin_amdgcn_s_setprio(2);
        __syncthreads();  // C: sorted, off32 complete; every scan of hist[cur] done
        if (STAMP) {
            const uint64_t ts1 = __builtin_amdgcn_s_memtime();
            st_c += ts1 - ts0;
            ++st_n;
        }
        if (!tile_ovf) {
            uint16_t *const tile_base = a.ids + (uint64_t)copy * P * a.cap;  // P*cap < 2^32 (host plan)
            uint32_t sb[P1_KEYS_PER_THREAD];
#pragma unroll
            for (int j = 0; j < P1_KEYS_PER_THREAD; ++j) sb[j] = sorted[tid + j * NT];
            uint32_t so[P1_KEYS_PER_THREAD];
#pragma unroll
            for (int j = 0; j < P1_KEYS_PER_THREAD; ++j) so[j] = off32[sb[j] >> PART_SHIFT];
#pragma unroll
            for (int j = 0; j < P1_KEYS_PER_THREAD; ++j)
                tile_base[(uint64_t)(so[j] + tid + j * NT)] = (uint16_t)(sb[j] & (PART_BUCKETS - 1));
        } else if (tid == 0) {
            atomicOr(a.overflow, 1u);
        }
        if (p0 < P) hist[cur][p0] = 0;  // for the tile after next
        if (p1 < P) hist[cur][p1] = 0;
        if (PRIO) __builtin_amdgcn_s_setprio(0);
    }
    if (STAMP && l == 0) {
        const uint64_t wg = (uint64_t)blockIdx.x * NW + w;
        a.counts[4 * wg + 0] = (uint32_t)(st_a >> 4);
        a.counts[4 * wg + 1] = (uint32_t)(st_c >> 4);
        a.counts[4 * wg + 2] = (uint32_t)((__builtin_amdgcn_s_memtime() - st_t0) >> 4);
        a.counts[4 * wg + 3] = st_n;
    }
}

// Pass 1, 13-byte keys, binned (k_pass1_d13c): ONE barrier per 16384-key tile.
// A key's 2-byte local id goes straight from the hash into its partition's
// LDS bin (rank from the bin counter, ds_add_rtn), so no bucket id or rank is
// kept in registers and there is no scan, no scatter pass and no sorted copy.
// Bins are double-buffered: while tile t hashes into bins[cur], the bins of
// tile t-1 are written out; partition p is owned by lane p / 16 of wave
// p % 16, which reserved p's run in the XCD-shared region with a cursor
// atomic right after tile t-1's barrier -- a whole tile earlier -- so the
// write-out reads the count and base with readlane and never waits on memory.
// A bin holds 128 ids (tile share 61 +- 8, i.e. 8.6 sigma); an overflowing bin
// raises the overflow flag and the chunk is recounted with direct atomics.
constexpr int D13C_NT = 1024;
constexpr int D13C_NW = D13C_NT / 64;
constexpr int D13C_TILE = D13C_NT * P1_KEYS_PER_THREAD;  // 16384
constexpr int D13C_CAPB = 128;                            // ids per bin
constexpr int D13C_MAXP = 288;                            // 2 x 288 x 256 B of bins = 144 KiB

template <int VARIANT>
__global__ __launch_bounds__(D13C_NT, 1) void k_pass1_d13c(P1Args a, uint64_t ntiles) {
    constexpr int NT = D13C_NT, NW = D13C_NW, TILE = D13C_TILE, CAPB = D13C_CAPB;
    __shared__ __align__(16) uint16_t bins[2][D13C_MAXP * CAPB];
    __shared__ uint32_t cnt[2][D13C_MAXP];
    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63;
    const uint32_t P = a.nparts;
    const uint32_t mult = (uint32_t)a.multiplier;
    const uint64_t G = gridDim.x;
    for (int i = tid; i < 2 * D13C_MAXP; i += NT) (&cnt[0][0])[i] = 0;
    uint64_t t = blockIdx.x;
    if (t >= ntiles) return;
    // partition owned by this lane (valid when < P)
    const uint32_t my_p = (uint32_t)l * NW + w;
    const uint32_t nj = (P + NW - 1) / NW;  // partitions per wave (upper bound)

    u32x4a X[D13_Q], Y[D13_Q];
    // Past the last tile the loads re-read tile blockIdx.x instead of being
    // skipped: a conditional load would make the waitcnt pass merge the two
    // paths and wait for the fresh prefetch before hashing the current quarter.
    const uint64_t t_first = blockIdx.x;
    auto load_q = [&](u32x4a(&R)[D13_Q], uint64_t tt, int q) {
        const uint64_t ts = tt < ntiles ? tt : t_first;
#pragma unroll
        for (int j = 0; j < D13_Q; ++j) {
            const uint64_t byte = (ts * TILE + tid + (q * D13_Q + j) * NT) * 13;
            R[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4a *>(a.keys + (byte & ~3ULL)));
        }
    };
    bool bin_ovf = false;
    auto hash_q = [&](const u32x4a(&R)[D13_Q], int q, uint32_t cur) {
#pragma unroll
        for (int j = 0; j < D13_Q; ++j) {
            const uint32_t kt = tid + (q * D13_Q + j) * NT;
            const uint32_t sh = ((kt * 13u) & 3u) * 8u;  // tile0*13 is a multiple of 4
            W64 s0, s1;
            spooky13_u(R[j].x, R[j].y, R[j].z, R[j].w, sh, a.seed, s0, s1);
            const uint32_t b = bucket_of_w(s0, mult);
            const uint32_t p = b >> PART_SHIFT;
            const uint32_t r = atomicAdd(&cnt[cur][p], 1u);
            // branch-free: an overflowing bin (flagged; the chunk is
            // recounted) keeps overwriting its last slot
            bins[cur][p * CAPB + (r < CAPB ? r : CAPB - 1)] = (uint16_t)(b & (PART_BUCKETS - 1));
            bin_ovf |= r >= CAPB;
        }
    };
    // owner state of the previous tile: count and cursor base of partition my_p
    uint32_t c_prev = 0, b_prev = 0, copy_prev = 0;
    bool have_prev = false, cap_ovf = false;
    // EXACT (VARIANT 2): a fixed number of unconditional stores / atomics
    // per tile (lanes with nothing to write store to a scratch word), so the
    // waitcnt pass counts the loop head exactly and no wave waits for its
    // own id stores before hashing.
    constexpr bool EXACT = VARIANT == 2;
    constexpr uint32_t MAXJ = (D13C_MAXP + NW - 1) / NW;
    uint16_t *const dummy = reinterpret_cast<uint16_t *>(a.scratch + 2048);
    auto write_out_exact = [&](uint32_t prev) {
        uint16_t *const rbase = a.ids + (uint64_t)copy_prev * P * a.cap;  // P*cap < 2^32 (host plan)
        const uint16_t *const bp = bins[prev];
        if (my_p < P && (uint64_t)b_prev + c_prev > a.cap) cap_ovf = true;
#pragma unroll
        for (uint32_t j = 0; j < MAXJ; ++j) {
            const uint32_t p = j * NW + w;
            uint32_t c = (uint32_t)__builtin_amdgcn_readlane(c_prev, j);
            const uint32_t b = (uint32_t)__builtin_amdgcn_readlane(b_prev, j);
            c = c < (uint32_t)CAPB ? c : (uint32_t)CAPB;
            if (p >= P || (uint64_t)b + c > a.cap) c = 0;
            const uint32_t ps = p < P ? p : 0;
            const uint16_t v0 = bp[ps * CAPB + l], v1 = bp[ps * CAPB + 64 + l];
            const uint32_t base = ps * (uint32_t)a.cap + b;
            uint16_t *const d0 = (uint32_t)l < c ? rbase + base + l : dummy + tid;
            uint16_t *const d1 = (uint32_t)l + 64 < c ? rbase + base + 64 + l : dummy + tid;
            *d0 = v0;
            *d1 = v1;
        }
    };
    auto write_out = [&](uint32_t prev) {
        uint16_t *const rbase = a.ids + (uint64_t)copy_prev * P * a.cap;  // P*cap < 2^32 (host plan)
        const uint16_t *const bp = bins[prev];
        if (my_p < P && (uint64_t)b_prev + c_prev > a.cap) cap_ovf = true;
        for (uint32_t j = 0; j < nj; ++j) {
            const uint32_t p = j * NW + w;
            if (p >= P) break;
            uint32_t c = (uint32_t)__builtin_amdgcn_readlane(c_prev, j);
            c = c < (uint32_t)CAPB ? c : (uint32_t)CAPB;
            const uint32_t b = (uint32_t)__builtin_amdgcn_readlane(b_prev, j);
            if ((uint64_t)b + c > a.cap) continue;  // region full: flagged above, never written past
            const uint32_t base = p * (uint32_t)a.cap + b;
            const uint16_t v0 = (uint32_t)l < c ? bp[p * CAPB + l] : 0;
            const uint16_t v1 = (uint32_t)l + 64 < c ? bp[p * CAPB + 64 + l] : 0;
            if ((uint32_t)l < c) rbase[base + l] = v0;
            if ((uint32_t)l + 64 < c) rbase[base + 64 + l] = v1;
        }
    };

    load_q(X, t, 0);
    load_q(Y, t, 1);
    if (EXACT) {
        // same shape as the loop head: 2*MAXJ stores and one atomic behind the prefetch
#pragma unroll
        for (uint32_t j = 0; j < 2 * MAXJ; ++j) *(volatile uint16_t *)(dummy + tid) = 0;
        (void)atomicAdd(a.scratch + tid, 0u);
    }
    __syncthreads();  // cnt zeroed
    uint32_t cur = 0;
    for (; t < ntiles; t += G, cur ^= 1) {
        hash_q(X, 0, cur);
        load_q(X, t, 2);
        hash_q(Y, 1, cur);
        load_q(Y, t, 3);
        hash_q(X, 2, cur);
        load_q(X, t + G, 0);
        hash_q(Y, 3, cur);
        load_q(Y, t + G, 1);
        if (EXACT) write_out_exact(cur ^ 1);  // first tile: c_prev = 0, all to scratch
        else if (have_prev && VARIANT != 1) write_out(cur ^ 1);
        __syncthreads();  // bins[cur] complete; bins[cur ^ 1] written out
        // owners: take partition my_p's count, re-arm its counter for the
        // tile after next, reserve its run (returns during the next tile)
        const uint32_t copy = (uint32_t)(t & (NCOPY - 1));
        c_prev = 0;
        b_prev = 0;
        if (my_p < P) {
            c_prev = cnt[cur][my_p];
            cnt[cur][my_p] = 0;
            if (!EXACT && c_prev && VARIANT != 1) b_prev = atomicAdd(a.cursor + copy * P + my_p, c_prev);
        }
        if (EXACT) b_prev = atomicAdd(my_p < P ? a.cursor + copy * P + my_p : a.scratch + tid, c_prev);
        copy_prev = copy;
        have_prev = true;
    }
    if (EXACT) write_out_exact(cur ^ 1);
    else if (have_prev && VARIANT != 1) write_out(cur ^ 1);
    if (bin_ovf || cap_ovf) atomicOr(a.overflow, 1u);
}

// Pass 1, 13-byte keys, warp-specialised (k_pass1_d13d) -- the production
// kernel.  One 1024-thread workgroup per CU:
//  * waves 0..11 hash.  A key's 2-byte partition-local id goes straight from
//    the hash into its partition's LDS bin (rank from the bin counter), so a
//    hashing wave keeps no bucket ids, issues no store and no global atomic:
//    its only vector-memory operations are its key loads, four quarters deep
//    (set q holds quarter q; the next tile's quarter q is loaded as soon as
//    this tile's is hashed), so every s_waitcnt the compiler emits is exact.
//  * waves 12..15 write.  After the tile's barrier a writer takes the counts
//    of its partitions (p = w' + 4k), re-arms their bin counters, reserves
//    each run in the XCD-shared region of copy t % 8 with one cursor atomic,
//    and streams the bins out while the hashers fill the other bin buffer.
// One barrier per 12288-key tile.  A bin holds 128 ids (tile share 46 +- 7,
// 12 sigma); an overflowing bin or region raises the overflow flag and the
// chunk is recounted with direct atomics.
constexpr int D13D_NT = 1024;
constexpr int D13D_HW = 12;                                   // hashing waves
constexpr int D13D_WW = 4;                                    // writing waves
constexpr int D13D_HT = D13D_HW * 64;                         // hashing threads
constexpr int D13D_TILE = D13D_HT * P1_KEYS_PER_THREAD;       // 12288
constexpr int D13D_CAPB = 128;
constexpr int D13D_MAXP = 288;

template <int VARIANT>
__global__ __launch_bounds__(D13D_NT, 1) void k_pass1_d13d(P1Args a, uint64_t ntiles) {
    constexpr int CAPB = D13D_CAPB, HT = D13D_HT, TILE = D13D_TILE;
    __shared__ __align__(16) uint16_t bins[2][D13D_MAXP * CAPB];
    __shared__ uint32_t cnt[2][D13D_MAXP];
    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63;  // wave index in an SGPR
    const uint32_t P = a.nparts;
    const uint64_t G = gridDim.x;
    for (int i = tid; i < 2 * D13D_MAXP; i += D13D_NT) (&cnt[0][0])[i] = 0;
    const uint64_t t0 = blockIdx.x;
    if (t0 >= ntiles) return;
    bool ovf = false;
    uint32_t cur = 0;
    if (w < D13D_HW) {
        // ---------------- hashing waves ----------------
        const uint32_t mult = (uint32_t)a.multiplier;
        u32x4a S[4][D13_Q];
        // past the last tile the loads re-read tile t0 (unconditional: keeps
        // the compiler's waitcnt bookkeeping exact)
        auto load_q = [&](int q, uint64_t tt) {
            const uint64_t ts = tt < ntiles ? tt : t0;
#pragma unroll
            for (int j = 0; j < D13_Q; ++j) {
                const uint64_t byte = (ts * TILE + tid + (q * D13_Q + j) * HT) * 13;
                S[q][j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4a *>(a.keys + (byte & ~3ULL)));
            }
        };
#pragma unroll
        for (int q = 0; q < 4; ++q) load_q(q, t0);
        __syncthreads();  // cnt zeroed
        for (uint64_t t = t0; t < ntiles; t += G, cur ^= 1) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
#pragma unroll
                for (int j = 0; j < D13_Q; ++j) {
                    const uint32_t kt = tid + (q * D13_Q + j) * HT;
                    const uint32_t sh = ((kt * 13u) & 3u) * 8u;  // tile0*13 is a multiple of 4
                    W64 s0, s1;
                    spooky13_u(S[q][j].x, S[q][j].y, S[q][j].z, S[q][j].w, sh, a.seed, s0, s1);
                    const uint32_t b = bucket_of_w(s0, mult);
                    const uint32_t p = b >> PART_SHIFT;
                    const uint32_t r = atomicAdd(&cnt[cur][p], 1u);
                    if (r < CAPB) bins[cur][p * CAPB + r] = (uint16_t)(b & (PART_BUCKETS - 1));
                    else ovf = true;
                }
                load_q(q, t + G);
            }
            __syncthreads();  // bins[cur] complete; bins[cur ^ 1] written out
        }
    } else {
        // ---------------- writing waves ----------------
        const uint32_t ww = (uint32_t)(w - D13D_HW);
        __syncthreads();  // cnt zeroed
        for (uint64_t t = t0; t < ntiles; t += G, cur ^= 1) {
            __syncthreads();  // bins[cur] complete
            // partitions p = ww + 4*(64*i + lane), i = 0, 1
            const uint32_t copy = (uint32_t)(t & (NCOPY - 1));
            uint32_t c[2], b[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const uint32_t p = ww + D13D_WW * (64 * i + l);
                c[i] = 0;
                b[i] = 0;
                if (p < P) {
                    c[i] = cnt[cur][p];
                    cnt[cur][p] = 0;  // re-armed for the tile after next
                    if (c[i] && VARIANT != 1) b[i] = atomicAdd(a.cursor + copy * P + p, c[i]);
                }
            }
            if (VARIANT == 1) continue;
            uint16_t *const rbase = a.ids + (uint64_t)copy * P * a.cap;  // P*cap < 2^32 (host plan)
            const uint16_t *const bp = bins[cur];
            // batches of 4 partitions: 8 LDS reads in flight, then 8 stores
            constexpr int BATCH = 4;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                if ((uint64_t)b[i] + c[i] > a.cap) ovf = true;
                for (uint32_t j0 = 0; j0 < 64; j0 += BATCH) {
                    if (ww + D13D_WW * (64 * i + j0) >= P) break;
                    uint32_t cj[BATCH], base[BATCH];
                    uint16_t v0[BATCH], v1[BATCH];
#pragma unroll
                    for (int u = 0; u < BATCH; ++u) {
                        const uint32_t p = ww + D13D_WW * (64 * i + j0 + u);
                        uint32_t cc = p < P ? (uint32_t)__builtin_amdgcn_readlane(c[i], j0 + u) : 0;
                        cc = cc < (uint32_t)CAPB ? cc : (uint32_t)CAPB;
                        const uint32_t bb = (uint32_t)__builtin_amdgcn_readlane(b[i], j0 + u);
                        if ((uint64_t)bb + cc > a.cap) cc = 0;  // full region: flagged, never written past
                        cj[u] = cc;
                        base[u] = p * (uint32_t)a.cap + bb;
                        const uint32_t ps = p < P ? p : 0;  // reads stay inside the bins
                        v0[u] = bp[ps * CAPB + l];
                        v1[u] = bp[ps * CAPB + 64 + l];
                    }
#pragma unroll
                    for (int u = 0; u < BATCH; ++u) {
                        if ((uint32_t)l < cj[u]) rbase[base[u] + l] = v0[u];
                        if ((uint32_t)l + 64 < cj[u]) rbase[base[u] + 64 + l] = v1[u];
                    }
                }
            }
        }
    }
    if (ovf) atomicOr(a.overflow, 1u);
}

// Pass 1, 13-byte keys, binned with 16-byte write-out (k_pass1_d13e).
// One 1024-thread workgroup per CU, 16384-key tiles, ONE barrier per tile.
//  * Hash: a key's 2-byte partition-local id goes from the hash straight into
//    its partition's LDS bin (rank = the bin counter's old value); no bucket
//    id or rank is held in registers, so the four quarters of a tile live in
//    four register sets and the next tile's quarter q is loaded as soon as
//    this tile's quarter q is hashed (three quarters of prefetch).
//  * Bins are double-buffered.  After the tile's barrier the owner lane of
//    partition p (lane p/16 of wave p%16) takes its count c, pads the bin to
//    a multiple of 8 ids with 0xFFFF (pass 2 adds 0 for a pad), re-arms the
//    counter and reserves the padded run in the XCD-shared region of copy
//    t % 8 with one cursor atomic; runs therefore start 16-byte aligned.
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
constexpr int D13E_CAPB = 128;
constexpr int D13E_MAXP = 288;
constexpr uint16_t ID_PAD = 0xFFFF;                       // not a local id (ids are < 2^15)

template <int VARIANT>
__global__ __launch_bounds__(D13E_NT, 1) void k_pass1_d13e(P1Args a, uint64_t ntiles) {
    constexpr int NT = D13E_NT, NW = D13E_NW, TILE = D13E_TILE, CAPB = D13E_CAPB;
    __shared__ __align__(16) uint16_t bins[2][D13E_MAXP * CAPB];
    __shared__ uint32_t cnt[2][D13E_MAXP];
    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63;
    const uint32_t P = a.nparts;
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
    // unconditional loads (past the last tile they re-read tile t0): keeps
    // the compiler's waitcnt bookkeeping free of merged paths
    auto load_q = [&](int q, uint64_t tt) {
        const uint64_t ts = tt < ntiles ? tt : t0;
#pragma unroll
        for (int j = 0; j < D13_Q; ++j) {
            const uint64_t byte = (ts * TILE + tid + (q * D13_Q + j) * NT) * 13;
            S[q][j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4a *>(a.keys + (byte & ~3ULL)));
        }
    };
    bool ovf = false;
    auto hash_q = [&](int q, uint32_t cur) {
#pragma unroll
        for (int j = 0; j < D13_Q; ++j) {
            const uint32_t kt = tid + (q * D13_Q + j) * NT;
            const uint32_t sh = ((kt * 13u) & 3u) * 8u;  // tile0*13 is a multiple of 4
            W64 s0, s1;
            spooky13_u(S[q][j].x, S[q][j].y, S[q][j].z, S[q][j].w, sh, a.seed, s0, s1);
            const uint32_t b = bucket_of_w(s0, mult);
            const uint32_t p = b >> PART_SHIFT;
            const uint32_t r = atomicAdd(&cnt[cur][p], 1u);
            // branch-free: an overflowing bin (flagged below) reuses its last slot
            bins[cur][p * CAPB + (r < CAPB ? r : CAPB - 1)] = (uint16_t)(b & (PART_BUCKETS - 1));
        }
    };
    // owner state of the previous tile: padded count and cursor base of my_p
    uint32_t c8_prev = 0, b_prev = 0, copy_prev = 0;
    auto write_out = [&](uint32_t prev) {
        // chunks (8 ids) of this wave's partitions, packed across lanes:
        // owner lane j covers chunk indices [st_j, st_j + nch_j)
        // b_prev is first touched here, a whole tile after its atomic: a
        // use right after the atomic would wait for the prefetch behind it.
        // Outstanding now, oldest first: the atomic, then this tile's
        // prefetch of quarters 0..2 (12 loads).
        if (VARIANT != 1 && VARIANT != 6) asm volatile("s_waitcnt vmcnt(12)" : "+v"(b_prev)::"memory");
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
                if (VARIANT == 2) {
                    if (v.x == 0x12345678u) a.overflow[1] = v.y;  // keep the read live
                } else if (VARIANT == 3) {
                    *reinterpret_cast<uint4 *>(a.ids + ((uint64_t)blockIdx.x * NT + tid) * 8) = v;
                } else {
                    *reinterpret_cast<uint4 *>(rbase + (uint64_t)p * a.cap + bj + 8 * k) = v;
                }
            }
        }
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
        if (have_prev && VARIANT != 1 && VARIANT != 5) write_out(cur ^ 1);
        load_q(3, t + G);
        stamp(st_w);
        __syncthreads();  // bins[cur] complete; bins[cur ^ 1] written out
        stamp(st_b);
        ++st_n;
        // owners: count, pad to a multiple of 8, re-arm, reserve
        const uint32_t copy = (uint32_t)(t & (a.ncopy - 1));
        c8_prev = 0;
        b_prev = 0;
        if (my_p < P) {
            const uint32_t c = cnt[cur][my_p];
            cnt[cur][my_p] = 0;  // the tile after next counts into it again
            ovf |= c > CAPB - 8;
            const uint32_t c8 = c > CAPB - 8 ? 0 : (c + 7) & ~7u;
            for (uint32_t e = c; e < c8; ++e) bins[cur][my_p * CAPB + e] = ID_PAD;
            c8_prev = c8;
        }
        // every lane issues the atomic (0 to a scratch word without a
        // partition): an unconditional instruction keeps the waitcnt pass
        // exact, so the write-out's wait for it never covers the prefetch
        // The atomic is inline asm, issued by the owner lanes only: hipcc
        // does not count it, so no waitcnt anywhere is widened by the
        // conditional issue; its one consumer (the write-out a tile later)
        // waits for it with an explicit, exact vmcnt.
        if (VARIANT != 1 && VARIANT != 6 && my_p < P) {
            uint32_t *const addr = a.cursor + copy * P + my_p;
            asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(b_prev) : "v"(addr), "v"(c8_prev) : "memory");
        }
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
    if (VARIANT != 1 && VARIANT != 6) asm volatile("s_waitcnt vmcnt(0)" : "+v"(b_prev)::"memory");
    if (have_prev && VARIANT != 1) write_out(cur ^ 1);
    if (ovf) atomicOr(a.overflow, 1u);
}

// Pass 2: LDS histogram of partition p = blockIdx.y over a group of regions
// (x / nslices) and one slice of each region (x % nslices), then one coalesced
// atomic flush of the 32768-bucket table into counts.
__global__ __launch_bounds__(P2_THREADS, 4) void k_pass2(const uint16_t *ids, const uint32_t *cursor,
                                                         const uint32_t *overflow, uint64_t cap,
                                                         uint32_t nparts, uint32_t nregions, uint32_t rpw,
                                                         uint32_t nslices, uint32_t slice,
                                                         uint64_t num_buckets, uint32_t *counts) {
    __shared__ uint32_t hist[PART_BUCKETS];
    if (*overflow) return;
    const int tid = threadIdx.x;
    const uint32_t p = blockIdx.y;
    const uint32_t grp = blockIdx.x / nslices, sl = blockIdx.x % nslices;
    const uint32_t r0 = grp * rpw, r1 = min(nregions, r0 + rpw);
    const uint64_t lo = (uint64_t)sl * slice;
    bool any = false;
    for (uint32_t r = r0; r < r1; ++r) any |= min((uint64_t)cursor[(uint64_t)r * nparts + p], cap) > lo;
    if (!any) return;
    for (int i = tid; i < PART_BUCKETS; i += P2_THREADS) hist[i] = 0;
    __syncthreads();
    for (uint32_t r = r0; r < r1; ++r) {
        const uint64_t fill = min((uint64_t)cursor[(uint64_t)r * nparts + p], cap);
        if (fill <= lo) continue;
        const uint64_t hi = min(fill, lo + slice);
        const uint16_t *src = ids + ((uint64_t)r * nparts + p) * cap;
        // lo and cap are multiples of 8: 16-B aligned vectors
        const uint64_t nvec = (hi - lo) >> 3;
        const uint4 *v = reinterpret_cast<const uint4 *>(src + lo);
        for (uint64_t i = tid; i < nvec; i += P2_THREADS) {
            const uint4 w = ntload16(v + i);
            atomicAdd(&hist[w.x & 0xFFFF], 1u); atomicAdd(&hist[w.x >> 16], 1u);
            atomicAdd(&hist[w.y & 0xFFFF], 1u); atomicAdd(&hist[w.y >> 16], 1u);
            atomicAdd(&hist[w.z & 0xFFFF], 1u); atomicAdd(&hist[w.z >> 16], 1u);
            atomicAdd(&hist[w.w & 0xFFFF], 1u); atomicAdd(&hist[w.w >> 16], 1u);
        }
        for (uint64_t i = lo + nvec * 8 + tid; i < hi; i += P2_THREADS) atomicAdd(&hist[src[i]], 1u);
    }
    __syncthreads();
    const uint64_t b0 = (uint64_t)p << PART_SHIFT;
    const uint32_t nb = (uint32_t)min((uint64_t)PART_BUCKETS, num_buckets - b0);
    for (uint32_t i = tid; i < nb; i += P2_THREADS) {
        const uint32_t h = hist[i];
        if (h) atomicAdd(counts + b0 + i, h);
    }
}

// Fallback when pass 1 overflowed a region (adversarial key sets): recount the
// whole launch with direct atomics.  Exits immediately in the normal case.
template <int SRC, int LFIX>
__global__ __launch_bounds__(P1_THREADS) void k_overflow_fallback(P1Args a) {
    if (*a.overflow == 0) return;
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
    const uint32_t *cursor;    // fills [R][P]
    const uint32_t *overflow;
    uint64_t cap, cap_tail;    // ids per segment of a main / tail region
    uint32_t nparts, nmain, ntail;
    uint64_t num_buckets;
    uint32_t *counts;
};

__device__ __forceinline__ uint64_t p2_seg_base(const P2Layout &L, uint32_t p, uint32_t r) {
    return r < L.nmain ? ((uint64_t)r * L.nparts + p) * L.cap
                       : (uint64_t)L.nmain * L.nparts * L.cap + ((uint64_t)(r - L.nmain) * L.nparts + p) * L.cap_tail;
}

constexpr int P2_ITEMS_PER_THREAD = 16;  // items <= 1024*16: P*R <= 16384

// pref[k] = ids before item k (exclusive), pref[NI] = total.  One workgroup.
__global__ __launch_bounds__(SCAN_THREADS) void k_pass2_plan(P2Layout L, uint64_t *pref) {
    __shared__ uint64_t wsum[SCAN_THREADS / 64];
    const uint32_t R = L.nmain + L.ntail, NI = L.nparts * R;
    const int tid = threadIdx.x;
    uint64_t f[P2_ITEMS_PER_THREAD], s = 0;
#pragma unroll
    for (int j = 0; j < P2_ITEMS_PER_THREAD; ++j) {
        const uint32_t k = tid * P2_ITEMS_PER_THREAD + j;
        f[j] = 0;
        if (k < NI) {
            const uint32_t p = k / R, r = k % R;
            f[j] = min((uint64_t)L.cursor[(uint64_t)r * L.nparts + p], r < L.nmain ? L.cap : L.cap_tail);
        }
        s += f[j];
    }
    uint64_t tot;
    uint64_t run = block_excl_scan64(s, wsum, tid, tot);
#pragma unroll
    for (int j = 0; j < P2_ITEMS_PER_THREAD; ++j) {
        const uint32_t k = tid * P2_ITEMS_PER_THREAD + j;
        if (k < NI) pref[k] = run;
        run += f[j];
    }
    if (tid == 0) pref[NI] = tot;
}

__global__ __launch_bounds__(P2_THREADS, 1) void k_pass2b(P2Layout L, const uint64_t *pref) {
    __shared__ uint32_t hist[PART_BUCKETS];
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
    int64_t cur_p = -1;
    for (uint32_t k = k_start; k < NI; ++k) {
        const uint64_t pk = pref[k], pk1 = pref[k + 1];
        if (pk >= hi) break;
        const uint64_t a = max(lo, pk) - pk, b = min(hi, pk1) - pk;
        if (a >= b) continue;
        const uint32_t p = k / R, r = k % R;
        if ((int64_t)p != cur_p) {
            if (cur_p >= 0) flush((uint32_t)cur_p);
            cur_p = p;
        }
        // segment base is a multiple of 64 ids: 16-byte vectors from a8 on
        const uint16_t *src = L.ids + p2_seg_base(L, p, r);
        const uint64_t a8 = min(b, (a + 7) & ~7ULL), b8 = max(a8, b & ~7ULL);
        // an id with the top bit set is a pad (ID_PAD): it adds 0
        auto add_id = [&](uint32_t id) { atomicAdd(&hist[id & 0x7FFF], 1u - (id >> 15)); };
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
