// gov_kernels.hip -- GOV MPHF construction on gfx950: bucket sort (A5),
// per-bucket solve (A8).  One workgroup owns one bucket at a time.
//
// The algorithm is the oracle's (oracle/bsdb_oracle.c, "GOV build"), step for
// step, so the device output is bit-identical to it:
//   edges   signatureToEquation(sorted sig, j<<56, nv)       (mph.c:63-71)
//   peel    rounds: every degree-1 vertex claims its edge (smallest wins)
//   orient  greedy first-free vertex in edge order (wave 0, 64 edges per
//           step resolved in registers) + BFS augmenting paths (wave 0)
//   solve   core blocks = SCCs of the hinge dependency graph (the big one
//           by forward/backward reach sweeps of the workgroup, the rest by
//           Tarjan on lane 0); small blocks Gauss-Jordan over F3 with the
//           whole workgroup (bit-sliced rows in a per-workgroup global
//           scratch), large ones through a feedback vertex set (Kahn
//           selection on wave 0, affine forms by dependency level, the heavy
//           system in LDS); peeled edges by rounds
//   store   hinge value or 3 if 0, non-hinge 0 (GOV:126-139); local seed in
//           the top 8 bits of edgeOffsetAndSeed[b] (GOV:434-436)
// The reference's own solver (sux4j 5.4.1 Linear3SystemSolver) is not
// available: its specific solution is parity-unpinned.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mph_kernels.hip"
#include "spooky_dev.hpp"

namespace bsdb {

#ifndef GOV_THREADS
#define GOV_THREADS 512  // workgroup size of the solver
#endif
constexpr int GS_THREADS = GOV_THREADS;
// Two solver workgroups per CU (LDS <= 80 KiB each): one's single-wave
// phases (greedy, BFS, FVS selection) overlap the other's.  4.2 sigma above
// the mean bucket; larger buckets (~1e-5 of them) take the global-slab path.
#ifndef GOV_PER_CU
#define GOV_PER_CU 2
#endif
#ifndef GOV_CMAX
#define GOV_CMAX 1664
#endif
// (GOV_PER_CU / GOV_CMAX other than 2 / 1664: measurement builds only,
// tools/build_variant.sh, with BSDB_PROBE_BUCKET_SIZE)
constexpr int GS_PER_CU = GOV_PER_CU;
constexpr int GS_CMAX = GOV_CMAX;    // keys per bucket solved in LDS (expected ~1500, sigma ~39)
constexpr int GS_NVMAX = GS_CMAX + GS_CMAX / 8;   // > vertex_offset span of GS_CMAX keys (1872)
constexpr int GS_TINY = 12;      // brute-force buckets (only in sets of < ~1500 keys)
#ifndef GOV_GJ_REG
// the heavy system's Gauss-Jordan in registers (gauss_jordan_reg): needs the
// VGPRs of two waves per SIMD (256-thread workgroups, two per CU)
#define GOV_GJ_REG (GOV_THREADS <= 256)
#endif
#ifndef GOV_GJ_REG_HW
#define GOV_GJ_REG_HW 6  // the widest heavy rows (64-bit words a plane) the register form takes
#endif
#ifndef GOV_GJ_FOLLOW
#define GOV_GJ_FOLLOW 1  // panel form: recorded pivots a following wave takes at once (2, 4, 8: slower)
#endif
#ifndef GOV_GJ_B2
#define GOV_GJ_B2 4  // panel form: a panel's columns a row's trailing update takes at once (a power of two)
#endif
#ifndef GOV_GJ_SLEEP
#define GOV_GJ_SLEEP 1   // panel form: s_sleep of a following wave that waits for the leader
#endif
#ifndef GOV_GJ_PANEL
// the heavy system's Gauss-Jordan by 64-column panels, pivots found by the
// leader wave (gauss_jordan_panel): bit-identical; C2 solve -10 %
#define GOV_GJ_PANEL 1
#endif
// LDS words of the panel form's scratch for n unknowns: the waves' pivot
// slots (5 words each), a panel's recorded pivots (4 words a column), the
// trailing update's table (9 entries of both planes for each of a panel's 32
// column pairs)
__host__ __device__ constexpr size_t gj_panel_words(uint32_t n) {
    return (size_t)(GOV_THREADS / 64) * 5 + (size_t)4 * 64 + (size_t)2 * 32 * 9;  // slots, pinfo, the pair table
}
#ifndef GOV_GREEDY_BRANCHFREE
#define GOV_GREEDY_BRANCHFREE 1  // greedy steps without exec-mask branches (dead-word stores)
#endif
#ifndef GOV_BACK_NOBARRIER
#define GOV_BACK_NOBARRIER 0  // peeled edges solved as their vertices become final, no barrier per round (back -23 %, the solve +0.3 %: more spills; not kept)
#endif
#ifndef GOV_SWEEP_INNER
#define GOV_SWEEP_INNER 1  // SCC reach sweeps: rounds of reads and marks per barrier (2: half the barriers, sweeps -13 %, the solve unchanged; not kept)
#endif
#ifndef GOV_CLOSURE_BRANCHFREE
#define GOV_CLOSURE_BRANCHFREE 1  // FVS closure batches without exec-mask branches (dead-word stores)
#endif
#ifndef GOV_BFS_BRANCHFREE
#define GOV_BFS_BRANCHFREE 1  // BFS rounds without exec-mask branches (dead-word stores)
#endif
#ifndef GOV_GREEDY_ROUNDS
#define GOV_GREEDY_ROUNDS 1  // greedy: a chunk's overlapping lanes decided in rounds (0: one at a time)
#endif
#ifndef GOV_GREEDY_CHUNK
#define GOV_GREEDY_CHUNK 64  // core edges the greedy orientation takes a step (wave 0)
#endif
#ifndef GOV_PICK_REPS
// FVS: pairs of heavy hinges taken per stuck cascade (with the in x out pick
// key, C2 at 6 / 8 / 12 / 16 / 20 / 24 / 28: 522 / 536 / 553 / 558 / 566–569 /
// 565 / 560 M keys/s, profiles/r4/pick_size_ab/, solver_sweep/; round 6, with
// the four-Russians trailing update: C2 gov 20 / 24 / 28 pairs 122.2 / 121.2 /
// 123.2 ms, profiles/r6/solver/)
#define GOV_PICK_REPS 24
#endif
constexpr int GS_WMAX = (GS_CMAX + 1 + 63) / 64;  // words per bit-sliced row
// Oversized buckets (adversarial or skewed key sets: > GS_CMAX keys, 14 sigma
// above the mean for random keys) are solved by the same code with its state
// in a per-workgroup slab of global memory, up to GB_CMAX keys.
constexpr int GB_CMAX = 16384;  // a power of two (the bitonic sort's padding)
// Oversized buckets up to GM_CMAX keys (every one of a random key set: the
// largest of C4's 8.8 M buckets holds ~1 720) are solved with their state in
// LDS by k_gov_solve_mid, one workgroup per CU; only larger (adversarial)
// buckets take the global-slab kernel, whose every state access goes to L2.
constexpr int GM_CMAX = 2048;
constexpr int GB_THREADS = 256;  // sort of an oversized bucket
// FVS: most heavy hinges of a block (a larger set falls back to Gauss-Jordan
// over the whole block).  SolveArgs::fvs_max may lower it (tests force the
// fallback with it); the result is the block's unique solution either way.
constexpr uint32_t FVS_NH_MAX = 380;
// FVS blocks whose heavy system is singular but consistent: at most NB_MAX
// null vectors are reduced in place (more fall back to Gauss-Jordan over the
// whole block, which reaches the same solution)
constexpr uint32_t NB_MAX = 128;

enum GovStatus : uint32_t { GOV_TOO_BIG = 1u, GOV_SEEDS = 2u, GOV_DUP = 4u, GOV_VERIFY = 8u };

// ---- A5: signatures grouped by bucket, sorted by unsigned (sig0, sig1) -------
// A build covers the buckets [b0, b0 + nb) of a GOV structure over all the
// keys (one GPU: b0 = 0, nb = m; a rank of the multi-GPU build, DESIGN.md
// §6: its bucket range).  Eb = E + b0 holds GLOBAL offsets (e0 = the keys in
// buckets below b0); the local signatures occupy positions E[b] - e0.
__global__ __launch_bounds__(256) void k_bucket_count(const uint64_t *sig, uint64_t n, uint32_t mult, uint32_t b0,
                                                      uint32_t *counts) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
        atomicAdd(counts + (bucket_of_w(w64(sig[2 * i]), mult) - b0), 1u);
}

// E[b0 + i] = e0 + local exclusive prefix (written by the scan at Eb)
__global__ __launch_bounds__(256) void k_add_base(uint64_t *Eb, uint64_t cnt, uint64_t e0) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < cnt; i += stride) Eb[i] += e0;
}

__global__ __launch_bounds__(256) void k_cursor_init(const uint64_t *Eb, uint64_t nb, uint64_t e0, uint64_t *cursor) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x; b < nb; b += stride) cursor[b] = (Eb[b] & OFFSET_MASK) - e0;
}

// pay_out (optional): the input position of each sorted signature (F2: the
// solver then writes each input's rank without a lookup pass)
__global__ __launch_bounds__(256) void k_bucket_scatter(const uint64_t *sig, uint64_t n, uint32_t mult, uint32_t b0,
                                                        unsigned long long *cursor, uint64_t *out, uint64_t *pay_out) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const ulonglong2 s = reinterpret_cast<const ulonglong2 *>(sig)[i];
        const uint64_t pos = atomicAdd(cursor + (bucket_of_w(w64(s.x), mult) - b0), 1ULL);
        reinterpret_cast<ulonglong2 *>(out)[pos] = s;
        if (pay_out) pay_out[pos] = i;
    }
}

// The same two steps for a range of at most SMALL_NB buckets (C1: 667), where
// one global atomic per key serialises on few addresses (C1: 0.26 + 0.20 ms
// for 1e6 keys): a workgroup counts a chunk of SMALL_CHUNK consecutive keys
// in LDS, then adds one count per bucket (count) or reserves one run per
// bucket with one cursor atomic and places each key at its LDS rank in that
// run (scatter).  The order inside a bucket stays arbitrary until
// k_bucket_sort, as with the per-key atomics.
constexpr uint32_t SMALL_NB = 4096, SMALL_KPT = 16, SMALL_CHUNK = 256 * SMALL_KPT;

__global__ __launch_bounds__(256) void k_bucket_count_small(const uint64_t *sig, uint64_t n, uint32_t mult, uint32_t b0,
                                                            uint32_t nb, uint32_t *counts) {
    __shared__ uint32_t c[SMALL_NB];
    for (uint32_t i = threadIdx.x; i < nb; i += 256) c[i] = 0;
    __syncthreads();
    const uint64_t lo = (uint64_t)blockIdx.x * SMALL_CHUNK;
#pragma unroll
    for (uint32_t j = 0; j < SMALL_KPT; ++j) {
        const uint64_t i = lo + j * 256 + threadIdx.x;
        if (i < n) atomicAdd(&c[bucket_of_w(w64(sig[2 * i]), mult) - b0], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nb; i += 256)
        if (c[i]) atomicAdd(counts + i, c[i]);
}

__global__ __launch_bounds__(256) void k_bucket_scatter_small(const uint64_t *sig, uint64_t n, uint32_t mult, uint32_t b0,
                                                              uint32_t nb, unsigned long long *cursor, uint64_t *out,
                                                              uint64_t *pay_out) {
    __shared__ uint32_t c[SMALL_NB];
    __shared__ unsigned long long base[SMALL_NB];
    for (uint32_t i = threadIdx.x; i < nb; i += 256) c[i] = 0;
    __syncthreads();
    const uint64_t lo = (uint64_t)blockIdx.x * SMALL_CHUNK;
    uint32_t bk[SMALL_KPT], rk[SMALL_KPT];
#pragma unroll
    for (uint32_t j = 0; j < SMALL_KPT; ++j) {
        const uint64_t i = lo + j * 256 + threadIdx.x;
        bk[j] = 0xFFFFFFFFu;
        if (i < n) {
            bk[j] = bucket_of_w(w64(sig[2 * i]), mult) - b0;
            rk[j] = atomicAdd(&c[bk[j]], 1u);
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nb; i += 256)
        if (c[i]) base[i] = atomicAdd(cursor + i, (unsigned long long)c[i]);
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < SMALL_KPT; ++j) {
        const uint64_t i = lo + j * 256 + threadIdx.x;
        if (bk[j] == 0xFFFFFFFFu) continue;
        const uint64_t pos = base[bk[j]] + rk[j];
        reinterpret_cast<ulonglong2 *>(out)[pos] = reinterpret_cast<const ulonglong2 *>(sig)[i];
        if (pay_out) pay_out[pos] = i;
    }
}

// Mid-size ranges (SMALL_NB < nb <= MID_NB, C2: 66 667 buckets), with no
// per-key global atomics (1e8 of them on random addresses: 4.1 ms for the
// count, 6.9 ms with the scatter's stores at C2):
//  1. k_bucket_count_mid: g workgroups (one per CU) each count their keys
//     (a fixed grid-stride share) into 16-bit LDS counters (two per word,
//     the whole range in 160 KB) and store them as cw[w][b];
//  2. k_mid_colsum: counts[b] = sum over w of cw[w][b];
//  3. (the offsets scan: E)
//  4. k_mid_colscan: base[w][b] = E[b] - e0 + sum over w' < w of cw[w'][b];
//  5. k_bucket_scatter_mid: the same workgroups, the same shares, place each
//     key at base[w][b] + its LDS rank among w's keys of bucket b.
// Positions are then a function of the input alone.  A counter that reaches
// 0x8000 in one workgroup (an adversarial set; random keys put ~3 per bucket
// in a share) raises *flag before its half could carry into its neighbour:
// k_bucket_count_redo then recounts with per-key atomics and the scatter
// falls back to cursor atomics.
constexpr uint32_t MID_NB = 80000, MID_THREADS = 1024;

__global__ __launch_bounds__(MID_THREADS) void k_bucket_count_mid(const uint64_t *sig, uint64_t n, uint32_t mult,
                                                                  uint32_t b0, uint32_t nb, uint16_t *cw,
                                                                  uint32_t *flag) {
    __shared__ uint32_t c2[MID_NB / 2];
    const uint32_t nw = (nb + 1) / 2;
    for (uint32_t i = threadIdx.x; i < nw; i += MID_THREADS) c2[i] = 0;
    __syncthreads();
    bool over = false;
    const uint64_t stride = (uint64_t)gridDim.x * MID_THREADS;
    for (uint64_t i = (uint64_t)blockIdx.x * MID_THREADS + threadIdx.x; i < n; i += stride) {
        const uint32_t b = bucket_of_w(w64(sig[2 * i]), mult) - b0, sh = (b & 1) * 16;
        const uint32_t old = atomicAdd(&c2[b >> 1], 1u << sh);
        over |= ((old >> sh) & 0xFFFFu) >= 0x7FFFu;
    }
    if (over) atomicOr(flag, 1u);
    __syncthreads();
    uint16_t *row = cw + (size_t)blockIdx.x * nb;
    for (uint32_t b = threadIdx.x; b < nb; b += MID_THREADS) row[b] = (uint16_t)(c2[b >> 1] >> ((b & 1) * 16));
}

__global__ __launch_bounds__(256) void k_mid_colsum(const uint16_t *cw, uint32_t g, uint32_t nb, uint32_t *counts) {
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    if (b >= nb) return;
    uint32_t t = 0;
    for (uint32_t w = 0; w < g; ++w) t += cw[(size_t)w * nb + b];
    counts[b] = t;
}

__global__ __launch_bounds__(256) void k_mid_colscan(const uint16_t *cw, uint32_t g, uint32_t nb, const uint64_t *Eb,
                                                     uint64_t e0, uint32_t *base) {
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    if (b >= nb) return;
    uint32_t run = (uint32_t)((Eb[b] & OFFSET_MASK) - e0);
    for (uint32_t w = 0; w < g; ++w) {
        base[(size_t)w * nb + b] = run;
        run += cw[(size_t)w * nb + b];
    }
}

__global__ __launch_bounds__(256) void k_bucket_count_redo(const uint64_t *sig, uint64_t n, uint32_t mult, uint32_t b0,
                                                           uint32_t nb, uint32_t *counts, const uint32_t *flag) {
    if (*flag == 0) return;  // (the normal case: nothing to do)
    // one workgroup clears, then counts (a grid-wide order one launch cannot give)
    if (blockIdx.x != 0) return;
    for (uint32_t b = threadIdx.x; b < nb; b += 256) counts[b] = 0;
    __syncthreads();
    for (uint64_t i = threadIdx.x; i < n; i += 256) atomicAdd(counts + (bucket_of_w(w64(sig[2 * i]), mult) - b0), 1u);
}

__global__ __launch_bounds__(MID_THREADS) void k_bucket_scatter_mid(const uint64_t *sig, uint64_t n, uint32_t mult,
                                                                    uint32_t b0, uint32_t nb, const uint32_t *base,
                                                                    const uint32_t *flag, unsigned long long *cursor,
                                                                    uint64_t *out, uint64_t *pay_out) {
    __shared__ uint32_t c2[MID_NB / 2];
    const uint64_t stride = (uint64_t)gridDim.x * MID_THREADS;
    if (*flag) {  // (uniform) the counts were redone: per-key cursor atomics
        for (uint64_t i = (uint64_t)blockIdx.x * MID_THREADS + threadIdx.x; i < n; i += stride) {
            const ulonglong2 s = reinterpret_cast<const ulonglong2 *>(sig)[i];
            const uint64_t pos = atomicAdd(cursor + (bucket_of_w(w64(s.x), mult) - b0), 1ULL);
            reinterpret_cast<ulonglong2 *>(out)[pos] = s;
            if (pay_out) pay_out[pos] = i;
        }
        return;
    }
    const uint32_t nw = (nb + 1) / 2;
    for (uint32_t i = threadIdx.x; i < nw; i += MID_THREADS) c2[i] = 0;
    __syncthreads();
    const uint32_t *bw = base + (size_t)blockIdx.x * nb;
    for (uint64_t i = (uint64_t)blockIdx.x * MID_THREADS + threadIdx.x; i < n; i += stride) {
        const ulonglong2 s = reinterpret_cast<const ulonglong2 *>(sig)[i];
        const uint32_t b = bucket_of_w(w64(s.x), mult) - b0, sh = (b & 1) * 16;
        const uint32_t rk = (atomicAdd(&c2[b >> 1], 1u << sh) >> sh) & 0xFFFFu;
        const uint64_t pos = (uint64_t)bw[b] + rk;
        reinterpret_cast<ulonglong2 *>(out)[pos] = s;
        if (pay_out) pay_out[pos] = i;
    }
}

__device__ __forceinline__ bool sig_less(ulonglong2 a, ulonglong2 b) { return a.x < b.x || (a.x == b.x && a.y < b.y); }

// Sort of one bucket (<= GS_CMAX keys) by unsigned (sig0, sig1) + duplicate
// check on neighbours (CBHS:969-972).  A bucket's sig0 are spread evenly over
// its slice of the 64-bit range (bucket = the high part of sig0 * 2m), so a
// counting sort on the top 11 bits of sig0 - min(sig0) puts ~0.8 keys in each
// of 2 048 sub-bins; each sub-bin is then insertion-sorted by one thread.  A
// handful of barriers per bucket instead of the 66 stages of a padded bitonic
// sort (10.4 ms at C2, bound by its LDS traffic).  Keys in registers (7 per
// thread), the placed keys in LDS: 48 KB, 3 workgroups per CU.  Adversarial
// sets (many keys in one sub-bin) only make that sub-bin's insertion slower.
__global__ __launch_bounds__(256) void k_bucket_sort(uint64_t *sig, const uint64_t *Eb, uint64_t nb, uint64_t e0,
                                                     uint32_t *status, uint64_t *pay) {
    constexpr uint32_t KPT = (GS_CMAX + 255) / 256, NBIN = 2048, BPT = NBIN / 256;
    __shared__ ulonglong2 o[GS_CMAX];
    __shared__ uint64_t op[GS_CMAX];  // payloads (pay != nullptr), moved with their signatures
    __shared__ uint32_t bin_off[NBIN + 1];
    __shared__ unsigned long long mn_mx[2];
    __shared__ uint32_t wsum[4];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (uint64_t b = blockIdx.x; b < nb; b += gridDim.x) {
        const uint64_t lo = (Eb[b] & OFFSET_MASK) - e0, hi = (Eb[b + 1] & OFFSET_MASK) - e0;
        const uint32_t cnt = (uint32_t)(hi - lo);
        if (cnt > GS_CMAX) continue;  // k_bucket_sort_big
        if (cnt < 2) continue;        // (uniform) nothing to order
        ulonglong2 *g = reinterpret_cast<ulonglong2 *>(sig) + lo;
        __syncthreads();  // (the previous bucket's LDS reads are done)
        for (uint32_t i = tid; i < NBIN; i += 256) bin_off[i] = 0;
        if (tid == 0) {
            mn_mx[0] = ~0ULL;
            mn_mx[1] = 0;
        }
        ulonglong2 v[KPT];
        uint64_t pv[KPT];
        unsigned long long lmn = ~0ULL, lmx = 0;
#pragma unroll
        for (uint32_t j = 0; j < KPT; ++j) {
            const uint32_t i = tid + 256 * j;
            v[j] = i < cnt ? g[i] : make_ulonglong2(0, 0);
            pv[j] = i < cnt && pay ? pay[lo + i] : 0;
            if (i < cnt) {
                lmn = min(lmn, (unsigned long long)v[j].x);
                lmx = max(lmx, (unsigned long long)v[j].x);
            }
        }
        __syncthreads();
        atomicMin(&mn_mx[0], lmn);
        atomicMax(&mn_mx[1], lmx);
        __syncthreads();
        const uint64_t mn = mn_mx[0], span = mn_mx[1] - mn;
        const uint32_t bits = span ? 64u - (uint32_t)__builtin_clzll(span) : 0u;  // span < 2^bits
        const uint32_t shift = bits > 11 ? bits - 11 : 0;                      // (x - mn) >> shift < 2048
        uint32_t rk[KPT];
#pragma unroll
        for (uint32_t j = 0; j < KPT; ++j)
            if (tid + 256 * j < cnt) rk[j] = atomicAdd(&bin_off[(uint32_t)((v[j].x - mn) >> shift)], 1u);
        __syncthreads();
        // exclusive scan of the 2 048 sub-bin counts: BPT per thread, then the waves
        uint32_t loc[BPT], tot = 0;
#pragma unroll
        for (uint32_t q = 0; q < BPT; ++q) {
            loc[q] = tot;
            tot += bin_off[tid * BPT + q];
        }
        uint32_t inc = tot;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)inc, d, 64);
            if (lane >= d) inc += y;
        }
        if (lane == 63) wsum[wave] = inc;
        __syncthreads();
        uint32_t wbase = 0;
        for (uint32_t w = 0; w < wave; ++w) wbase += wsum[w];
        const uint32_t base = wbase + inc - tot;
#pragma unroll
        for (uint32_t q = 0; q < BPT; ++q) bin_off[tid * BPT + q] = base + loc[q];
        if (tid == 0) bin_off[NBIN] = cnt;
        __syncthreads();
#pragma unroll
        for (uint32_t j = 0; j < KPT; ++j)
            if (tid + 256 * j < cnt) {
                const uint32_t p = bin_off[(uint32_t)((v[j].x - mn) >> shift)] + rk[j];
                o[p] = v[j];
                if (pay) op[p] = pv[j];
            }
        __syncthreads();
        // each sub-bin in order (insertion sort); equal neighbours are duplicates
        bool dup = false;
#pragma unroll
        for (uint32_t q = 0; q < BPT; ++q) {
            const uint32_t a0 = bin_off[tid * BPT + q], a1 = bin_off[tid * BPT + q + 1];
            for (uint32_t x = a0 + 1; x < a1; ++x) {
                const ulonglong2 key = o[x];
                const uint64_t kp = pay ? op[x] : 0;
                uint32_t y = x;
                while (y > a0 && sig_less(key, o[y - 1])) {
                    o[y] = o[y - 1];
                    if (pay) op[y] = op[y - 1];
                    --y;
                }
                o[y] = key;
                if (pay) op[y] = kp;
            }
            for (uint32_t x = a0 + 1; x < a1; ++x)
                if (o[x].x == o[x - 1].x && o[x].y == o[x - 1].y) dup = true;
        }
        __syncthreads();
        for (uint32_t i = tid; i < cnt; i += 256) {
            g[i] = o[i];
            if (pay) pay[lo + i] = op[i];
        }
        if (dup) atomicOr(status, (uint32_t)GOV_DUP);
    }
}

// Oversized buckets (> GS_CMAX keys): list them (status[3] counts them; a
// bucket over GB_CMAX keys cannot be solved and raises GOV_TOO_BIG).
__global__ __launch_bounds__(256) void k_big_list(const uint64_t *Eb, uint64_t nb, uint32_t *status, uint32_t *list,
                                                  uint32_t cap) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x; b < nb; b += stride) {
        const uint64_t cnt = (Eb[b + 1] & OFFSET_MASK) - (Eb[b] & OFFSET_MASK);
        if (cnt <= (uint64_t)GS_CMAX) continue;
        if (cnt > (uint64_t)GB_CMAX) {
            atomicOr(status, (uint32_t)GOV_TOO_BIG);
            continue;
        }
        const uint64_t nv = vertex_offset(Eb[b + 1] & OFFSET_MASK) - vertex_offset(Eb[b] & OFFSET_MASK);
        if (cnt > (uint64_t)GM_CMAX || nv > (uint64_t)(GM_CMAX + GM_CMAX / 8)) atomicAdd(status + 1, 1u);  // global-slab kernel
        const uint32_t i = atomicAdd(status + 3, 1u);
        if (i < cap) list[i] = (uint32_t)b;
    }
}

// The same bitonic sort + duplicate check for the listed oversized buckets, in
// a per-workgroup global slab of GB_CMAX entries (padded with sentinels).
__global__ __launch_bounds__(GB_THREADS) void k_bucket_sort_big(uint64_t *sig, const uint64_t *Eb, uint64_t e0,
                                                                const uint32_t *list, uint32_t nbig, ulonglong2 *slab,
                                                                uint32_t *status, uint64_t *pay) {
    ulonglong2 *s = slab + (size_t)blockIdx.x * GB_CMAX;
    uint64_t *sp = reinterpret_cast<uint64_t *>(slab + (size_t)gridDim.x * GB_CMAX) + (size_t)blockIdx.x * GB_CMAX;
    for (uint32_t li = blockIdx.x; li < nbig; li += gridDim.x) {
        const uint32_t b = list[li];
        const uint64_t lo = (Eb[b] & OFFSET_MASK) - e0, hi = (Eb[b + 1] & OFFSET_MASK) - e0;
        const uint32_t cnt = (uint32_t)(hi - lo);
        uint32_t p2 = 1;
        while (p2 < cnt) p2 <<= 1;
        ulonglong2 *g = reinterpret_cast<ulonglong2 *>(sig) + lo;
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < p2; i += GB_THREADS) {
            s[i] = i < cnt ? g[i] : make_ulonglong2(~0ULL, ~0ULL);
            if (pay) sp[i] = i < cnt ? pay[lo + i] : 0u;
        }
        __syncthreads();
        for (uint32_t k = 2; k <= p2; k <<= 1) {
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t i = threadIdx.x; i < p2; i += GB_THREADS) {
                    const uint32_t l = i ^ j;
                    if (l > i) {
                        const ulonglong2 a = s[i], c = s[l];
                        const bool up = (i & k) == 0;
                        if (up ? sig_less(c, a) : sig_less(a, c)) {
                            s[i] = c;
                            s[l] = a;
                            if (pay) {
                                const uint64_t t = sp[i];
                                sp[i] = sp[l];
                                sp[l] = t;
                            }
                        }
                    }
                }
                __syncthreads();
            }
        }
        bool dup = false;
        for (uint32_t i = threadIdx.x; i < cnt; i += GB_THREADS) {
            g[i] = s[i];
            if (pay) pay[lo + i] = sp[i];
            if (i && s[i].x == s[i - 1].x && s[i].y == s[i - 1].y) dup = true;
        }
        if (dup) atomicOr(status, (uint32_t)GOV_DUP);
    }
}

// ---- A8: per-bucket solve --------------------------------------------------
// Seeds of one bucket may be tried by several workgroups at once.  claim[b]
// hands out seed numbers in increasing order; a failed seed sets its bit in
// fail[b] (256 bits); a solved one max-es won[b] with 256 - seed (so won holds
// the lowest solved seed) and waits until every lower seed has failed (it is
// the bucket's seed: it stores the solution) or a lower one solved (it drops
// its own).  A lower seed's workgroup never waits on a higher one, and every
// handed-out seed is being tried by a resident workgroup, so the waits end.
struct SeedLedger {
    uint32_t *claim;          // [nb] next seed to hand out
    uint32_t *won;            // [nb] 256 - lowest solved seed, 0 = none yet
    unsigned long long *fail; // [nb][4] failed seeds
    uint32_t *done;           // [nb] 1 once the bucket's solution is stored (or its seeds ran out)
    uint32_t *active;         // [grid] the bucket each workgroup works on (0xFFFFFFFF = none)
};

struct SolveArgs {
    const uint64_t *sig;  // sorted signatures of buckets [b0, m), the first at global offset e0
    uint64_t m;           // end of the bucket range
    uint64_t *E;          // in: offsets; out: | seed << 56 (global bucket index)
    uint64_t *values;     // zeroed 2-bit value array (global vertex positions)
    uint64_t *scratch;    // per workgroup: solve_scratch_words<SolveLds>() words
    uint32_t *status;
    uint64_t *prof;       // optional per-workgroup phase cycle counters [grid][GP_N] (BSDB_GOV_PROFILE)
    uint32_t fvs_max;     // heavy-set limit, <= FVS_NH_MAX
    uint64_t b0, e0;      // first bucket of the range, keys before it
    // A11 + F2, fused into the solve: each key's rank is E[b] + the hinge
    // vertices before its hinge (exactly the lookup's count of nonzero
    // 2-bit values, GOV:557-580, as those sit at the hinges)
    uint64_t *sigbits;    // checksum bit list (width > 0): sig0 & mask at each rank (GOV:492-508)
    uint32_t width;
    const uint64_t *pay;  // input position of each sorted signature (rank_out / index_out)
    int64_t *rank_out;    // optional: rank of input signature i at [i]
    // optional, A13 fused into the solve (W:129-145): the key at input
    // position p has index.db slot r = its rank; index_out[r - idx_lo] =
    // byte-reversed address, addr[p] or addr_base + addr_stride * p
    uint64_t *index_out;
    uint64_t idx_lo;
    const uint64_t *addr;
    uint64_t addr_base, addr_stride;
    // the seed ledger of k_gov_solve (per bucket of the range, zeroed; active
    // per workgroup, all ones): workgroups with no bucket left try the next
    // seeds of buckets still being solved; the bucket's seed is still the
    // first one that solves it (GOV:425-432)
    SeedLedger led;
    // speculation policy: bits 0-7 = most seeds of one bucket in flight at
    // once for a speculating workgroup to add one (0 = no limit); bit 8 =
    // speculative attempts at a lower wave priority than a workgroup's own
    // bucket (BSDB_GOV_SPEC)
    uint32_t spec;
};


// phase counters (cycles, or counts for the GP_N_* slots)
enum GovProf { GP_EDGES, GP_PEEL, GP_GREEDY, GP_BFS, GP_TARJAN, GP_SINGLE, GP_DENSE, GP_BACK, GP_STORE,
               GP_N_SEEDS, GP_N_BFS, GP_N_BFS_POPS, GP_N_DENSE_ROWS, GP_N_DENSE_MAX, GP_N_CORE, GP_N_BLOCKS, GP_N_BIG_ROWS,
               GP_N_SCC_SWEEPS, GP_N_SMALL_S, GP_FVS_SEL, GP_FVS_FORMS, GP_FVS_GJ,
               GP_N_FAIL_DEGEN, GP_N_FAIL_ORIENT, GP_N_FAIL_INCONS, GP_FAILED_CYCLES, GP_BFS_FLIP, GP_N_BFS_ITERS,
               GP_N_FLIP_STEPS, GP_N_SEL_BATCHES, GP_N_SEL_PICKS, GP_SEL_PICK_CYCLES, GP_SEL_PREP_CYCLES,
               GP_N_SING_SOLVED, GP_N_NULL_VECS, GP_N_SPEC_LOST, GP_N_FVS_BLOCKS, GP_N_FORM_LEVELS, GP_N_HEAVY,
               GP_GJ_COLUMNS, GP_GJ_BARRIER, GP_GJ_ROWS_WAVE7, GP_TJ_PREP, GP_TJ_SWEEP, GP_TJ_COMPACT,
               GP_GJ_LEAD, GP_GJ_FOLLOW, GP_GJ_SLOTCOLS, GP_GJ_LEADCOLS, GP_GJ_TRAIL, GP_GJ_PANELS, GP_N };

// Solver state for buckets of up to CMAX_ keys: LDS for GS_CMAX, a global
// slab per workgroup for GB_CMAX (same code; indices fit int16 either way).
template <int CMAX_>
struct SolveLdsT {
    static constexpr int CMAX = CMAX_;
    static constexpr int NVMAX = CMAX_ + CMAX_ / 8;  // > vertex_offset span of CMAX keys (281/256)
    static constexpr int WMAX = (CMAX_ + 1 + 63) / 64;
    static_assert(CMAX_ < 32767, "int16 edge indices");
    // one region: the pivot row (Gauss-Jordan), a0, b0 and b1 -- and, during
    // the FVS selection (none of those live), the u32 pending counts (pend())
    uint64_t prow[2 * WMAX];
    int16_t a0[CMAX];
    uint8_t b0[NVMAX], b1[CMAX];
    // another: deg, claim, dep, a1, a3 -- dead once an FVS block's forms are
    // built, when it holds the heavy system (hs(), word-major)
    alignas(8) uint32_t deg[NVMAX];
    uint32_t claim[CMAX];
    int16_t dep[3 * CMAX];   // Tarjan: owner of edge k's i-th non-hinge vertex, or -1
    int16_t a1[CMAX], a3[CMAX];
    uint16_t e[3 * CMAX];
    uint32_t xe[NVMAX];
    int16_t hinge[CMAX];
    int16_t round_of[CMAX];
    int16_t vowner[NVMAX];
    uint8_t xval[NVMAX];
    int16_t a2[CMAX];        // (orientation BFS / Tarjan arrays a0-a3 are not live together)
    int16_t members[CMAX];   // components, in emission order
    int16_t comp_end[CMAX];  // end (exclusive) of component c in members
    int16_t col_of[CMAX];
    uint32_t ncomp, flag, pivot, rounds, chg, nleft, nscc, qtail;
    uint32_t nfree, npos;    // Gauss-Jordan: free columns; null-space reduction: last nonzero + 1
    uint32_t hbin[64];       // FVS selection: open members per in-degree
    __device__ uint32_t *pend() { return reinterpret_cast<uint32_t *>(prow); }
    __device__ uint64_t *hs() { return reinterpret_cast<uint64_t *>(deg); }
    static constexpr size_t HS_WORDS = (4 * (size_t)NVMAX + 4 * CMAX + 6 * CMAX + 2 * CMAX + 2 * CMAX) / 8;
    static constexpr size_t PEND_ROOM = sizeof(uint64_t) * 2 * WMAX + 2 * CMAX + NVMAX + CMAX;
    static_assert(PEND_ROOM >= 4 * (size_t)CMAX, "pending counts fit the pivot-row region");
    static_assert(NVMAX >= CMAX + 1 + 64, "the FVS pick's wave counts fit past the reverse CSR offsets");
};
using SolveLds = SolveLdsT<GS_CMAX>;
using SolveBig = SolveLdsT<GB_CMAX>;
using SolveMid = SolveLdsT<GM_CMAX>;
static_assert(SolveMid::NVMAX == GM_CMAX + GM_CMAX / 8, "k_big_list's mid test");
static_assert(sizeof(SolveMid) + 64 <= 160 * 1024, "k_gov_solve_mid: one workgroup per CU");
static_assert(SolveLds::NVMAX == GS_NVMAX && SolveLds::WMAX == GS_WMAX, "LDS layout");
static_assert(sizeof(SolveLds) + 64 <= 160 * 1024 / GS_PER_CU, "GS_PER_CU solver workgroups per CU");
// per-workgroup global scratch of the dense phase (bit-sliced rows, forms)
template <class Lds>
// FVS null vectors (bytes) at word 30 CMAX of the scratch, past the forms
// (words [16, 28) CMAX) and the reverse dependency CSR ([28, 29.5) CMAX):
// within the dense rows' words at production sizes
constexpr size_t solve_scratch_words() {
    const size_t dense = (size_t)2 * Lds::CMAX * Lds::WMAX, fvs = ((size_t)30 * 8 + NB_MAX) * Lds::CMAX / 8;
    return dense > fvs ? dense : fvs;
}
static_assert(GS_CMAX != 1664 || 30 * 8 + NB_MAX <= 8 * 2 * GS_WMAX, "FVS null-vector basis fits the dense scratch");

// a workgroup-uniform word read from LDS, as a scalar (the compiler treats
// LDS reads as per-lane; control flow on them is then exec-mask bookkeeping)
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

__device__ __forceinline__ uint64_t readfirstlane64(uint64_t x) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
}

__device__ __forceinline__ void gf3_add(uint64_t &x1, uint64_t &x2, uint64_t y1, uint64_t y2) {
    // one-hot planes (x1 = [x == 1], x2 = [x == 2]); or/xor form, 7 VALU per
    // 32-bit half (the and/or/not form took 9-12)
    const uint64_t t = (x1 | y2) ^ (x2 | y1);
    const uint64_t s1 = (x2 | y2) ^ t, s2 = (x1 | y1) ^ t;
    x1 = s1;
    x2 = s2;
}

// The single-wave phases (greedy and BFS orientation, the Tarjan walk, the
// singletons, the FVS closure, the Gauss-Jordan leader) hold up their whole
// workgroup: that wave takes the highest issue priority while it works, so
// the co-resident waves of the CU's other solver workgroup (throughput work)
// do not delay it at its SIMD.  GOV_PRIO=0 builds the form without.
#ifndef GOV_PRIO
#define GOV_PRIO 1
#endif
__device__ __forceinline__ void crit_on() {
    if (GOV_PRIO) __builtin_amdgcn_s_setprio(3);
}
__device__ __forceinline__ void crit_off() {
    if (GOV_PRIO) __builtin_amdgcn_s_setprio(0);
}

// Phase counters; P = false (production) compiles them away, so the
// profiling pointer and clock hold no registers in the solver.
template <bool P>
struct PhaseClock {
    uint64_t *acc;  // nullptr = off
    uint64_t t;
    __device__ bool on() const { return P && acc; }
    __device__ void start() { if (on()) t = clock64(); }
    __device__ void lap(int slot) {
        if (on()) {
            const uint64_t now = clock64();
            if (threadIdx.x == 0) acc[slot] += now - t;
            t = now;
        }
    }
    __device__ void add(int slot, uint64_t v) { if (on() && threadIdx.x == 0) acc[slot] += v; }
    __device__ void max(int slot, uint64_t v) { if (on() && threadIdx.x == 0 && v > acc[slot]) acc[slot] = v; }
    // from lane 0 of any wave (the counters are summed atomically)
    __device__ void add_any(int slot, uint64_t v) {
        if (on() && (threadIdx.x & 63) == 0) atomicAdd((unsigned long long *)(acc + slot), (unsigned long long)v);
    }
    __device__ uint64_t now() const { return on() ? clock64() : 0; }
};

// In-place exclusive scan of a[0..n) by the whole workgroup, 3 * GS_THREADS
// entries per round; wsum: 16 words of scratch.  Ends with a barrier.
__device__ void wg_excl_scan3(uint32_t *a, uint32_t n, uint32_t *wsum) {
    const uint32_t tid = threadIdx.x;
    uint32_t carry = 0;
    for (uint32_t r0 = 0; r0 < n; r0 += 3 * GS_THREADS) {
        const uint32_t i0 = r0 + 3 * tid;
        const uint32_t c0 = i0 < n ? a[i0] : 0, c1 = i0 + 1 < n ? a[i0 + 1] : 0, c2 = i0 + 2 < n ? a[i0 + 2] : 0;
        const uint32_t tot = c0 + c1 + c2;
        uint32_t inc = tot;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = (uint32_t)__shfl_up((int)inc, d, 64);
            if ((tid & 63) >= (uint32_t)d) inc += o;
        }
        if ((tid & 63) == 63) wsum[tid >> 6] = inc;
        __syncthreads();
        uint32_t base = carry, all = carry;
        for (uint32_t w = 0; w < GS_THREADS / 64; ++w) {
            const uint32_t s = wsum[w];
            if (w < (tid >> 6)) base += s;
            all += s;
        }
        const uint32_t ex = base + inc - tot;
        __syncthreads();
        if (i0 < n) a[i0] = ex;
        if (i0 + 1 < n) a[i0 + 1] = ex + c0;
        if (i0 + 2 < n) a[i0 + 2] = ex + c0 + c1;
        carry = all;
    }
    __syncthreads();
}

// Tries local seed j on bucket (sig, cnt, nv).  Returns (WG-uniform) true on
// success with L.xval / L.vowner describing the solution.
template <class Lds, class PC>
__device__ __forceinline__ bool try_seed(Lds &L, const ulonglong2 *sig, uint32_t cnt, uint32_t nv, uint64_t seed_bits,
                         uint64_t *scr, PC &pc, uint32_t fvs_max) {
    const int tid = threadIdx.x;
    // bit 31 (BSDB_GOV_PICK_EXACT, a test aid): every FVS pick by the exact
    // rounds of wave 0 instead of the binned one, a different heavy set
    const bool pick_exact = (fvs_max >> 31) != 0;
    fvs_max &= 0x7FFFFFFFu;
    pc.start();
    pc.add(GP_N_SEEDS, 1);
    const bool tiny = cnt <= GS_TINY;
    if (tid == 0) {
        L.flag = 0;
        L.pivot = 0;  // (core edges and core vertices after the peel, below)
        L.nscc = 0;
    }
    for (uint32_t v = tid; v < nv; v += GS_THREADS) {
        L.deg[v] = 0;
        L.vowner[v] = -1;
        L.xval[v] = 0;
    }
    __syncthreads();
    for (uint32_t k = tid; k < cnt; k += GS_THREADS) {
        const ulonglong2 s = sig[k];
        uint32_t e[3];
        sig_to_equation(s.x, s.y, seed_bits, nv, e);
        if (e[0] == e[1] && e[1] == e[2] && !tiny) L.flag = 1;
        for (int i = 0; i < 3; ++i) {
            L.e[3 * k + i] = (uint16_t)e[i];
            atomicAdd(&L.deg[e[i]], 1u);
        }
        L.hinge[k] = -1;
        L.round_of[k] = -1;
    }
    __syncthreads();
    pc.lap(GP_EDGES);
    if (uni(L.flag)) {
        pc.add(GP_N_FAIL_DEGEN, 1);
        return false;
    }
    if (cnt == 1 && nv == 1) {
        if (tid == 0) {
            L.vowner[0] = 0;
            L.hinge[0] = 0;
            L.xval[0] = 0;
        }
        __syncthreads();
        return true;
    }

    // ---- 1. peeling in rounds, from the edge side: an unpeeled edge with a
    // vertex of degree 1 is peeled in this round, its hinge the smallest such
    // vertex -- the edge every degree-1 vertex claims (its only remaining
    // one), the smallest claimant winning.  Two barriers a round (claims by
    // vertex took four), and the LDS solver's edges stay in registers.
    int r = 0;
    {
        constexpr uint32_t KPT = (Lds::CMAX + GS_THREADS - 1) / GS_THREADS;
        constexpr bool REG = KPT <= 4;  // (the global-slab instance reads its edges each round)
        constexpr uint32_t KR = REG ? KPT : 1;
        uint32_t pe[KR][3];
        uint32_t live = 0;  // (REG) bit j: edge tid + j * GS_THREADS not peeled
        if constexpr (REG) {
#pragma unroll
            for (uint32_t j = 0; j < KR; ++j) {
                const uint32_t k = tid + j * GS_THREADS;
                pe[j][0] = pe[j][1] = pe[j][2] = 0;
                if (k < cnt) {
                    live |= 1u << j;
                    pe[j][0] = L.e[3 * k];
                    pe[j][1] = L.e[3 * k + 1];
                    pe[j][2] = L.e[3 * k + 2];
                }
            }
        }
        auto try_peel = [&](uint32_t k, uint32_t v0, uint32_t v1, uint32_t v2) -> bool {
            const uint32_t d0 = L.deg[v0], d1 = L.deg[v1], d2 = L.deg[v2];
            uint32_t h = 0xFFFFFFFFu;
            if (d0 == 1u) h = v0;
            if (d1 == 1u) h = min(h, v1);
            if (d2 == 1u) h = min(h, v2);
            if (h == 0xFFFFFFFFu) return false;
            L.hinge[k] = (int16_t)h;
            L.vowner[h] = (int16_t)k;
            L.round_of[k] = (int16_t)r;
            return true;
        };
        for (;; ++r) {
            uint32_t newp = 0;
            if constexpr (REG) {
#pragma unroll
                for (uint32_t j = 0; j < KR; ++j)
                    if (((live >> j) & 1u) && try_peel(tid + j * GS_THREADS, pe[j][0], pe[j][1], pe[j][2]))
                        newp |= 1u << j;
                live &= ~newp;
            } else {
                for (uint32_t k = tid; k < cnt; k += GS_THREADS)
                    if (L.round_of[k] < 0 && try_peel(k, L.e[3 * k], L.e[3 * k + 1], L.e[3 * k + 2])) newp = 1;
            }
            if (!__syncthreads_or(newp != 0)) break;
            if constexpr (REG) {
#pragma unroll
                for (uint32_t j = 0; j < KR; ++j)
                    if ((newp >> j) & 1u)
                        for (int i = 0; i < 3; ++i) atomicSub(&L.deg[pe[j][i]], 1u);
            } else {
                for (uint32_t k = tid; k < cnt; k += GS_THREADS)
                    if (L.round_of[k] == r)
                        for (int i = 0; i < 3; ++i) atomicSub(&L.deg[L.e[3 * k + i]], 1u);
            }
            __syncthreads();
        }
    }
    const int rounds = r;
    pc.lap(GP_PEEL);
    // An orientation gives every core edge its own hinge among the core's
    // vertices, so a core with more edges than vertices has none: the seed
    // fails here (GOV:425-432, sux4j's unorientable), as the augmenting paths
    // below would find after the greedy and every BFS.  Measured on the
    // oracle's edges (3e5 keys' buckets, every seed up to the solving one),
    // this count catches every unorientable attempt of a random set, and they
    // are ~18 % of attempts.  Same outcome, so the same seeds and output.
    {
        uint32_t ce = 0, cv = 0;
        for (uint32_t k = tid; k < cnt; k += GS_THREADS) ce += L.round_of[k] < 0 ? 1u : 0u;
        for (uint32_t v = tid; v < nv; v += GS_THREADS) cv += L.deg[v] != 0u ? 1u : 0u;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            ce += (uint32_t)__shfl_xor((int)ce, d, 64);
            cv += (uint32_t)__shfl_xor((int)cv, d, 64);
        }
        if ((tid & 63) == 0) {
            atomicAdd(&L.pivot, ce);
            atomicAdd(&L.nscc, cv);
        }
        __syncthreads();
        const bool over = uni(L.pivot) > uni(L.nscc);  // (uniform; both words are next written after the BFS's barrier)
        if (over) {
            pc.add(GP_N_FAIL_ORIENT, 1);
            return false;
        }
    }

    // ---- 2. orientation of the core: greedy (wave 0), then BFS augmenting paths (wave 0).
    // A vertex is seen by BFS number `epoch` when seen[v] == epoch (the peel
    // degrees hold the greedy's counts first, then the stamps), so no BFS
    // clears the vertex array.
    uint32_t *seen = L.deg;
    // xe: the lowest lane of a chunk touching a vertex, as tag | lane with a
    // tag that DEcreases every chunk, so an atomicMin needs no reset between
    // chunks (a smaller value than every earlier chunk's)
    for (uint32_t v = tid; v < nv; v += GS_THREADS) L.xe[v] = ~0u;
    __syncthreads();
    uint32_t lane_tag = 0x3FFFFFFu << 6;  // (wave 0's register: 2^26 chunks per attempt)
    // Greedy: every core edge in increasing order takes, among its free
    // vertices, the one with the fewest core edges still to come (count =
    // the vertex's occurrences in core edges not yet processed, the peel's
    // degrees decremented as edges pass; ties: the first in the edge), then
    // decrements its three vertices.  (First-free instead left 12 % of the
    // core to augmenting paths, this 5 %: 126 -> 56 BFS per attempt.)
    // Wave 0 takes 64 edges at once: a lane none of whose vertices an
    // earlier lane of the chunk touches ("independent") decides at once
    // (nothing before it in the chunk changes its vertices' ownership or
    // counts, and it touches no vertex of an earlier lane); the others
    // resolve in edge order in registers after reloading ownership and
    // counts (which then hold every independent lane's effect -- an
    // independent lane shares no vertex with an earlier one, so those are
    // all earlier lanes): lane j's choice and vertices are broadcast, the
    // later lanes clear the chosen vertex and take j's decrements.
    // Together, the sequential outcome.
    if (tid < 64) {
        crit_on();  // (the one wave working: first at its SIMD)
        uint32_t *firstl = L.xe;  // (dead after peeling) lowest lane of the chunk touching a vertex
        uint32_t *ccnt = L.deg;   // core edges to come per vertex (the peel's degrees)
        auto pick = [](bool f0, bool f1, bool f2, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t v0, uint32_t v1,
                       uint32_t v2) -> int {
            int best = -1;
            uint32_t bc = 0xFFFFFFFFu;
            if (f0 && c0 < bc) { best = (int)v0; bc = c0; }
            if (f1 && c1 < bc) { best = (int)v1; bc = c1; }
            if (f2 && c2 < bc) { best = (int)v2; }
            return best;
        };
        // a chunk's edges and vertices are read one chunk ahead (neither
        // changes here), so a chunk starts at its ownership reads
#if GOV_GREEDY_BRANCHFREE
        // (every lane reads -- a lane past the edges reads edge 0 -- and the
        // lanes with nothing to do aim their atomics and stores at a dead
        // word of their own: no exec-mask branches in a step)
        uint32_t *const dead = L.hbin;  // (dead until the FVS selection, which clears them)
        int16_t *const dead16 = reinterpret_cast<int16_t *>(dead);
        auto chunk_edges = [&](uint32_t k, bool &a, uint32_t &u0, uint32_t &u1, uint32_t &u2) {
            const uint32_t kc = k < cnt ? k : 0u;
            const int ro = L.round_of[kc];
            u0 = L.e[3 * kc];
            u1 = L.e[3 * kc + 1];
            u2 = L.e[3 * kc + 2];
            a = k < cnt && ro < 0;
        };
#else
        auto chunk_edges = [&](uint32_t k, bool &a, uint32_t &u0, uint32_t &u1, uint32_t &u2) {
            a = k < cnt && L.round_of[k] < 0;
            u0 = u1 = u2 = 0;
            if (a) {
                u0 = L.e[3 * k];
                u1 = L.e[3 * k + 1];
                u2 = L.e[3 * k + 2];
            }
        };
#endif
        bool nact;
        uint32_t n0, n1, n2;
        // GOV_GREEDY_CHUNK edges a step (lanes above it idle): fewer lanes
        // whose vertices an earlier lane of the step touches, each of which
        // costs a serial step below
        constexpr uint32_t GCH = GOV_GREEDY_CHUNK;
        static_assert(GCH >= 1 && GCH <= 64, "greedy chunk");
        chunk_edges(tid < GCH ? tid : cnt, nact, n0, n1, n2);
        for (uint32_t k0 = 0; k0 < cnt; k0 += GCH) {
            const uint32_t k = k0 + tid;
            const bool act = nact;
            uint32_t v0 = n0, v1 = n1, v2 = n2, c0 = 0, c1 = 0, c2 = 0;
            chunk_edges(tid < GCH ? k + GCH : cnt, nact, n0, n1, n2);
            bool f0 = false, f1 = false, f2 = false;
            const uint32_t me = lane_tag | tid;
            lane_tag -= 64;
#if GOV_GREEDY_BRANCHFREE
            // decide: the lane's choice (or none) and its decrements, stores
            // aimed at the dead words unless `on`
            auto decide = [&](bool on, int &ch) {
                f0 = L.vowner[v0] < 0;
                f1 = L.vowner[v1] < 0;
                f2 = L.vowner[v2] < 0;
                c0 = ccnt[v0];
                c1 = ccnt[v1];
                c2 = ccnt[v2];
                const int c = pick(f0, f1, f2, c0, c1, c2, v0, v1, v2);
                const bool st = on && c >= 0;
                *(st ? &L.vowner[c < 0 ? 0 : c] : &dead16[tid]) = (int16_t)k;
                *(st ? &L.hinge[k] : &dead16[64 + tid]) = (int16_t)c;
                atomicSub(on ? &ccnt[v0] : &dead[tid], 1u);
                atomicSub(on ? &ccnt[v1] : &dead[tid], 1u);
                atomicSub(on ? &ccnt[v2] : &dead[tid], 1u);
                if (on) ch = c;
            };
            // (the first step's reads come before any of its stores: the
            // ownership and counts every lane sees are the chunk's start)
            f0 = L.vowner[v0] < 0;
            f1 = L.vowner[v1] < 0;
            f2 = L.vowner[v2] < 0;
            c0 = ccnt[v0];
            c1 = ccnt[v1];
            c2 = ccnt[v2];
            atomicMin(act ? &firstl[v0] : &dead[tid], me);
            atomicMin(act ? &firstl[v1] : &dead[tid], me);
            atomicMin(act ? &firstl[v2] : &dead[tid], me);
            __builtin_amdgcn_wave_barrier();
            const bool ovl = act && (firstl[v0] < me || firstl[v1] < me || firstl[v2] < me);
            int chosen = -1;
            {
                const bool on = act && !ovl;
                const int c = pick(f0, f1, f2, c0, c1, c2, v0, v1, v2);
                const bool st = on && c >= 0;
                *(st ? &L.vowner[c < 0 ? 0 : c] : &dead16[tid]) = (int16_t)k;
                *(st ? &L.hinge[k] : &dead16[64 + tid]) = (int16_t)c;
                atomicSub(on ? &ccnt[v0] : &dead[tid], 1u);
                atomicSub(on ? &ccnt[v1] : &dead[tid], 1u);
                atomicSub(on ? &ccnt[v2] : &dead[tid], 1u);
                if (on) chosen = c;
            }
            uint64_t todo = __builtin_amdgcn_ballot_w64(ovl);
            while (todo) {  // (wave-uniform) the overlapping lanes in rounds, as below
                const bool pend = ((todo >> tid) & 1ULL) != 0;
                const uint32_t me2 = lane_tag | tid;
                lane_tag -= 64;
                atomicMin(pend ? &firstl[v0] : &dead[tid], me2);
                atomicMin(pend ? &firstl[v1] : &dead[tid], me2);
                atomicMin(pend ? &firstl[v2] : &dead[tid], me2);
                __builtin_amdgcn_wave_barrier();
                const bool wait = pend && (firstl[v0] < me2 || firstl[v1] < me2 || firstl[v2] < me2);
                decide(pend && !wait, chosen);
                todo = __builtin_amdgcn_ballot_w64(wait);
                __builtin_amdgcn_wave_barrier();
            }
            (void)chosen;
#else
            if (act) {
                f0 = L.vowner[v0] < 0;
                f1 = L.vowner[v1] < 0;
                f2 = L.vowner[v2] < 0;
                c0 = ccnt[v0];
                c1 = ccnt[v1];
                c2 = ccnt[v2];
                atomicMin(&firstl[v0], me);
                atomicMin(&firstl[v1], me);
                atomicMin(&firstl[v2], me);
            }
            __builtin_amdgcn_wave_barrier();
            const bool ovl = act && (firstl[v0] < me || firstl[v1] < me || firstl[v2] < me);
            int chosen = -1;
            if (act && !ovl) {
                chosen = pick(f0, f1, f2, c0, c1, c2, v0, v1, v2);
                if (chosen >= 0) {
                    L.vowner[chosen] = (int16_t)k;
                    L.hinge[k] = (int16_t)chosen;
                }
                atomicSub(&ccnt[v0], 1u);
                atomicSub(&ccnt[v1], 1u);
                atomicSub(&ccnt[v2], 1u);
            }
            uint64_t todo = __builtin_amdgcn_ballot_w64(ovl);
#if GOV_GREEDY_ROUNDS
            // the overlapping lanes in rounds: a lane no earlier lane still
            // to decide shares a vertex with sees, after the previous rounds,
            // every earlier effect on its vertices, so it decides now (the
            // lanes of a round touch disjoint vertices); the rest wait
            while (todo) {  // (wave-uniform)
                const bool pend = ((todo >> tid) & 1ULL) != 0;
                const uint32_t me2 = lane_tag | tid;
                lane_tag -= 64;
                if (pend) {
                    atomicMin(&firstl[v0], me2);
                    atomicMin(&firstl[v1], me2);
                    atomicMin(&firstl[v2], me2);
                }
                __builtin_amdgcn_wave_barrier();
                const bool wait = pend && (firstl[v0] < me2 || firstl[v1] < me2 || firstl[v2] < me2);
                if (pend && !wait) {
                    f0 = L.vowner[v0] < 0;
                    f1 = L.vowner[v1] < 0;
                    f2 = L.vowner[v2] < 0;
                    c0 = ccnt[v0];
                    c1 = ccnt[v1];
                    c2 = ccnt[v2];
                    chosen = pick(f0, f1, f2, c0, c1, c2, v0, v1, v2);
                    if (chosen >= 0) {
                        L.vowner[chosen] = (int16_t)k;
                        L.hinge[k] = (int16_t)chosen;
                    }
                    atomicSub(&ccnt[v0], 1u);
                    atomicSub(&ccnt[v1], 1u);
                    atomicSub(&ccnt[v2], 1u);
                }
                todo = __builtin_amdgcn_ballot_w64(wait);
                __builtin_amdgcn_wave_barrier();
            }
#else
            if (todo) {  // (wave-uniform)
                __builtin_amdgcn_wave_barrier();
                if (ovl) {  // the independent lanes' choices and decrements (all earlier, see above)
                    f0 = L.vowner[v0] < 0;
                    f1 = L.vowner[v1] < 0;
                    f2 = L.vowner[v2] < 0;
                    c0 = ccnt[v0];
                    c1 = ccnt[v1];
                    c2 = ccnt[v2];
                }
                while (todo) {
                    const uint32_t j = (uint32_t)__builtin_ctzll(todo);
                    todo &= todo - 1;
                    if (tid == j) chosen = pick(f0, f1, f2, c0, c1, c2, v0, v1, v2);
                    const int c = __builtin_amdgcn_readlane(chosen, j);
                    const uint32_t w0 = __builtin_amdgcn_readlane(v0, j), w1 = __builtin_amdgcn_readlane(v1, j),
                                   w2 = __builtin_amdgcn_readlane(v2, j);
                    if (c >= 0) {
                        f0 = f0 && v0 != (uint32_t)c;
                        f1 = f1 && v1 != (uint32_t)c;
                        f2 = f2 && v2 != (uint32_t)c;
                    }
                    c0 -= (uint32_t)(v0 == w0) + (uint32_t)(v0 == w1) + (uint32_t)(v0 == w2);
                    c1 -= (uint32_t)(v1 == w0) + (uint32_t)(v1 == w1) + (uint32_t)(v1 == w2);
                    c2 -= (uint32_t)(v2 == w0) + (uint32_t)(v2 == w1) + (uint32_t)(v2 == w2);
                }
                if (ovl) {
                    if (chosen >= 0) {
                        L.vowner[chosen] = (int16_t)k;
                        L.hinge[k] = (int16_t)chosen;
                    }
                    atomicSub(&ccnt[v0], 1u);
                    atomicSub(&ccnt[v1], 1u);
                    atomicSub(&ccnt[v2], 1u);
                }
            }
#endif
#endif
            __builtin_amdgcn_wave_barrier();
        }
        // the counts' words become the BFS's stamps
        for (uint32_t v = tid; v < nv; v += 64) seen[v] = 0;
        __builtin_amdgcn_wave_barrier();
        pc.lap(GP_GREEDY);
        crit_off();
    }
    // BFS augmenting paths, one wave: the queue is consumed in chunks of up
    // to 21 edges, lane 3e+i taking vertex i of the chunk's edge e, which is
    // the sequential visit order; a vertex repeated in the chunk counts for
    // its lowest lane only (atomicMin over its stamp word), the first free
    // vertex in lane order ends the BFS (lanes after it do nothing, as the
    // sequential loop breaks there), and the newly reached owners are
    // appended in lane order.  Same queue, same marks, same path.  (Queue
    // entries carrying their edge's vertices, read by the appending lane, to
    // save the next chunk a round trip: BFS 7.15e6 -> 8.30e6 cycles, not kept.)
    if (tid < 64) {
        crit_on();  // (the one wave working: first at its SIMD)
        int16_t *bfs_prev = L.a0, *queue = L.a1;
        uint32_t *first_lane = L.xe;  // (dead after peeling)
        const uint32_t lane = tid;
        uint32_t epoch = 0, ok = 1, nbfs = 0, npops = 0, ncore = 0, niters = 0, nflip = 0;
        uint64_t flip_cyc = 0;
        if (pc.on())
            for (uint32_t k = 0; k < cnt; ++k) ncore += L.round_of[k] < 0;
        // unmatched core edges, 64 at a time by ballot (a BFS only matches its
        // own root: the path it flips runs through matched edges, so the
        // chunk's mask stays exact while its edges are taken in order)
        uint64_t pendm = 0;
        uint32_t base = 0;
        for (;;) {
            while (!pendm && base < cnt) {
                const uint32_t k = base + lane;
                bool un = false;
                if (k < cnt) {  // (both words read in one round trip)
                    const int ro = L.round_of[k], hi = L.hinge[k];
                    un = (ro < 0) & (hi < 0);
                }
                pendm = __builtin_amdgcn_ballot_w64(un);
                base += 64;
            }
            if (!pendm || !ok) break;
            const uint32_t k0 = base - 64 + (uint32_t)__builtin_ctzll(pendm);
            pendm &= pendm - 1;
            ++epoch;
            ++nbfs;
            if (lane == 0) {
                queue[0] = (int16_t)k0;
                bfs_prev[k0] = -1;
            }
            __builtin_amdgcn_wave_barrier();
            uint32_t qh = 0, qt = 1;
            int found_v = -1, found_e = -1;
            while (qh < qt && found_v < 0) {
                const uint32_t ch = min(21u, qt - qh);
                const bool act = lane < 3 * ch;
                const uint32_t ei = lane / 3, vi = lane - 3 * ei;
                const uint32_t me = lane_tag | lane;
                lane_tag -= 64;
#if GOV_BFS_BRANCHFREE
                // every lane reads (a lane past the chunk reads its last
                // edge) and the lanes past it aim their atomic and stores at
                // a dead word of their own: no exec-mask branches in a round
                uint32_t *const dead = L.hbin;  // (the FVS pick's bins: dead until the selection, which clears them)
                const int k = queue[qh + min(ei, ch - 1)];
                const uint32_t v = L.e[3 * k + vi];
                const uint32_t sn = seen[v];
                const int o = L.vowner[v];
                atomicMin(act ? &first_lane[v] : &dead[lane], me);
#else
                int k = 0, o = -1;
                uint32_t v = 0, sn = 0;
                if (act) {
                    k = queue[qh + ei];
                    v = L.e[3 * k + vi];
                    sn = seen[v];
                    o = L.vowner[v];
                    atomicMin(&first_lane[v], me);
                }
#endif
                __builtin_amdgcn_wave_barrier();
                // (the root's iteration without the queue read and the
                // atomics, duplicates compared in registers: BFS +2 %, not kept)
                const bool valid = act && first_lane[v] == me && sn != epoch;
                const uint64_t fb = __builtin_amdgcn_ballot_w64(valid && o < 0);
                const uint32_t F = fb ? (uint32_t)__builtin_ctzll(fb) : 64u;
                const bool take = valid && lane < F;  // (o >= 0 below F)
                const uint64_t tb = __builtin_amdgcn_ballot_w64(take);
#if GOV_BFS_BRANCHFREE
                {
                    const uint32_t pos = qt + __builtin_amdgcn_mbcnt_hi((uint32_t)(tb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)tb, 0u));
                    int16_t *const dead16 = reinterpret_cast<int16_t *>(dead);
                    *(valid && lane <= F ? &seen[v] : &dead[lane]) = epoch;
                    *(take ? &bfs_prev[o] : &dead16[lane]) = (int16_t)k;
                    *(take ? &queue[pos] : &dead16[64 + lane]) = (int16_t)o;
                }
#else
                if (valid && lane <= F) seen[v] = epoch;
                if (take) {
                    const uint32_t pos = qt + __builtin_amdgcn_mbcnt_hi((uint32_t)(tb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)tb, 0u));
                    bfs_prev[o] = (int16_t)k;
                    queue[pos] = (int16_t)o;
                }
#endif
                qt += (uint32_t)__builtin_popcountll(tb);
                qh += ch;
                npops += ch;
                ++niters;
                if (fb) {
                    found_v = __builtin_amdgcn_readlane((int)v, (int)F);
                    found_e = __builtin_amdgcn_readlane(k, (int)F);
                }
                __builtin_amdgcn_wave_barrier();
            }
            if (found_v < 0) {
                ok = 0;
                break;
            }
            const uint64_t tf = pc.on() ? clock64() : 0;
            if (lane == 0) {
                int k = found_e, v = found_v;
                for (;;) {
                    // (both reads of a step issued before its writes: one
                    // LDS round trip a step)
                    const int old = L.hinge[k], up = bfs_prev[k];
                    L.hinge[k] = (int16_t)v;
                    L.vowner[v] = (int16_t)k;
                    ++nflip;
                    if (k == (int)k0) break;
                    v = old;
                    k = up;
                }
            }
            if (pc.on()) flip_cyc += clock64() - tf;
            __builtin_amdgcn_wave_barrier();
        }
        if (lane == 0) {
            L.flag = ok;
            pc.add(GP_N_BFS, nbfs);
            pc.add(GP_N_BFS_POPS, npops);
            pc.add(GP_N_CORE, ncore);
            pc.add(GP_BFS_FLIP, flip_cyc);
            pc.add(GP_N_BFS_ITERS, niters);
            pc.add(GP_N_FLIP_STEPS, nflip);
        }
        crit_off();
    }
    __syncthreads();
    pc.lap(GP_BFS);
    if (!uni(L.flag)) {
        pc.add(GP_N_FAIL_ORIENT, 1);
        return false;
    }

    // ---- tiny buckets: first satisfying assignment in base-3 order (lane 0)
    if (tiny) {
        if (tid == 0) {
            uint32_t total = 1;
            for (uint32_t k = 0; k < cnt; ++k) total *= 3;
            uint32_t found = 0;
            for (uint32_t a = 0; a < total && !found; ++a) {
                uint32_t t = a;
                for (uint32_t k = 0; k < cnt; ++k) {
                    L.xval[L.hinge[k]] = (uint8_t)(t % 3);
                    t /= 3;
                }
                uint32_t okk = 1;
                for (uint32_t k = 0; k < cnt && okk; ++k) {
                    int h = 0;
                    while (L.e[3 * k + h] != (uint32_t)L.hinge[k]) ++h;
                    const uint32_t sum = L.xval[L.e[3 * k]] + L.xval[L.e[3 * k + 1]] + L.xval[L.e[3 * k + 2]];
                    okk = sum % 3 == (uint32_t)h;
                }
                found = okk;
            }
            L.flag = found;
        }
        __syncthreads();
        return L.flag != 0;
    }

    // ---- 3a. SCCs of the core dependency graph (lane 0, iterative Tarjan).
    // Edge k depends on the owners of its non-hinge vertices: precomputed by
    // the whole workgroup (hinges and owners are fixed from here on), so the
    // walk reads one word per neighbour instead of three dependent ones.
    for (uint32_t k = tid; k < cnt; k += GS_THREADS) {
        L.a0[k] = -1;     // tidx
        L.col_of[k] = -1;
        L.b0[k] = 0;      // onst
        if (L.round_of[k] < 0)
            for (int i = 0; i < 3; ++i) {
                const uint32_t v = L.e[3 * k + i];
                L.dep[3 * k + i] = (v != (uint32_t)L.hinge[k]) ? L.vowner[v] : (int16_t)-1;
            }
    }
    __syncthreads();
    // The core is nearly one strongly connected component (~97 % of its
    // edges).  That component is found by the whole workgroup: S = F & B,
    // F = edges reachable from a pivot along dependencies, B = edges that
    // reach it (fixpoint sweeps, one barrier each).  Tarjan on lane 0 then
    // only walks the rest: first from roots in F \ S (closed under
    // dependencies), then S as one component, then from the other roots
    // (F is finished by then).  SCCs are unique and this is a valid
    // dependency order, and a nonsingular block has one solution, so the
    // values are those of a whole-core Tarjan.
    // bit 0: in F, bit 1: in B, a word an edge (claim is dead after peeling;
    // 16 edges packed a word measured slower: the ORs then meet on one word)
    uint32_t *fbw = L.claim;
    auto fb = [&](uint32_t k) -> uint32_t { return fbw[k]; };
    auto fb_or = [&](uint32_t k, uint32_t bits) { atomicOr(&fbw[k], bits); };
    int16_t *roots = reinterpret_cast<int16_t *>(L.xe);  // Tarjan roots: F \ S, then the rest (dead after the BFS)
    if (tid == 0) {
        L.pivot = 0xFFFFFFFFu;
        L.nscc = 0;
    }
    for (uint32_t k = tid; k < cnt; k += GS_THREADS) fbw[k] = 0;
    __syncthreads();
    for (uint32_t k = tid; k < cnt; k += GS_THREADS)
        if (L.round_of[k] < 0) {
            atomicMin(&L.pivot, k);
            break;
        }
    __syncthreads();
    if (tid == 0 && L.pivot != 0xFFFFFFFFu) {
        crit_on();
        // follow first dependencies from the first core edge: the walk ends
        // on a cycle, almost surely inside the big component
        int p = (int)L.pivot;
        for (int step = 0; step < 64; ++step) {
            const int d0 = L.dep[3 * p], d1 = L.dep[3 * p + 1], d2 = L.dep[3 * p + 2];
            const int nx = d0 >= 0 ? d0 : d1 >= 0 ? d1 : d2;
            if (nx < 0) break;
            p = nx;
        }
        L.pivot = (uint32_t)p;
        fb_or((uint32_t)p, 3u);
        crit_off();
    }
    __syncthreads();
    pc.lap(GP_TJ_PREP);
    if (L.pivot != 0xFFFFFFFFu) {
        // a thread's edges and their dependencies stay in registers across the
        // sweeps, so a sweep is two rounds of independent LDS reads (the
        // edges' marks, then their dependencies') and fire-and-forget ORs
        // instead of a chain of dependent reads per edge
        constexpr uint32_t KPT = (Lds::CMAX + GS_THREADS - 1) / GS_THREADS;
        int dk[KPT][3];
#pragma unroll
        for (uint32_t j = 0; j < KPT; ++j) {
            const uint32_t k = tid + j * GS_THREADS;
            const bool core = k < cnt && L.round_of[k] < 0;
#pragma unroll
            for (int i = 0; i < 3; ++i) dk[j][i] = core ? (int)L.dep[3 * k + i] : -1;
        }
        // GOV_SWEEP_INNER rounds a barrier: a round's reads see this
        // thread's earlier marks and whatever other threads' marks have
        // landed, so a barrier covers up to that many levels; the marks only
        // grow, so the fixpoint (F, B) is the same, and a barrier interval
        // in which no thread marks anything ends the sweeps
        for (;;) {
          int ch = 0;
          for (uint32_t inner = 0; inner < GOV_SWEEP_INNER; ++inner) {
            uint32_t fk[KPT], fw[KPT][3];
#pragma unroll
            for (uint32_t j = 0; j < KPT; ++j) {
                const uint32_t k = tid + j * GS_THREADS;
                fk[j] = k < cnt ? fb(k) : 0u;
#pragma unroll
                for (int i = 0; i < 3; ++i) fw[j][i] = dk[j][i] >= 0 ? fb((uint32_t)dk[j][i]) : 0u;
            }
#pragma unroll
            for (uint32_t j = 0; j < KPT; ++j) {
                uint32_t nk = fk[j];
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    const int w = dk[j][i];
                    if (w < 0) continue;
                    if ((fk[j] & 1u) && !(fw[j][i] & 1u)) {  // F: push
                        fb_or((uint32_t)w, 1u);
                        ch = 1;
                    }
                    nk |= fw[j][i] & 2u;  // B: pull
                }
                if (nk & ~fk[j] & 2u) {
                    fb_or(tid + j * GS_THREADS, 2u);
                    ch = 1;
                }
            }
          }
            pc.add(GP_N_SCC_SWEEPS, 1);
            if (!__syncthreads_or(ch)) break;
        }
        uint32_t ns = 0;
        for (uint32_t k = tid; k < cnt; k += GS_THREADS) ns += fb(k) == 3u;
        if (ns) atomicAdd(&L.nscc, ns);
        __syncthreads();
    }
    pc.lap(GP_TJ_SWEEP);
    const bool big = uni(L.nscc) >= 64;  // (a small S: plain Tarjan over the whole core)
    if (!big) pc.add(GP_N_SMALL_S, 1);
    // ordered compaction (wave ballots, wave totals by barrier): class 0 =
    // F \ S roots, 1 = S (straight into members[], after the F \ S
    // components, which hold exactly |F \ S| members), 2 = the other roots
    uint32_t *wcnt = L.deg;  // 3 x 16 wave totals (the BFS stamps are dead)
    const uint32_t lane = tid & 63, wv = tid >> 6;
    uint32_t base0 = 0, base1 = 0, base2 = 0;
    for (int phase = 0; phase < 2; ++phase) {  // 0: class sizes; 1: positions
        uint32_t run0 = 0, run1 = 0, run2 = 0;
        for (uint32_t k0 = 0; k0 < cnt; k0 += GS_THREADS) {
            const uint32_t k = k0 + tid;
            uint32_t cl = 3;
            if (k < cnt && L.round_of[k] < 0) {
                const uint32_t f = big ? fb(k) : 0u;
                cl = f == 1u ? 0u : f == 3u ? 1u : 2u;
            }
            const uint64_t b0 = __builtin_amdgcn_ballot_w64(cl == 0), b1 = __builtin_amdgcn_ballot_w64(cl == 1),
                           b2 = __builtin_amdgcn_ballot_w64(cl == 2);
            if (lane == 0) {
                wcnt[wv] = (uint32_t)__builtin_popcountll(b0);
                wcnt[16 + wv] = (uint32_t)__builtin_popcountll(b1);
                wcnt[32 + wv] = (uint32_t)__builtin_popcountll(b2);
            }
            __syncthreads();
            uint32_t p0 = 0, p1 = 0, p2 = 0, t0 = 0, t1 = 0, t2 = 0;
            for (uint32_t w = 0; w < GS_THREADS / 64; ++w) {
                const uint32_t c0 = wcnt[w], c1 = wcnt[16 + w], c2 = wcnt[32 + w];
                if (w < wv) { p0 += c0; p1 += c1; p2 += c2; }
                t0 += c0; t1 += c1; t2 += c2;
            }
            if (phase == 1 && cl < 3) {
                const uint64_t bm = cl == 0 ? b0 : cl == 1 ? b1 : b2;
                const uint32_t r = (uint32_t)__builtin_popcountll(bm & ((1ULL << lane) - 1ULL));
                if (cl == 0) roots[base0 + run0 + p0 + r] = (int16_t)k;
                else if (cl == 1) {
                    L.members[base1 + run1 + p1 + r] = (int16_t)k;
                    L.a0[k] = 0x7FFF;  // S is finished for Tarjan (never on its stack)
                }
                else roots[base2 + run2 + p2 + r] = (int16_t)k;
            }
            run0 += t0; run1 += t1; run2 += t2;
            __syncthreads();
        }
        base1 = run0;             // S members follow the F \ S components
        base2 = run0;             // roots: F \ S, then the rest
        if (phase == 0) { L.rounds = run0; L.chg = run1; L.nleft = run2; }
    }
    const uint32_t nA = uni(L.rounds), nS = uni(L.chg), nC = uni(L.nleft);
    pc.lap(GP_TJ_COMPACT);
    if (tid == 0) {
        crit_on();  // (the one wave working: first at its SIMD)
        int16_t *tidx = L.a0, *tlow = L.a1, *tstk = L.a2, *cstk = L.a3;
        uint8_t *onst = L.b0, *cpos = L.b1;
        int counter = 0, sp = 0, nm = 0, nc = 0;
        for (uint32_t ri = 0; ri <= nA + nC; ++ri) {
            if (ri == nA && nS) {  // S, one component
                nm += (int)nS;
                L.comp_end[nc++] = (int16_t)nm;
            }
            if (ri == nA + nC) break;
            const uint32_t r0 = (uint32_t)roots[ri];
            if (tidx[r0] >= 0) continue;
            // the top frame lives in registers (its edge, next dependency
            // slot, low link, index and dependencies); the frames below it in
            // cstk / cpos / tlow.  The same walk, in the same order, as one
            // with every frame in LDS, with a third of the dependent LDS round
            // trips per step.
            int csp = 0, k = (int)r0, pos = 0, tk = counter++, lowk = tk;
            int d0 = L.dep[3 * k], d1 = L.dep[3 * k + 1], d2 = L.dep[3 * k + 2];
            tidx[k] = (int16_t)tk;
            tstk[sp++] = (int16_t)k;
            onst[k] = 1;
            for (;;) {
                if (pos < 3) {
                    const int w = pos == 0 ? d0 : pos == 1 ? d1 : d2;
                    ++pos;
                    if (w < 0) continue;
                    const int tw = tidx[w];
                    const bool on = onst[w] != 0;
                    if (tw < 0) {  // descend: the current frame goes to the stack
                        cstk[csp] = (int16_t)k;
                        cpos[csp] = (uint8_t)pos;
                        tlow[k] = (int16_t)lowk;
                        ++csp;
                        k = w;
                        pos = 0;
                        tk = lowk = counter++;
                        d0 = L.dep[3 * k];
                        d1 = L.dep[3 * k + 1];
                        d2 = L.dep[3 * k + 2];
                        tidx[k] = (int16_t)tk;
                        tstk[sp++] = (int16_t)k;
                        onst[k] = 1;
                    } else if (on && tw < lowk) {
                        lowk = tw;
                    }
                    continue;
                }
                if (lowk == tk) {  // k roots a component
                    for (;;) {
                        const int w = tstk[--sp];
                        onst[w] = 0;
                        L.members[nm++] = (int16_t)w;
                        if (w == k) break;
                    }
                    L.comp_end[nc++] = (int16_t)nm;
                }
                if (csp == 0) break;
                // back to the parent frame, its low link taking the child's
                const int lowc = lowk;
                --csp;
                k = cstk[csp];
                pos = cpos[csp];
                lowk = tlow[k];
                tk = tidx[k];
                d0 = L.dep[3 * k];
                d1 = L.dep[3 * k + 1];
                d2 = L.dep[3 * k + 2];
                if (lowc < lowk) lowk = lowc;
            }
        }
        L.ncomp = (uint32_t)nc;
        crit_off();
    }
    __syncthreads();
    pc.lap(GP_TARJAN);

    // ---- 3b. blocks in emission order: singletons on lane 0, blocks with the WG
    const uint32_t ncomp = uni(L.ncomp);
    uint32_t c = 0;
    while (c < ncomp) {
        if (tid == 0) {
            crit_on();  // (the one wave working: first at its SIMD)
            // run of singletons
            while (c < ncomp) {
                const int beg = c ? L.comp_end[c - 1] : 0;
                if (L.comp_end[c] - beg != 1) break;
                const int k = L.members[beg];
                int h = 0;
                while (L.e[3 * k + h] != (uint32_t)L.hinge[k]) ++h;
                uint32_t s = 0, coef = 0;
                for (int i = 0; i < 3; ++i) {
                    if (L.e[3 * k + i] == (uint32_t)L.hinge[k]) ++coef;
                    else s += L.xval[L.e[3 * k + i]];
                }
                const uint32_t rhs = ((uint32_t)h + 6 - s % 3) % 3;
                if (coef % 3 == 0) {
                    L.flag = 0;  // singular singleton (cannot happen: triple edges rejected)
                    c = ncomp;
                    break;
                }
                L.xval[L.hinge[k]] = (uint8_t)(coef == 1 ? rhs : (2 * rhs) % 3);
                ++c;
            }
            L.pivot = c;
            crit_off();
        }
        __syncthreads();
        pc.lap(GP_SINGLE);
        c = uni(L.pivot);
        if (c >= ncomp) break;
        // dense block c
        const uint32_t beg = c ? uni((uint32_t)L.comp_end[c - 1]) : 0;
        const uint32_t sz = uni((uint32_t)L.comp_end[c]) - beg;
        // the block's columns in increasing edge order (the order that
        // defines the solution of a singular block, see gauss_jordan): S
        // comes out of the ordered compaction sorted, Tarjan's blocks in stack
        // order are ranked (tiny, or rare: no big S)
        {
            bool unsorted = false;
            for (uint32_t i = tid; i + 1 < sz; i += GS_THREADS) unsorted |= L.members[beg + i] > L.members[beg + i + 1];
            if (__syncthreads_or(unsorted)) {
                int16_t *tmp = L.a3;  // (Tarjan's stack is dead; the FVS queue comes later)
                for (uint32_t i = tid; i < sz; i += GS_THREADS) {
                    const int16_t k = L.members[beg + i];
                    uint32_t rk = 0;
                    for (uint32_t j = 0; j < sz; ++j) rk += L.members[beg + j] < k;
                    tmp[rk] = k;
                }
                __syncthreads();
                for (uint32_t i = tid; i < sz; i += GS_THREADS) L.members[beg + i] = tmp[i];
                __syncthreads();
            }
        }
        for (uint32_t i = tid; i < sz; i += GS_THREADS) L.col_of[L.members[beg + i]] = (int16_t)i;
        __syncthreads();
        // Rows live word-major in the workgroup's scratch: plane q (the two
        // bit planes of GF(3)) of word w of row rr at scr[(2w + q) * Lds::CMAX
        // + rr], so a wave's 64 rows read 64 consecutive words (row-major
        // rows 2W words apart cost a 64-byte sector per lane).
        auto X = [&](uint32_t rr, uint32_t w, uint32_t q) -> uint64_t & { return scr[(size_t)(2 * w + q) * Lds::CMAX + rr]; };
        uint8_t *colval = L.b0;  // (Tarjan's arrays are dead here)

        // The shared tail of both Gauss-Jordan forms below: each column's
        // value from its pivot row, and the consistency of the rows without one.
        auto gj_tail = [&](uint32_t n, auto &&X) -> bool {
            int16_t *piv = L.a0;
            uint8_t *used = L.b1;
            // column cc's pivot row reads cf * x + (free columns, all 0) = rhs
            // with cf in {1, 2} (every other pivot column eliminated), so
            // x = cf * rhs mod 3; a row without a pivot is all zero and must
            // read rhs = 0
            const uint64_t rbit = 1ULL << (n & 63);
            for (uint32_t cc = tid; cc < n; cc += GS_THREADS) {
                const int pr = piv[cc];
                if (pr < 0) {
                    colval[cc] = 0;
                    continue;
                }
                const uint64_t cbit = 1ULL << (cc & 63);
                const uint32_t rhs = (X(pr, n >> 6, 0) & rbit) ? 1 : (X(pr, n >> 6, 1) & rbit) ? 2 : 0;
                const uint32_t cf = (X(pr, cc >> 6, 1) & cbit) ? 2 : 1;
                colval[cc] = (uint8_t)(cf * rhs % 3);
            }
            bool bad = false;
            for (uint32_t rr = tid; rr < n; rr += GS_THREADS)
                if (!used[rr] && ((X(rr, n >> 6, 0) | X(rr, n >> 6, 1)) & rbit)) bad = true;
            const bool ok = !__syncthreads_or(bad);
            if (!ok && tid == 0) L.flag = 0;
            __syncthreads();
            return ok;
        };
        // Gauss-Jordan on rows 0..n-1 of X (n equations, n unknowns, the
        // right-hand side in column n), without row swaps: column cc's pivot
        // is the first unused row with a nonzero there, piv[cc] remembers it
        // (-1: no such row, a free column).  The result is the reduced row
        // echelon form up to the order of its rows, whatever the pivot rows,
        // so the pivot columns, and the solution with every free column 0,
        // equal the oracle's row-swapping elimination.  Returns whether the
        // system is consistent (every row left without a pivot reads 0 = 0);
        // colval[cc] = x_cc, L.nfree = the free columns (GOV:425-432: only an
        // inconsistent system is "unsolvable" and moves to the next seed).
        // ONE barrier per column: every row reads the
        // pivot row where it lies (its owner last wrote it before the
        // previous barrier and leaves it alone in its own column); while a
        // row is eliminated it bids for the next column's pivot (the lowest
        // candidate lane of each wave, one LDS atomicMin).  The bid word is
        // triple-buffered by column (read in cc, bid into in cc, re-armed in
        // cc + 1: each use a barrier apart).
        auto gauss_jordan = [&](uint32_t n, auto &&X) -> bool {
            const uint32_t W = (n + 1 + 63) / 64;
            int16_t *piv = L.a0;
            uint8_t *used = L.b1;
            uint32_t *bid = L.hbin;  // bid[cc % 3]
            for (uint32_t rr = tid; rr < n; rr += GS_THREADS) used[rr] = 0;
            if (tid < 3) bid[tid] = 0xFFFFFFFFu;
            if (tid == 0) L.nfree = 0;
            __threadfence_block();
            __syncthreads();
            for (uint32_t rr = tid; rr < n; rr += GS_THREADS) {
                const bool cand = (X(rr, 0, 0) | X(rr, 0, 1)) & 1ULL;
                const uint64_t bal = __builtin_amdgcn_ballot_w64(cand);
                if (cand && (uint32_t)__builtin_ctzll(bal) == (tid & 63)) atomicMin(&bid[0], rr);
            }
            __syncthreads();
            for (uint32_t cc = 0; cc < n; ++cc) {
                const uint32_t p = uni(bid[cc % 3]);
                if (p == 0xFFFFFFFFu) {  // a free column (uniform): x_cc = 0
                    const uint32_t cn = cc + 1, wn = cn >> 6;
                    const uint64_t nbit = 1ULL << (cn & 63);
                    if (tid == 0) {
                        piv[cc] = -1;
                        ++L.nfree;
                        bid[(cc + 2) % 3] = 0xFFFFFFFFu;
                    }
                    for (uint32_t rr = tid; rr < n; rr += GS_THREADS) {
                        const bool cand = cn < n && !used[rr] && ((X(rr, wn, 0) | X(rr, wn, 1)) & nbit);
                        const uint64_t bal = __builtin_amdgcn_ballot_w64(cand);
                        if (cand && (uint32_t)__builtin_ctzll(bal) == (tid & 63)) atomicMin(&bid[cn % 3], rr);
                    }
                    __syncthreads();
                    continue;
                }
                const uint32_t wc = cc >> 6;
                const uint64_t bit = 1ULL << (cc & 63);
                const bool two = (X(p, wc, 1) & bit) != 0;  // pivot coefficient 2: its row normalised = planes swapped
                if (tid == 0) {
                    piv[cc] = (int16_t)p;
                    bid[(cc + 2) % 3] = 0xFFFFFFFFu;
                }
                const uint32_t cn = cc + 1, wn = cn >> 6;
                const uint64_t nbit = 1ULL << (cn & 63);
                for (uint32_t rr = tid; rr < n; rr += GS_THREADS) {
                    bool cand = false;
                    if (rr == p) {
                        used[rr] = 1;
                    } else {
                        const uint64_t f1 = X(rr, wc, 0) & bit, f2 = X(rr, wc, 1) & bit;
                        if (f1 || f2) {
                            const bool sw = (f1 != 0) != two;  // subtract cf * (normalised pivot row)
                            for (uint32_t w = wc; w < W; ++w) {
                                const uint64_t q1 = X(p, w, 0), q2 = X(p, w, 1);
                                gf3_add(X(rr, w, 0), X(rr, w, 1), sw ? q2 : q1, sw ? q1 : q2);
                            }
                        }
                        cand = cn < n && !used[rr] && ((X(rr, wn, 0) | X(rr, wn, 1)) & nbit);
                    }
                    // a wave's lanes hold consecutive rows: its lowest
                    // candidate lane alone bids (one LDS atomic per wave)
                    const uint64_t bal = __builtin_amdgcn_ballot_w64(cand);
                    if (cand && (uint32_t)__builtin_ctzll(bal) == (tid & 63)) atomicMin(&bid[cn % 3], rr);
                }
                // (profiling: columns, and thread 0's wait at the column's
                // barrier -- the time the workgroup's slowest row takes
                // beyond thread 0's own)
                const uint64_t tb = pc.on() ? clock64() : 0;
                __syncthreads();
                if (pc.on()) {
                    pc.add(GP_GJ_COLUMNS, 1);
                    pc.add(GP_GJ_BARRIER, clock64() - tb);
                }
            }
            return gj_tail(n, X);
        };
        // The heavy system's Gauss-Jordan with each row in its own thread's
        // registers (n <= GS_THREADS rows of H words a plane; the solver's
        // 256-thread form has the VGPRs for it, GOV_GJ_REG): per column,
        // every wave's lowest candidate row for the next pivot publishes its
        // index and words in the wave's slot (double-buffered by column
        // parity); after the column's one barrier every thread reads the
        // waves' bids, takes the lowest row -- the pivot the LDS form's
        // atomicMin picks -- reads its words from that wave's slot and
        // eliminates in registers: two LDS round trips a column instead of the
        // LDS form's chain of ~6.  Same pivots, same reduced
        // rows (written back at the end), same tail.
        auto gauss_jordan_reg = [&](uint32_t n, auto hw, auto &&X, uint64_t *slots) -> bool {
            constexpr uint32_t H = decltype(hw)::value;
            constexpr uint32_t NW = GS_THREADS / 64, SW = 2 * H + 1;  // a slot: the row index, then its words
            int16_t *piv = L.a0;
            uint8_t *used_m = L.b1;
            const uint32_t rr = tid, lane = tid & 63, wv = tid >> 6;
            const bool mine = rr < n;
            uint64_t r1[H], r2[H];
#pragma unroll
            for (uint32_t w = 0; w < H; ++w) {
                r1[w] = mine ? X(rr, w, 0) : 0;
                r2[w] = mine ? X(rr, w, 1) : 0;
            }
            bool used = false;
            uint32_t nfree = 0;
            auto publish = [&](uint32_t c, uint32_t par) {  // the wave's lowest candidate for column c
                bool cand = false;
                if (mine && !used && c < n) {
                    uint64_t t = 0;
#pragma unroll
                    for (uint32_t w = 0; w < H; ++w)
                        if (w == (c >> 6)) t = r1[w] | r2[w];
                    cand = ((t >> (c & 63)) & 1ULL) != 0;
                }
                const uint64_t bal = __builtin_amdgcn_ballot_w64(cand);
                uint64_t *sl = slots + (size_t)(par * NW + wv) * SW;
                if (!bal) {
                    if (lane == 0) sl[0] = ~0ULL;
                } else if (lane == (uint32_t)__builtin_ctzll(bal)) {
                    sl[0] = rr;
#pragma unroll
                    for (uint32_t w = 0; w < H; ++w) {
                        sl[1 + 2 * w] = r1[w];
                        sl[2 + 2 * w] = r2[w];
                    }
                }
            };
            __syncthreads();  // (every row read before the slots, which may share its words, are written)
            publish(0, 0);
            __syncthreads();
            for (uint32_t cc = 0; cc < n; ++cc) {
                const uint32_t par = cc & 1;
                uint64_t best = ~0ULL;
                uint32_t bw = 0;
#pragma unroll
                for (uint32_t w = 0; w < NW; ++w) {
                    const uint64_t b = slots[(size_t)(par * NW + w) * SW];
                    if (b < best) {
                        best = b;
                        bw = w;
                    }
                }
                if (best == ~0ULL) {  // a free column (uniform): x_cc = 0
                    if (tid == 0) piv[cc] = -1;
                    ++nfree;
                    publish(cc + 1, par ^ 1u);
                    __syncthreads();
                    continue;
                }
                const uint64_t *ps = slots + (size_t)(par * NW + bw) * SW;
                uint64_t q1[H], q2[H];
#pragma unroll
                for (uint32_t w = 0; w < H; ++w) {
                    q1[w] = ps[1 + 2 * w];
                    q2[w] = ps[2 + 2 * w];
                }
                const uint32_t wc = cc >> 6;
                const uint64_t bit = 1ULL << (cc & 63);
                uint64_t pq2 = 0, f1 = 0, f2 = 0;
#pragma unroll
                for (uint32_t w = 0; w < H; ++w)
                    if (w == wc) {
                        pq2 = q2[w];
                        f1 = r1[w] & bit;
                        f2 = r2[w] & bit;
                    }
                const bool two = (pq2 & bit) != 0;  // pivot coefficient 2: its row normalised = planes swapped
                if (tid == 0) piv[cc] = (int16_t)best;
                if (rr == (uint32_t)best) {
                    used = true;
                } else if (mine && (f1 | f2)) {
                    const bool sw = (f1 != 0) != two;  // subtract cf * (normalised pivot row)
#pragma unroll
                    for (uint32_t w = 0; w < H; ++w)
                        if (w >= wc) gf3_add(r1[w], r2[w], sw ? q2[w] : q1[w], sw ? q1[w] : q2[w]);
                }
                publish(cc + 1, par ^ 1u);
                __syncthreads();
            }
            if (mine) {
#pragma unroll
                for (uint32_t w = 0; w < H; ++w) {
                    X(rr, w, 0) = r1[w];
                    X(rr, w, 1) = r2[w];
                }
                used_m[rr] = used ? 1 : 0;
            }
            if (tid == 0) L.nfree = nfree;
            __syncthreads();
            return gj_tail(n, X);
        };
        // The heavy system's Gauss-Jordan by 64-column panels (GOV_GJ_PANEL).
        // Per panel (one word of every row), a row per thread holds in
        // registers its panel word and its multiplier word M over the
        // panel's pivots (row now = row at the panel's start + sum_j M[j]
        // pivot row j at the panel's start); eliminating column c with pivot
        // p adds s (p's panel word) to a row's panel word and s (e_c + M[p])
        // to its M.  The columns are taken in order with gauss_jordan's pivots
        // (the lowest unused row with a nonzero), found without a barrier per
        // column: the LEADER, the lowest wave with an unused row, holds the
        // lowest unused rows, so while it has a candidate the pivot is its
        // own -- it runs through the panel's columns alone (ballot, readlane)
        // and records each pivot's words; then the other waves take the
        // recorded eliminations in order, and a column the leader has no
        // candidate for is settled by every wave's lowest candidate (slots).
        // After the panel every row's trailing words take sum_j M[j] Q_j
        // (Q_j: pivot row j's trailing words at the panel's start).  Same
        // pivots, the same linear combinations of the rows: the same reduced
        // rows, the same tail.  pw: LDS scratch of gj_panel_words(n) words.
        auto gauss_jordan_panel = [&](uint32_t n, auto &&X, uint64_t *pw) -> bool {
            constexpr uint32_t NW = GS_THREADS / 64, SW = 5;  // a slot: the row index, its panel word, its M
            const uint32_t W = (n + 1 + 63) / 64;            // words a plane, the right-hand side (column n) included
            int16_t *piv = L.a0;
            uint8_t *used_m = L.b1;
            uint32_t *flags = L.hbin;                         // [w]: wave w has an unused row; [16]: the leader's block end
            uint64_t *slots = pw, *pinfo = pw + NW * SW;      // pinfo[4 cl ..]: pivot panel word, e_c + M[p]
            uint64_t *Q = pinfo + 4 * 64;                     // the pair table of the trailing update
            const uint32_t rr = tid, lane = tid & 63, wv = tid >> 6;
            const bool mine = rr < n;
            bool used = false;
            uint32_t nfree = 0;
            // blocks of this call are numbered 1, 2, ...: a progress word left
            // by an earlier call or block never reads as the current block's
            // (the reset is ordered before any use by the first block's barrier)
            uint32_t seq = 0;
            if (tid == 0) flags[16] = 0xFFFFFFFFu;
            for (uint32_t wc = 0; 64 * wc < n; ++wc) {
                const uint32_t TW = W - wc - 1, cn = min(64u, n - 64 * wc);
                uint64_t r1 = mine ? X(rr, wc, 0) : 0, r2 = mine ? X(rr, wc, 1) : 0, m1 = 0, m2 = 0;
                // (the multipliers' high half untouched below column 32 and the
                // rows' low half from column 32 on without a free column,
                // skipped by uniform branches: leader +12 % cycles, not kept)
                auto apply = [&](uint64_t bit, uint64_t q1, uint64_t q2, uint64_t d1, uint64_t d2, uint32_t p) {
                    if (rr == p) {
                        used = true;
                    } else if (mine) {
                        const uint64_t f1 = r1 & bit, f2 = r2 & bit;
                        if (f1 | f2) {
                            const bool sw = (f1 != 0) != ((q2 & bit) != 0);  // subtract cf * (normalised pivot row)
                            gf3_add(r1, r2, sw ? q2 : q1, sw ? q1 : q2);
                            gf3_add(m1, m2, sw ? d2 : d1, sw ? d1 : d2);
                        }
                    }
                };
                uint32_t cl = 0;
                while (cl < cn) {  // (uniform)
                    const uint64_t un = __builtin_amdgcn_ballot_w64(mine && !used);
                    if (lane == 0) flags[wv] = un != 0;
                    __syncthreads();
                    uint32_t lead = NW;
                    for (uint32_t w = 0; w < NW; ++w)
                        if (flags[w]) {
                            lead = w;
                            break;
                        }
                    // (values read from LDS are per-lane to the compiler; these
                    // are the same in every lane, and the loops below are then
                    // scalar loops: no exec-mask bookkeeping per column)
                    lead = (uint32_t)__builtin_amdgcn_readfirstlane((int)lead);
                    // The leader's progress word: (block sequence << 16) |
                    // columns recorded | 0x8000 once the block has ended.  The
                    // other waves take each recorded column as soon as it is
                    // published, beside the leader (no barrier between).
                    ++seq;  // (< 0xFFFF: a block takes at least one column)
                    uint32_t ce = cl;
                    const uint64_t tl0 = pc.now();
                    if (wv == lead) {
                        crit_on();  // (the one wave working: first at its SIMD)
                        for (; ce < cn; ++ce) {
                            const uint64_t bit = 1ULL << ce;
                            const uint64_t bal = __builtin_amdgcn_ballot_w64(mine && !used && ((r1 | r2) & bit));
                            if (!bal) break;
                            const uint32_t pl = (uint32_t)__builtin_ctzll(bal), p = 64 * wv + pl;
                            const uint64_t q1 = readlane64(r1, (int)pl), q2 = readlane64(r2, (int)pl);
                            const uint64_t d1 = readlane64(m1, (int)pl) | bit, d2 = readlane64(m2, (int)pl);  // M[p][c] = 0
                            if (lane == 0) {
                                pinfo[4 * ce] = q1;
                                pinfo[4 * ce + 1] = q2;
                                pinfo[4 * ce + 2] = d1;
                                pinfo[4 * ce + 3] = d2;
                                piv[64 * wc + ce] = (int16_t)p;
                                // (publishing every 2 or 4 columns: no change, not kept)
                                // LDS operations of a wave are performed in
                                // the order it issues them, so the progress
                                // word lands after the pivot's words without
                                // a release wait for them; the signal fence
                                // keeps the compiler from reordering the stores
                                __atomic_signal_fence(__ATOMIC_SEQ_CST);
                                __hip_atomic_store(&flags[16], seq << 16 | (ce + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            }
                            apply(bit, q1, q2, d1, d2, p);
                        }
                        __atomic_signal_fence(__ATOMIC_SEQ_CST);
                        if (lane == 0) __hip_atomic_store(&flags[16], seq << 16 | 0x8000u | ce, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        crit_off();
                        pc.add_any(GP_GJ_LEAD, pc.now() - tl0);
                        pc.add_any(GP_GJ_LEADCOLS, ce - cl);
                    } else if (lead < NW) {
                        uint32_t c2 = cl;
                        for (;;) {
                            const uint32_t v = (uint32_t)__builtin_amdgcn_readfirstlane(
                                (int)__hip_atomic_load(&flags[16], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
                            const bool mine_seq = (v >> 16) == seq;
                            const uint32_t lim = mine_seq ? (v & 0x7FFFu) : cl;
                            constexpr uint32_t FU = GOV_GJ_FOLLOW;
                            for (; c2 + FU <= lim; c2 += FU) {  // (the recorded pivots FU at a time: loads issued together)
                                // (a pivot row is the leader's, never this wave's)
                                uint64_t pv4[4 * FU];
#pragma unroll
                                for (uint32_t k = 0; k < 4 * FU; ++k) pv4[k] = pinfo[4 * c2 + k];
#pragma unroll
                                for (uint32_t k = 0; k < FU; ++k)
                                    apply(1ULL << (c2 + k), pv4[4 * k], pv4[4 * k + 1], pv4[4 * k + 2], pv4[4 * k + 3],
                                          0xFFFFFFFFu);
                            }
                            if (mine_seq && (v & 0x8000u)) {
                                for (; c2 < lim; ++c2) {
                                    const uint64_t *pi = pinfo + 4 * c2;
                                    apply(1ULL << c2, pi[0], pi[1], pi[2], pi[3], 0xFFFFFFFFu);
                                }
                                ce = lim;
                                pc.add_any(GP_GJ_FOLLOW, pc.now() - tl0);
                                break;
                            }
                            if (GOV_GJ_SLEEP && c2 + FU > lim) __builtin_amdgcn_s_sleep(GOV_GJ_SLEEP);
                        }
                    }
                    // (every wave has ce; uniform)
                    cl = (uint32_t)__builtin_amdgcn_readfirstlane((int)ce);
                    if (cl < cn) {
                        // column cl: no candidate in the leader -- every
                        // wave's lowest candidate (or a free column)
                        const uint64_t bit = 1ULL << cl;
                        const uint64_t bal = __builtin_amdgcn_ballot_w64(mine && !used && ((r1 | r2) & bit));
                        uint64_t *sl = slots + (size_t)wv * SW;
                        if (!bal) {
                            if (lane == 0) sl[0] = ~0ULL;
                        } else if (lane == (uint32_t)__builtin_ctzll(bal)) {
                            sl[0] = rr;
                            sl[1] = r1;
                            sl[2] = r2;
                            sl[3] = m1;
                            sl[4] = m2;
                        }
                        __syncthreads();
                        uint64_t best = ~0ULL;
                        uint32_t bw = 0;
                        for (uint32_t w = 0; w < NW; ++w) {
                            const uint64_t b = slots[(size_t)w * SW];
                            if (b < best) {
                                best = b;
                                bw = w;
                            }
                        }
                        best = readfirstlane64(best);
                        bw = (uint32_t)__builtin_amdgcn_readfirstlane((int)bw);
                        const uint32_t c = 64 * wc + cl;
                        pc.add(GP_GJ_SLOTCOLS, 1);
                        if (best == ~0ULL) {  // a free column (uniform): x_c = 0
                            if (tid == 0) piv[c] = -1;
                            ++nfree;
                        } else {
                            const uint64_t *ps = slots + (size_t)bw * SW;
                            if (tid == 0) piv[c] = (int16_t)best;
                            apply(bit, ps[1], ps[2], ps[3] | bit, ps[4], (uint32_t)best);
                        }
                        ++cl;
                    }
                }
                if (mine) {
                    X(rr, wc, 0) = r1;
                    X(rr, wc, 1) = r2;
                }
                const uint64_t tt0 = pc.now();
                pc.add(GP_GJ_PANELS, 1);
                if (TW) {
                    // row += sum_j M[j] Q_j, Q_j = pivot row j's trailing words
                    // at the panel's start, one trailing word at a time by the
                    // method of four Russians over F3: the panel's columns in
                    // pairs, T[c][d0 + 3 d1] = d0 Q_2c + d1 Q_2c+1 (9 entries a
                    // pair, built by the workgroup from the pivot rows, which no
                    // row has updated in this word yet), then each row adds one
                    // entry a pair (its two M digits) instead of a conditional
                    // add a column: a third of the VALU work
                    for (uint32_t t = 0; t < TW; ++t) {
                        __syncthreads();  // (the previous word's rows are done with T)
                        for (uint32_t ix = tid; ix < 32 * 9; ix += GS_THREADS) {
                            const uint32_t c = ix / 9, d = ix - 9 * c, d0 = d % 3, d1 = d / 3;
                            uint64_t e1 = 0, e2 = 0;
                            for (uint32_t h = 0; h < 2; ++h) {
                                const uint32_t j = 2 * c + h, dj = h ? d1 : d0;
                                const int pr = (j < cn && dj) ? piv[64 * wc + j] : -1;
                                if (pr >= 0) {
                                    const uint64_t q1 = X((uint32_t)pr, wc + 1 + t, 0), q2 = X((uint32_t)pr, wc + 1 + t, 1);
                                    gf3_add(e1, e2, dj == 1 ? q1 : q2, dj == 1 ? q2 : q1);
                                }
                            }
                            Q[2 * ix] = e1;
                            Q[2 * ix + 1] = e2;
                        }
                        __syncthreads();
                        if (mine && (m1 | m2)) {
                            // four pairs a step, their entries loaded together and
                            // added unconditionally (entry 0 of a pair is zero)
                            const uint32_t npair = (65 - (uint32_t)__builtin_clzll(m1 | m2)) >> 1;
                            uint64_t t1 = X(rr, wc + 1 + t, 0), t2 = X(rr, wc + 1 + t, 1);
                            for (uint32_t c0 = 0; c0 < npair; c0 += 4) {
                                uint64_t e1[4], e2[4];
#pragma unroll
                                for (uint32_t u = 0; u < 4; ++u) {
                                    const uint32_t c = c0 + u;  // (c < 32: pairs past npair read their zero entry)
                                    const uint32_t b1 = (uint32_t)(m1 >> (2 * c)) & 3u, b2 = (uint32_t)(m2 >> (2 * c)) & 3u;
                                    // digits: d = bit of m1 + 2 bit of m2, per column of the pair
                                    const uint32_t idx = (b1 & 1u) + 2 * (b2 & 1u) + 3 * ((b1 >> 1) + 2 * (b2 >> 1));
                                    const uint64_t *te = Q + 2 * (9 * c + idx);
                                    e1[u] = te[0];
                                    e2[u] = te[1];
                                }
#pragma unroll
                                for (uint32_t u = 0; u < 4; ++u) gf3_add(t1, t2, e1[u], e2[u]);
                            }
                            X(rr, wc + 1 + t, 0) = t1;
                            X(rr, wc + 1 + t, 1) = t2;
                        }
                    }
                }
                __syncthreads();
                pc.add(GP_GJ_TRAIL, pc.now() - tt0);
            }
            if (mine) used_m[rr] = used ? 1 : 0;
            if (tid == 0) L.nfree = nfree;
            __syncthreads();
            return gj_tail(n, X);
        };
        // Block equation of member i: cf*x_hinge + sum of its other vertices
        // = h (mod 3), h = the hinge's position in the edge, cf = its count.
        // Large blocks: heavy variables chosen so that the others follow in
        // dependency order (a feedback vertex set of the block's dependency
        // graph); every other hinge becomes an affine form of the heavy ones
        // (vectors over nH heavy columns + a constant column), the heavy
        // hinges' own equations are an nH x nH system (~20 % of the block),
        // and the forms are evaluated.  Block elimination by a triangular
        // part with unit-or-two diagonal: the block's solutions are exactly
        // x = T y + t over the heavy system's solutions y (solvable exactly
        // when the block is, with the same null space dimension); a singular
        // one is then moved to the block's own canonical solution (free
        // columns 0) through that null space, below.
#ifndef GOV_FVS_MIN
#define GOV_FVS_MIN 96
#endif
        constexpr uint32_t FVS_MIN = GOV_FVS_MIN, FW = 6;  // <= 6 words per form / heavy row
        static_assert(FVS_NH_MAX + 1 <= 64 * FW, "heavy columns + the constant column must fit FW words");
        constexpr size_t V0 = (size_t)16 * Lds::CMAX;          // affine forms, past that region
        bool solved = false;
        if (sz >= FVS_MIN) {
            uint32_t *st = L.xe, *indeg = L.claim;  // 0 open, 1 formed, 2 heavy, after the selection (dead arrays)
            int16_t *rnd = L.a1, *hid = L.a2;
            auto in_dep = [&](uint32_t k, int i) -> int {  // member index of the owner of vertex i, or -1
                const uint32_t v = L.e[3 * k + i];
                if (v == (uint32_t)L.hinge[k]) return -1;
                const int o = L.vowner[v];
                return (o >= 0 && L.col_of[o] >= 0) ? L.col_of[o] : -1;
            };
            // lvl (st's words until the selection ends): 1 + the highest
            // level of the member's dependencies placed so far (heavy: 0)
            uint32_t *lvl = st;
            // the block's dependency graph, once: idep[3i+t] = member index
            // of the owner of member i's vertex t, or -1 (L.dep is dead here)
            int16_t *idep = L.dep;
            for (uint32_t i = tid; i < sz; i += GS_THREADS) {
                lvl[i] = 1;
                const uint32_t k = (uint32_t)L.members[beg + i];
                for (int t = 0; t < 3; ++t) idep[3 * i + t] = (int16_t)in_dep(k, t);
            }
            __syncthreads();
            // Selection, Kahn style: a member is placed (formed) once every
            // in-block dependency is placed; with none ready, the open member
            // most open members depend on turns heavy (ties: lowest index).
            // The ready closure is the same whatever order it is reached in,
            // so the heavy set is that of level-synchronous rounds.  A formed
            // member's level is 1 + its dependencies' highest (heavy: 0):
            // the forms are evaluated level by level.
            // pend[i]: i's dependency slots not yet placed, + 0x100 once i is
            // heavy (so it never reads 1 -> 0); open = 1..0xFF, formed = 0.
            // A placed member raises its dependents' lvl before it releases
            // their pending slots (one wave, LDS operations in order), so a
            // member's lvl is final when its last slot is released: the
            // closure costs one returned LDS atomic per dependency.
            uint32_t *roff = L.deg;                                        // reverse CSR offsets
            uint32_t *pend = L.pend();
            int16_t *queue = L.a3;
            for (uint32_t i = tid; i <= sz; i += GS_THREADS) roff[i] = 0;
            if (tid == 0) {
                L.qtail = 0;
                L.rounds = 0;
            }
            __syncthreads();
            for (uint32_t i = tid; i < sz; i += GS_THREADS) {
                uint32_t np = 0;
                for (int t = 0; t < 3; ++t) {
                    const int d = idep[3 * i + t];
                    if (d >= 0) {
                        atomicAdd(&roff[d], 1u);
                        ++np;
                    }
                }
                pend[i] = np;
            }
            __syncthreads();
            wg_excl_scan3(roff, sz + 1, L.xe + Lds::CMAX);
            // the dependents (int16, roff[sz] of them) in LDS when they fit the
            // free tails of idep's and indeg's arrays (every block of a random
            // set but the largest): the closure's chain per dependency is then
            // an LDS read and a returned LDS atomic, not a global load first;
            // otherwise in the workgroup's scratch past the forms (words
            // [28 CMAX, 29.5 CMAX))
            const uint32_t rev_cap1 = 3 * (Lds::CMAX - sz), nrev = uni(roff[sz]);
            const bool rev_lds = nrev <= rev_cap1 + 2 * (Lds::CMAX - sz);  // (uniform)
            int16_t *const revA = rev_lds ? L.dep + 3 * sz : reinterpret_cast<int16_t *>(scr + (size_t)28 * Lds::CMAX);
            int16_t *const revB = reinterpret_cast<int16_t *>(L.claim + sz);
            auto rev = [&](uint32_t x) -> int16_t & { return (!rev_lds || x < rev_cap1) ? revA[x] : revB[x - rev_cap1]; };
            for (uint32_t d = tid; d < sz; d += GS_THREADS) indeg[d] = roff[d];
            __syncthreads();
            for (uint32_t i = tid; i < sz; i += GS_THREADS)
                for (int t = 0; t < 3; ++t) {
                    const int d = idep[3 * i + t];
                    if (d >= 0) rev(atomicAdd(&indeg[d], 1u)) = (int16_t)i;
                }
            __syncthreads();
            for (uint32_t d = tid; d < sz; d += GS_THREADS) {
                indeg[d] = roff[d + 1] - roff[d];  // slots of open members on d (all open)
                if (pend[d] == 0) queue[atomicAdd(&L.qtail, 1u)] = (int16_t)d;
            }
            __syncthreads();
            pc.lap(GP_SEL_PREP_CYCLES);
            const uint32_t lane = tid & 63, wv = tid >> 6;
            uint32_t qh = 0, nh = 0, nbatch = 0, npick = 0;  // (qh: wave 0's)
            uint64_t pick_cyc = 0;
            bool fb = false;
            for (;;) {
                // the ready closure (wave 0)
                if (tid < 64) {
                    crit_on();  // (the one wave working: first at its SIMD)
                    uint32_t qt = uni(L.qtail);
                    while (qh < qt) {
                        ++nbatch;
                        const uint32_t nb = min(64u, qt - qh);
                        uint32_t x0 = 0, x1 = 0, myl = 0;
#if GOV_CLOSURE_BRANCHFREE
                        // (every lane reads -- a lane past the batch reads its
                        // last member -- and the lanes with nothing to do aim
                        // their atomics and stores at a dead word of their own)
                        uint32_t *const dead = L.hbin;  // (the pick's bins: cleared by each pick before use)
                        int16_t *const dead16 = reinterpret_cast<int16_t *>(dead);
                        {
                            const bool inb = lane < nb;
                            const uint32_t p = (uint32_t)queue[qh + min(lane, nb - 1)];
                            const int d0 = idep[3 * p], d1 = idep[3 * p + 1], d2 = idep[3 * p + 2];
                            x0 = roff[p];
                            x1 = inb ? roff[p + 1] : x0;
                            const uint32_t pp = pend[p], lp = lvl[p];
                            atomicSub(inb && d0 >= 0 ? &indeg[d0] : &dead[lane], 1u);
                            atomicSub(inb && d1 >= 0 ? &indeg[d1] : &dead[lane], 1u);
                            atomicSub(inb && d2 >= 0 ? &indeg[d2] : &dead[lane], 1u);
                            // (a heavy member's lvl may have been raised
                            // while it waited in the queue: its level is 0)
                            myl = pp >= 0x100u ? 1u : lp + 1;
                        }
#else
                        if (lane < nb) {
                            const uint32_t p = (uint32_t)queue[qh + lane];
                            for (int t = 0; t < 3; ++t) {
                                const int d = idep[3 * p + t];
                                if (d >= 0) atomicSub(&indeg[d], 1u);
                            }
                            x0 = roff[p];
                            x1 = roff[p + 1];
                            // (a heavy member's lvl may have been raised
                            // while it waited in the queue: its level is 0)
                            myl = pend[p] >= 0x100u ? 1u : lvl[p] + 1;
                        }
#endif
                        // the batch's dependents, one per lane per step; the
                        // members they make ready are appended in lane order
                        // by ballot (the ready closure, the levels and so the
                        // heavy set do not depend on the queue order).  (Up
                        // to 4 per lane per step, issued together: slower,
                        // 7.3e6 -> 8.4e6 selection cycles.)
                        // (the next dependent read beside a step's atomics:
                        // no change, C2 gov 114.5 vs 114.5 ms, not kept)
                        // (flattened: the batch's dependents spread over the
                        // lanes by a ballot prefix sum, 64 a step: selection
                        // 3.52e6 -> 3.61e6 cycles, not kept -- a batch's
                        // members have few dependents each)
#if GOV_CLOSURE_BRANCHFREE
                        for (uint32_t x = x0;; ++x) {
                            const bool act = x < x1;
                            if (__builtin_amdgcn_ballot_w64(act) == 0) break;
                            const uint32_t i = (uint32_t)rev(act ? x : 0u);
                            atomicMax(act ? &lvl[i] : &dead[lane], myl);
                            const bool ready = atomicSub(act ? &pend[i] : &dead[lane], 1u) == 1u && act;  // its last slot
                            const uint64_t rm = __builtin_amdgcn_ballot_w64(ready);
                            const uint32_t pos = qt + __builtin_amdgcn_mbcnt_hi((uint32_t)(rm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)rm, 0u));
                            *(ready ? &queue[pos] : &dead16[64 + lane]) = (int16_t)i;
                            qt += (uint32_t)__builtin_popcountll(rm);
                        }
#else
                        for (uint32_t x = x0;; ++x) {
                            const bool act = x < x1;
                            if (__builtin_amdgcn_ballot_w64(act) == 0) break;
                            bool ready = false;
                            uint32_t i = 0;
                            if (act) {
                                i = (uint32_t)rev(x);
                                atomicMax(&lvl[i], myl);
                                ready = atomicSub(&pend[i], 1u) == 1u;  // its last slot
                            }
                            const uint64_t rm = __builtin_amdgcn_ballot_w64(ready);
                            if (ready)
                                queue[qt + __builtin_amdgcn_mbcnt_hi((uint32_t)(rm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)rm, 0u))] = (int16_t)i;
                            qt += (uint32_t)__builtin_popcountll(rm);
                        }
#endif
                        qh += nb;
                        __builtin_amdgcn_wave_barrier();
                    }
                    if (lane == 0) L.qtail = qt;
                    crit_off();
                }
                __syncthreads();
                const uint32_t qt = uni(L.qtail);
                if (qt >= sz) break;  // every member placed (each enters the queue once)
                // a pick adds up to 2 heavy hinges: the heavy set stays
                // <= fvs_max, so forms and heavy rows (constant column at nH)
                // fit FW words
                if (nh + 2 > fvs_max) {
                    fb = true;
                    break;
                }
                // The next heavy hinges: the `want` open members of the
                // largest key (pick_key below, then lowest index) -- the set
                // GOV_PICK_REPS rounds of "the best two" (below) pick, as
                // nothing is placed between those rounds: any feedback vertex
                // set gives the same unique solution and is singular exactly
                // when the block is.  The workgroup bins the open members by
                // key (64 bins), then takes every member above the
                // threshold bin and the lowest-index ones of that bin.
                const uint64_t tpk = pc.on() ? clock64() : 0;
                ++npick;
                const uint32_t want = 2 * min((uint32_t)GOV_PICK_REPS, (fvs_max - nh) / 2);
                auto is_open = [&](uint32_t pv) { return pv != 0u && pv < 0x100u; };
                // the pick key of an open member: its open dependents x its
                // open dependency slots (the usual greedy feedback-vertex-set
                // score: a member many others wait on and that waits on many
                // breaks the most cycles).  Against open dependents alone:
                // heavy set 223 -> 204 per block, C2 524 -> 537 M keys/s
                // (`profiles/r4/pick_key_ab/`; GOV_PICK_KEY=0 builds that)
                auto pick_key = [&](uint32_t i) -> uint32_t {
#if defined(GOV_PICK_KEY) && GOV_PICK_KEY == 0
                    return indeg[i];
#else
                    return indeg[i] * (pend[i] & 0xFFu);
#endif
                };
                auto make_heavy = [&](uint32_t i, uint32_t j, uint32_t slot) {
                    pend[i] += 0x100u;
                    lvl[i] = 0;
                    hid[i] = (int16_t)j;
                    queue[slot] = (int16_t)i;
                };
                uint32_t *hb = L.hbin;
                if (tid < 64) hb[tid] = 0;
                __syncthreads();
                for (uint32_t i = tid; i < sz; i += GS_THREADS)
                    if (is_open(pend[i])) atomicAdd(&hb[min(pick_key(i), 63u)], 1u);
                __syncthreads();
                uint32_t suf = hb[lane];  // -> open members of in-degree >= lane (every wave alike)
#pragma unroll
                for (int dd = 1; dd < 64; dd <<= 1) {
                    const uint32_t y = (uint32_t)__shfl_down((int)suf, dd, 64);
                    if (lane + dd < 64) suf += y;
                }
                const uint64_t okm = __builtin_amdgcn_ballot_w64(suf >= want);
                const uint32_t T = okm ? 63u - (uint32_t)__builtin_clzll(okm) : 0u;
                const uint32_t above = T < 63 ? (uint32_t)__builtin_amdgcn_readlane((int)suf, (int)T + 1) : 0u;
                const uint32_t in_t = (uint32_t)__builtin_amdgcn_readlane((int)suf, (int)T) - above;
                const uint32_t take_t = okm ? want - above : in_t;  // (fewer open members than want: all)
                if (T < 63 && !pick_exact) {
                    // in index order: per chunk of GS_THREADS members, each
                    // wave's counts of threshold-bin and above-threshold open
                    // members (double-buffered by chunk), one barrier a chunk
                    uint32_t *wc = L.deg + Lds::CMAX + 1;  // (past roff)
                    uint32_t run_eq = 0, got = 0, par = 0;
                    for (uint32_t k0 = 0; k0 < sz; k0 += GS_THREADS, par ^= 1u) {
                        const uint32_t i = k0 + tid;
                        const bool open = i < sz && is_open(pend[i]);
                        const uint32_t dvc = open ? min(pick_key(i), 63u) : 0u;
                        const bool eq = open && dvc == T, gt = open && dvc > T;
                        const uint64_t em = __builtin_amdgcn_ballot_w64(eq), gm = __builtin_amdgcn_ballot_w64(gt);
                        if (lane == 0) {
                            wc[32 * par + wv] = (uint32_t)__builtin_popcountll(em);
                            wc[32 * par + 16 + wv] = (uint32_t)__builtin_popcountll(gm);
                        }
                        __syncthreads();
                        uint32_t eb = run_eq, sb = got, my_eb = 0, my_sb = 0;
                        for (uint32_t w2 = 0; w2 < GS_THREADS / 64; ++w2) {
                            if (w2 == wv) {
                                my_eb = eb;
                                my_sb = sb;
                            }
                            const uint32_t e_w = wc[32 * par + w2], g_w = wc[32 * par + 16 + w2];
                            sb += g_w + min(e_w, take_t > eb ? take_t - eb : 0u);
                            eb += e_w;
                        }
                        const uint32_t rk = my_eb + __builtin_amdgcn_mbcnt_hi((uint32_t)(em >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)em, 0u));
                        const bool sel = gt || (eq && rk < take_t);
                        const uint64_t sm = __builtin_amdgcn_ballot_w64(sel);
                        if (sel) {
                            const uint32_t pos = my_sb + __builtin_amdgcn_mbcnt_hi((uint32_t)(sm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sm, 0u));
                            make_heavy(i, nh + pos, qt + pos);
                        }
                        run_eq = uni(eb);
                        got = uni(sb);
                    }
                    nh += got;
                    if (tid == 0) L.qtail = qt + got;
                } else if (tid < 64) {
                    // (64+ open members of in-degree >= 63 reach the
                    // threshold: the exact rounds on wave 0, loads issued 8
                    // at a time)
                    uint32_t nh0 = nh, q = qt;
                    for (int rep = 0; rep < GOV_PICK_REPS && nh0 + 2 <= fvs_max; ++rep) {
                        uint32_t key = 0, key2 = 0;
                        for (uint32_t q0 = 0; q0 * 64 < sz; q0 += 8) {
                            uint32_t sv[8], dv[8];
#pragma unroll
                            for (uint32_t u = 0; u < 8; ++u) {
                                const uint32_t i = lane + 64 * (q0 + u);
                                sv[u] = i < sz ? pend[i] : 0u;
                                dv[u] = i < sz ? min(pick_key(i), 0xFFFFu) : 0u;
                            }
#pragma unroll
                            for (uint32_t u = 0; u < 8; ++u)
                                if (is_open(sv[u])) {
                                    const uint32_t k = (dv[u] << 16) | (0xFFFFu - (lane + 64 * (q0 + u)));
                                    key2 = max(key2, min(key, k));
                                    key = max(key, k);
                                }
                        }
#pragma unroll
                        for (int dd = 32; dd >= 1; dd >>= 1) {
                            const uint32_t o1 = (uint32_t)__shfl_xor((int)key, dd, 64), o2 = (uint32_t)__shfl_xor((int)key2, dd, 64);
                            key2 = max(min(key, o1), max(key2, o2));
                            key = max(key, o1);
                        }
                        if (key == 0) break;  // (no open member left; wave-uniform)
                        if (lane == 0) {
                            make_heavy(0xFFFFu - (key & 0xFFFFu), nh0, q);
                            if (key2) make_heavy(0xFFFFu - (key2 & 0xFFFFu), nh0 + 1, q + 1);
                        }
                        nh0 += key2 ? 2 : 1;
                        q += key2 ? 2 : 1;
                        __builtin_amdgcn_wave_barrier();
                    }
                    if (lane == 0) {
                        L.qtail = q;
                        L.nleft = nh0;
                    }
                }
                __syncthreads();
                if (T >= 63 || pick_exact) nh = uni(L.nleft);  // (the exact rounds ran)
                if (pc.on()) pick_cyc += clock64() - tpk;
            }
            // st and the levels; the highest level
            uint32_t ml = 1;
            for (uint32_t i = tid; i < sz; i += GS_THREADS) {
                const uint32_t pv = pend[i], lv = lvl[i];
                const uint32_t s = pv == 0u ? 1u : pv >= 0x100u ? 2u : 0u;
                st[i] = s;  // (lvl's word)
                rnd[i] = (int16_t)(s == 1u ? lv : s == 2u ? 0u : 0xFFFFu);
                if (s == 1u) ml = max(ml, lv);
            }
#pragma unroll
            for (int dd = 32; dd >= 1; dd >>= 1) ml = max(ml, (uint32_t)__shfl_xor((int)ml, dd, 64));
            if (lane == 0) atomicMax(&L.rounds, ml + 1);
            if (tid == 0) {
                L.nleft = nh;
                L.chg = fb ? 1u : 0u;
                pc.add(GP_N_SEL_BATCHES, nbatch);
                pc.add(GP_N_SEL_PICKS, npick);
                pc.add(GP_SEL_PICK_CYCLES, pick_cyc);
            }
            __syncthreads();
            const uint32_t nH = uni(L.nleft), r = uni(L.rounds);
            const bool fall_back = uni(L.chg) != 0;
            pc.lap(GP_FVS_SEL);
            pc.add(GP_N_FVS_BLOCKS, 1);
            pc.add(GP_N_FORM_LEVELS, r);
            pc.add(GP_N_HEAVY, nH);
            if (!fall_back) {
                const uint32_t HW = (nH + 1 + 63) / 64;  // words per form (column nH = constant)
                // forms member-major: member i's 2 * HW words (planes of a
                // word adjacent) in one piece, so a dependency's form is one
                // or two cache lines (word-major they spanned 2 * HW lines
                // per read; forms 7.97e6 -> 7.40e6 cycles)
                auto V = [&](uint32_t i, uint32_t w, uint32_t q) -> uint64_t & { return scr[V0 + ((size_t)i * HW + w) * 2 + q]; };
                for (uint32_t i = tid; i < sz; i += GS_THREADS)
                    if (st[i] == 2)
                        for (uint32_t w = 0; w < HW; ++w) {
                            V(i, w, 0) = (w == (uint32_t)hid[i] >> 6) ? 1ULL << (hid[i] & 63) : 0;
                            V(i, w, 1) = 0;
                        }
                __syncthreads();
                auto hinge_pos = [&](uint32_t k, uint32_t &h, uint32_t &cf) {
                    h = 0;
                    while (L.e[3 * k + h] != (uint32_t)L.hinge[k]) ++h;
                    cf = 0;
                    for (int t = 0; t < 3; ++t) cf += L.e[3 * k + t] == (uint32_t)L.hinge[k];
                };
                const uint32_t cw = nH >> 6;
                const uint64_t cbit = 1ULL << (nH & 63);
                // formed members listed by round (counting sort), each with its
                // in-block dependencies (idep) and constant (h - known values,
                // cf) precomputed: a round reads only its own members, rounds
                // that only picked a heavy hinge cost nothing
                uint32_t *roff = L.deg, *rcur = indeg;  // (peel degrees / BFS stamps dead; indeg done)
                int16_t *rlist = L.a3, *rinfo = L.a0;   // (Tarjan's arrays dead; a0 is reused by the GJ later)
                for (uint32_t R = tid; R <= r; R += GS_THREADS) roff[R] = 0;
                __syncthreads();
                for (uint32_t i = tid; i < sz; i += GS_THREADS) {
                    if (st[i] != 1) continue;
                    atomicAdd(&roff[rnd[i]], 1u);
                    const uint32_t k = (uint32_t)L.members[beg + i];
                    uint32_t h, cf, cst = 0;
                    hinge_pos(k, h, cf);
                    for (int t = 0; t < 3; ++t) {
                        const uint32_t v = L.e[3 * k + t];
                        if (v != (uint32_t)L.hinge[k] && idep[3 * i + t] < 0) cst += L.xval[v];
                    }
                    rinfo[i] = (int16_t)(((h + 3 * 64 - cst) % 3) | (cf == 2 ? 4u : 0u));
                }
                __syncthreads();
                wg_excl_scan3(roff, r + 1, L.xe + Lds::CMAX);  // (16 words past st[]; xe holds Lds::NVMAX)
                for (uint32_t R = tid; R < r; R += GS_THREADS) rcur[R] = roff[R];
                __syncthreads();
                for (uint32_t i = tid; i < sz; i += GS_THREADS)
                    if (st[i] == 1) rlist[atomicAdd(&rcur[rnd[i]], 1u)] = (int16_t)i;
                __syncthreads();
                // the levels, with register arrays of exactly HW words (the
                // FW-word form spilled part of them to scratch at the
                // kernel's 128-VGPR limit: a scratch round trip per member)
                // (wave 0 alone with a wave fence per level instead of the
                // workgroup barrier: forms 4.13e6 -> 4.59e6 cycles, not kept;
                // the next level's members read from LDS during this level's
                // loads: forms 4.11e6 -> 4.39e6, more spills, not kept)
                // A word of a form per thread (H threads a member, adjacent
                // lanes on adjacent words: the dependencies' forms read as
                // consecutive 16-byte pairs); a level's VALU spreads over H
                // times the lanes of the member-per-thread form, whose one
                // wave carried a typical level's ~20 members alone.
                auto form_levels = [&](auto hw) {
                    constexpr uint32_t H = decltype(hw)::value;
                    for (uint32_t R = 0; R < r; ++R) {
                        const uint32_t o0 = uni(roff[R]), nR = uni(roff[R + 1]) - o0;
                        if (nR == 0) continue;  // (uniform)
                        for (uint32_t t = tid; t < nR * H; t += GS_THREADS) {
                            const uint32_t mi = t / H, w = t - mi * H;
                            const uint32_t i = (uint32_t)rlist[o0 + mi];
                            const int d0 = idep[3 * i], d1 = idep[3 * i + 1], d2 = idep[3 * i + 2];
                            const uint32_t info = (uint32_t)rinfo[i];
                            uint64_t a1 = 0, a2 = 0;
                            if (d0 >= 0) gf3_add(a1, a2, V(d0, w, 0), V(d0, w, 1));
                            if (d1 >= 0) gf3_add(a1, a2, V(d1, w, 0), V(d1, w, 1));
                            if (d2 >= 0) gf3_add(a1, a2, V(d2, w, 0), V(d2, w, 1));
                            // x = cf * (h - sum): -sum has the planes swapped;
                            // add h - cst in the constant column of (a2, a1)
                            const uint32_t kk = info & 3u;
                            if (w == cw) gf3_add(a2, a1, kk == 1 ? cbit : 0, kk == 2 ? cbit : 0);
                            // times cf = 2 swaps the planes back
                            V(i, w, 0) = (info & 4u) ? a1 : a2;
                            V(i, w, 1) = (info & 4u) ? a2 : a1;
                        }
                        __syncthreads();
                    }
                };
                switch (HW) {
                    case 1: form_levels(std::integral_constant<uint32_t, 1>{}); break;
                    case 2: form_levels(std::integral_constant<uint32_t, 2>{}); break;
                    case 3: form_levels(std::integral_constant<uint32_t, 3>{}); break;
                    case 4: form_levels(std::integral_constant<uint32_t, 4>{}); break;
                    case 5: form_levels(std::integral_constant<uint32_t, 5>{}); break;
                    default: form_levels(std::integral_constant<uint32_t, FW>{}); break;
                }
                pc.lap(GP_FVS_FORMS);
                // the heavy members' equations: cf*x_j + forms = h, in LDS
                // (the forms' selection arrays are dead now) when they fit
                const bool hs_lds = (size_t)2 * HW * nH <= Lds::HS_WORDS;
                // the panel form: its scratch in LDS past the rows (rows in
                // the global scratch: the whole region)
                const size_t pscr = gj_panel_words(nH);
                // (LDS state only: the following waves poll the leader's
                // progress word, which a global slab -- SolveBig -- would put
                // behind the vector L1)
                const bool panel = GOV_GJ_PANEL && !std::is_same<Lds, SolveBig>::value && nH <= (uint32_t)GS_THREADS &&
                                   hs_lds && (size_t)2 * HW * nH + pscr <= Lds::HS_WORDS;
                uint64_t *const hsb = L.hs();
                auto HSL = [&](uint32_t rr, uint32_t w, uint32_t q) -> uint64_t & { return hsb[(2 * w + q) * nH + rr]; };
                // a word of a heavy row per thread (as the forms)
                for (uint32_t t = tid; t < sz * HW; t += GS_THREADS) {
                    const uint32_t i = t / HW, w = t - i * HW;
                    if (st[i] != 2) continue;
                    const uint32_t k = (uint32_t)L.members[beg + i], j = (uint32_t)hid[i];
                    uint64_t a1 = 0, a2 = 0;
                    uint32_t cst = 0, h, cf;
                    // the member's other vertices: in-block ones as forms, the
                    // rest as known values
                    for (int t3 = 0; t3 < 3; ++t3) {
                        const uint32_t v = L.e[3 * k + t3];
                        if (v == (uint32_t)L.hinge[k]) continue;
                        const int o = L.vowner[v];
                        if (o >= 0 && L.col_of[o] >= 0) {
                            const uint32_t d = (uint32_t)L.col_of[o];
                            gf3_add(a1, a2, V(d, w, 0), V(d, w, 1));
                        } else {
                            cst += L.xval[v];
                        }
                    }
                    hinge_pos(k, h, cf);
                    if (w == (j >> 6)) gf3_add(a1, a2, cf == 1 ? 1ULL << (j & 63) : 0, cf == 2 ? 1ULL << (j & 63) : 0);
                    if (w == cw) {
                        // the forms' constant column moves to the right-hand
                        // side: rhs = h - cst - const
                        const uint32_t cform = (a1 & cbit) ? 1 : (a2 & cbit) ? 2 : 0;
                        a1 &= ~cbit;
                        a2 &= ~cbit;
                        const uint32_t rhs = (h + 3 * 64 - cst - cform) % 3;
                        gf3_add(a1, a2, rhs == 1 ? cbit : 0, rhs == 2 ? cbit : 0);
                    }
                    if (hs_lds) {
                        HSL(j, w, 0) = a1;
                        HSL(j, w, 1) = a2;
                    } else {
                        X(j, w, 0) = a1;
                        X(j, w, 1) = a2;
                    }
                }
                __syncthreads();
                // (rows in X: words < 12 CMAX, below the forms)
                // the register form when the heavy rows are in LDS, one per
                // thread, with room past them for the wave slots
                constexpr uint32_t NWV = GS_THREADS / 64;
                const bool reg = GOV_GJ_REG && hs_lds && nH <= (uint32_t)GS_THREADS && HW <= GOV_GJ_REG_HW &&
                                 (size_t)2 * HW * nH + (size_t)2 * NWV * (2 * HW + 1) <= Lds::HS_WORDS;
                bool hok;
                if (reg) {
                    uint64_t *slots = hsb + (size_t)2 * HW * nH;
                    switch (HW) {
                        case 1: hok = gauss_jordan_reg(nH, std::integral_constant<uint32_t, 1>{}, HSL, slots); break;
                        case 2: hok = gauss_jordan_reg(nH, std::integral_constant<uint32_t, 2>{}, HSL, slots); break;
                        case 3: hok = gauss_jordan_reg(nH, std::integral_constant<uint32_t, 3>{}, HSL, slots); break;
                        case 4: hok = gauss_jordan_reg(nH, std::integral_constant<uint32_t, GOV_GJ_REG_HW < 4 ? 1 : 4>{}, HSL, slots); break;
                        case 5: hok = gauss_jordan_reg(nH, std::integral_constant<uint32_t, GOV_GJ_REG_HW < 5 ? 1 : 5>{}, HSL, slots); break;
                        default: hok = gauss_jordan_reg(nH, std::integral_constant<uint32_t, GOV_GJ_REG_HW < 6 ? 1 : FW>{}, HSL, slots); break;
                    }
                } else if (panel) {
                    hok = gauss_jordan_panel(nH, HSL, hsb + (size_t)2 * HW * nH);
                } else {
                    hok = hs_lds ? gauss_jordan(nH, HSL) : gauss_jordan(nH, X);
                }
                pc.lap(GP_FVS_GJ);
                if (!hok) {
                    pc.add(GP_N_FAIL_INCONS, 1);
                    return false;
                }
                const uint32_t nfree = uni(L.nfree);
                // evaluate: x_i = forms . (x_heavy, 1)
                uint64_t *X1 = L.prow, *X2 = L.prow + 8;
                for (uint32_t w = tid; w < 16; w += GS_THREADS) L.prow[w] = 0;
                __syncthreads();
                for (uint32_t j = tid; j < nH; j += GS_THREADS) {
                    if (colval[j] == 1) atomicOr((unsigned long long *)&X1[j >> 6], 1ULL << (j & 63));
                    if (colval[j] == 2) atomicOr((unsigned long long *)&X2[j >> 6], 1ULL << (j & 63));
                }
                __syncthreads();
                for (uint32_t i = tid; i < sz; i += GS_THREADS) {
                    const uint32_t k = (uint32_t)L.members[beg + i];
                    uint32_t val;
                    if (st[i] == 2) {
                        val = colval[hid[i]];
                    } else {
                        uint32_t s = 0;
                        for (uint32_t w = 0; w < HW; ++w) {
                            const uint64_t p1 = V(i, w, 0), p2 = V(i, w, 1);
                            s += __builtin_popcountll(p1 & X1[w]) + 2 * __builtin_popcountll(p1 & X2[w]) +
                                 2 * __builtin_popcountll(p2 & X1[w]) + __builtin_popcountll(p2 & X2[w]);
                        }
                        s += (V(i, cw, 0) & cbit) ? 1 : (V(i, cw, 1) & cbit) ? 2 : 0;
                        val = s % 3;
                    }
                    L.xval[L.hinge[k]] = (uint8_t)val;
                }
                __syncthreads();
                if (nfree && nfree <= NB_MAX) {
                    // x0 above solves the block; with a singular heavy system
                    // the block's solutions are x0 + span{T z_f}, z_f the heavy
                    // null vectors (z_f: x_f = 1 at free heavy column f, 0 at
                    // the other free ones, -cf_c * a_cf at pivot column c).  The
                    // canonical solution has 0 at the block's free columns =
                    // the last nonzero positions (in member = increasing edge
                    // order) of its null vectors: the T z_f are reduced to a
                    // basis n_p with distinct last nonzero p, n_p[p] = 1 and 0
                    // at the other basis positions, and x = x0 - sum x0[p] n_p.
                    pc.add(GP_N_SING_SOLVED, 1);
                    pc.add(GP_N_NULL_VECS, nfree);
                    const int16_t *piv = L.a0;
                    uint8_t *coef = L.b1;                                   // (GJ's marks are dead)
                    int16_t *bpos = reinterpret_cast<int16_t *>(L.hbin);    // basis positions (NB_MAX)
                    uint8_t *nbv = reinterpret_cast<uint8_t *>(scr + (size_t)30 * Lds::CMAX);  // past the reverse CSR
                    auto NBV = [&](uint32_t l, uint32_t i) -> uint8_t & { return nbv[(size_t)l * Lds::CMAX + i]; };
                    auto HSA = [&](uint32_t rr, uint32_t w, uint32_t q) -> uint64_t { return hs_lds ? HSL(rr, w, q) : X(rr, w, q); };
                    uint64_t *Z1 = L.prow, *Z2 = L.prow + 8;
                    uint32_t nb = 0;
                    for (uint32_t f = 0; f < nH; ++f) {
                        if (piv[f] >= 0) continue;  // (uniform)
                        for (uint32_t w = tid; w < 16; w += GS_THREADS) L.prow[w] = 0;
                        if (tid == 0) L.npos = 0;
                        __syncthreads();
                        for (uint32_t cc = tid; cc < nH; cc += GS_THREADS) {
                            const int pr = piv[cc];
                            uint32_t zc = 0;
                            if (cc == f) {
                                zc = 1;
                            } else if (pr >= 0) {
                                const uint64_t fbit = 1ULL << (f & 63), cbit = 1ULL << (cc & 63);
                                const uint32_t av = (HSA(pr, f >> 6, 0) & fbit) ? 1 : (HSA(pr, f >> 6, 1) & fbit) ? 2 : 0;
                                const uint32_t cf = (HSA(pr, cc >> 6, 1) & cbit) ? 2 : 1;
                                zc = (3 - cf * av % 3) % 3;
                            }
                            if (zc) atomicOr((unsigned long long *)&(zc == 1 ? Z1 : Z2)[cc >> 6], 1ULL << (cc & 63));
                        }
                        __syncthreads();
                        // u = T z: the forms without their constant column (z has
                        // no bit there); a heavy member's form is its unit vector
                        for (uint32_t i = tid; i < sz; i += GS_THREADS) {
                            uint32_t sm = 0;
                            for (uint32_t w = 0; w < HW; ++w) {
                                const uint64_t p1 = V(i, w, 0), p2 = V(i, w, 1);
                                sm += __builtin_popcountll(p1 & Z1[w]) + 2 * __builtin_popcountll(p1 & Z2[w]) +
                                      2 * __builtin_popcountll(p2 & Z1[w]) + __builtin_popcountll(p2 & Z2[w]);
                            }
                            NBV(nb, i) = (uint8_t)(sm % 3);
                        }
                        __syncthreads();
                        for (uint32_t l = tid; l < nb; l += GS_THREADS) coef[l] = NBV(nb, (uint32_t)bpos[l]);
                        __syncthreads();
                        for (uint32_t i = tid; i < sz; i += GS_THREADS) {
                            uint32_t t = 0;
                            for (uint32_t l = 0; l < nb; ++l) t += coef[l] * NBV(l, i);
                            const uint32_t u = (NBV(nb, i) + 2 * t) % 3;  // u - t (mod 3)
                            NBV(nb, i) = (uint8_t)u;
                            if (u) atomicMax(&L.npos, i + 1);
                        }
                        __syncthreads();
                        const uint32_t pnew = uni(L.npos) - 1;  // (T z is independent of the basis: npos > 0)
                        const uint32_t sc = NBV(nb, pnew);  // 1 or 2 = its own inverse
                        for (uint32_t l = tid; l < nb; l += GS_THREADS) coef[l] = NBV(l, pnew);
                        __syncthreads();
                        for (uint32_t i = tid; i < sz; i += GS_THREADS) {
                            const uint32_t u = NBV(nb, i) * sc % 3;
                            NBV(nb, i) = (uint8_t)u;
                            for (uint32_t l = 0; l < nb; ++l) NBV(l, i) = (uint8_t)((NBV(l, i) + 2 * coef[l] * u) % 3);
                        }
                        if (tid == 0) bpos[nb] = (int16_t)pnew;
                        __syncthreads();
                        ++nb;
                    }
                    for (uint32_t l = tid; l < nb; l += GS_THREADS)
                        coef[l] = L.xval[L.hinge[L.members[beg + (uint32_t)bpos[l]]]];
                    __syncthreads();
                    for (uint32_t i = tid; i < sz; i += GS_THREADS) {
                        uint32_t t = 0;
                        for (uint32_t l = 0; l < nb; ++l) t += coef[l] * NBV(l, i);
                        uint8_t &xv = L.xval[L.hinge[L.members[beg + i]]];
                        xv = (uint8_t)((xv + 2 * t) % 3);
                    }
                    __syncthreads();
                }
                // (more null vectors than NB_MAX, never seen: the whole-block
                // Gauss-Jordan below)
                solved = nfree <= NB_MAX;
            }
        }
        if (!solved) {
            const uint32_t W = (sz + 1 + 63) / 64;
            for (uint32_t rr = tid; rr < sz; rr += GS_THREADS) {
                for (uint32_t w = 0; w < W; ++w) X(rr, w, 0) = X(rr, w, 1) = 0;
                const int k = L.members[beg + rr];
                int h = 0;
                while (L.e[3 * k + h] != (uint32_t)L.hinge[k]) ++h;
                uint32_t sub = 0;
                for (int i = 0; i < 3; ++i) {
                    const uint32_t v = L.e[3 * k + i];
                    const int o = L.vowner[v];
                    if (o >= 0 && L.col_of[o] >= 0) {
                        const uint32_t cc = (uint32_t)L.col_of[o];
                        gf3_add(X(rr, cc >> 6, 0), X(rr, cc >> 6, 1), 1ULL << (cc & 63), 0);
                    } else {
                        sub += L.xval[v];
                    }
                }
                const uint32_t rhs = ((uint32_t)h + 6 - sub % 3) % 3;
                if (rhs == 1) X(rr, sz >> 6, 0) |= 1ULL << (sz & 63);
                if (rhs == 2) X(rr, sz >> 6, 1) |= 1ULL << (sz & 63);
            }
            if (!gauss_jordan(sz, X)) {
                pc.add(GP_N_FAIL_INCONS, 1);
                return false;
            }
            for (uint32_t cc = tid; cc < sz; cc += GS_THREADS) L.xval[L.hinge[L.members[beg + cc]]] = colval[cc];
        }
        for (uint32_t i = tid; i < sz; i += GS_THREADS) L.col_of[L.members[beg + i]] = -1;
        __syncthreads();
        pc.lap(GP_DENSE);
        pc.add(GP_N_DENSE_ROWS, sz);
        pc.max(GP_N_DENSE_MAX, sz);
        pc.add(GP_N_BLOCKS, 1);
        if (sz > 440) pc.add(GP_N_BIG_ROWS, sz);
        ++c;
    }
    if (!uni(L.flag)) return false;

    // ---- 4. peeled edges, last round first
#if GOV_BACK_NOBARRIER
    // An edge's value needs only its other vertices' final values (hinges of
    // edges peeled in later rounds, core hinges, or free vertices = 0), so
    // no barrier per round: a peeled edge's hinge is marked pending, and each
    // wave retries its lanes' pending edges until they are solved, reading
    // the other waves' results as they land (LDS, no caching).  The later
    // rounds' edges are always ready, so every retry makes progress; the
    // values are those of the rounds in order.
    {
        constexpr uint8_t PEND = 0x80u;
        for (uint32_t k = tid; k < cnt; k += GS_THREADS)
            if (L.round_of[k] >= 0) L.xval[L.hinge[k]] = PEND;
        __syncthreads();
        volatile uint8_t *xv = L.xval;
        constexpr uint32_t KPT = (Lds::CMAX + GS_THREADS - 1) / GS_THREADS;
        uint32_t todo = 0;  // bit j: edge tid + j * GS_THREADS still to solve
        for (uint32_t j = 0; j < KPT && tid + j * GS_THREADS < cnt; ++j)
            if (L.round_of[tid + j * GS_THREADS] >= 0) todo |= 1u << j;
        static_assert(KPT <= 32, "edges a thread");
        while (__builtin_amdgcn_ballot_w64(todo != 0)) {  // (the wave's own loop)
            for (uint32_t j = 0; j < KPT; ++j) {
                if (!((todo >> j) & 1u)) continue;
                const uint32_t k = tid + j * GS_THREADS;
                const uint32_t hg = (uint32_t)L.hinge[k];
                uint32_t s = 0, coef = 0, h = 3;
                bool ready = true;
                for (int i = 0; i < 3; ++i) {
                    const uint32_t v = L.e[3 * k + i];
                    if (v == hg) {
                        ++coef;
                        if (h == 3) h = (uint32_t)i;
                    } else {
                        const uint32_t x = xv[v];
                        ready = ready && !(x & PEND);
                        s += x;
                    }
                }
                if (!ready) continue;
                const uint32_t rhs = (h + 6 - s) % 3;
                xv[hg] = (uint8_t)(coef == 1 ? rhs : (2 * rhs) % 3);
                todo &= ~(1u << j);
            }
        }
        __syncthreads();
    }
#else
    for (int rr = rounds - 1; rr >= 0; --rr) {
        for (uint32_t k = tid; k < cnt; k += GS_THREADS) {
            if (L.round_of[k] != rr) continue;
            int h = 0;
            while (L.e[3 * k + h] != (uint32_t)L.hinge[k]) ++h;
            uint32_t s = 0, coef = 0;
            for (int i = 0; i < 3; ++i) {
                if (L.e[3 * k + i] == (uint32_t)L.hinge[k]) ++coef;
                else s += L.xval[L.e[3 * k + i]];
            }
            const uint32_t rhs = ((uint32_t)h + 6 - s) % 3;
            L.xval[L.hinge[k]] = (uint8_t)(coef == 1 ? rhs : (2 * rhs) % 3);
        }
        __syncthreads();
    }
#endif
    (void)rounds;
    pc.lap(GP_BACK);
    return true;
}

template <class Lds, class PC>
__device__ __forceinline__ void store_bucket(Lds &L, const SolveArgs &a, uint64_t b, uint32_t j, PC &pc);

// Solves bucket b with state L (LDS or a global slab) and stores its values
// and local seed.  Workgroup-uniform.
template <class Lds, class PC>
__device__ __forceinline__ void solve_bucket(Lds &L, const SolveArgs &a, uint64_t b, uint64_t *scr, PC &pc) {
    const uint64_t lo = a.E[b] & OFFSET_MASK, hi = a.E[b + 1] & OFFSET_MASK;
    const uint32_t cnt = (uint32_t)(hi - lo);
    const uint64_t vo = vertex_offset(lo);
    const uint32_t nv = (uint32_t)(vertex_offset(hi) - vo);
    if (cnt == 0) return;
    if (cnt > (uint32_t)Lds::CMAX || nv > (uint32_t)Lds::NVMAX) {
        if (threadIdx.x == 0) atomicOr(a.status, (uint32_t)GOV_TOO_BIG);
        return;
    }
    const ulonglong2 *sig = reinterpret_cast<const ulonglong2 *>(a.sig) + (lo - a.e0);
    uint32_t j = 0;
    for (; j < 256; ++j) {
        const uint64_t t_try = pc.on() ? clock64() : 0;
        if (try_seed(L, sig, cnt, nv, (uint64_t)j << 56, scr, pc, a.fvs_max)) break;
        if (pc.on()) pc.add(GP_FAILED_CYCLES, clock64() - t_try);
    }
    pc.start();
    if (j == 256) {
        if (threadIdx.x == 0) atomicOr(a.status, (uint32_t)GOV_SEEDS);
        return;
    }
    store_bucket(L, a, b, j, pc);
}

// Stores bucket b's solution (L after a successful try_seed with seed j):
// its 2-bit values, the seed in E[b]'s top byte and the F2 / A11 / A13
// outputs.  Workgroup-uniform.
template <class Lds, class PC>
__device__ __forceinline__ void store_bucket(Lds &L, const SolveArgs &a, uint64_t b, uint32_t j, PC &pc) {
    const uint64_t lo = a.E[b] & OFFSET_MASK, hi = a.E[b + 1] & OFFSET_MASK;
    const uint32_t cnt = (uint32_t)(hi - lo);
    const uint64_t vo = vertex_offset(lo);
    const uint32_t nv = (uint32_t)(vertex_offset(hi) - vo);
    const ulonglong2 *sig = reinterpret_cast<const ulonglong2 *>(a.sig) + (lo - a.e0);
    // values: hinge -> xval or 3, other vertices 0; words shared with the
    // neighbouring buckets are OR-ed.  A vertex per lane: a wave's two 32-lane
    // halves are two aligned value words, packed from the lanes' two bit
    // planes (ballots) by lanes 0 and 32
    const uint64_t w0 = vo >> 5, w1 = (vo + nv + 31) >> 5;
    static_assert(GS_THREADS % 64 == 0, "whole waves");
    auto spread = [](uint32_t x32) {  // bit t -> bit 2t
        uint64_t x = x32;
        x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
        x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
        x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
        x = (x | (x << 2)) & 0x3333333333333333ull;
        return (x | (x << 1)) & 0x5555555555555555ull;
    };
    for (uint64_t p0 = w0 * 32; p0 < w1 * 32; p0 += GS_THREADS) {  // (uniform)
        const uint64_t pos = p0 + threadIdx.x;
        uint32_t val = 0;
        if (pos >= vo && pos < vo + nv) {
            const uint32_t v = (uint32_t)(pos - vo);
            val = L.vowner[v] >= 0 ? (L.xval[v] ? L.xval[v] : 3u) : 0u;
        }
        const uint64_t pl = __builtin_amdgcn_ballot_w64((val & 1u) != 0), ph = __builtin_amdgcn_ballot_w64((val & 2u) != 0);
        if ((threadIdx.x & 31) == 0) {
            const uint64_t w = pos >> 5;
            const uint32_t sh = threadIdx.x & 32;
            const uint64_t word = spread((uint32_t)(pl >> sh)) | (spread((uint32_t)(ph >> sh)) << 1);
            const bool inner = w * 32 >= vo && (w + 1) * 32 <= vo + nv;
            if (w < w1) {
                if (inner) a.values[w] = word;
                else if (word) atomicOr((unsigned long long *)(a.values + w), (unsigned long long)word);
            }
        }
    }
    if (threadIdx.x == 0) a.E[b] |= (uint64_t)j << 56;
    if (a.width || a.rank_out || a.index_out) {
        uint32_t *pre = L.deg;  // (dead after the solve) hinge vertices before v
        for (uint32_t v = threadIdx.x; v < nv; v += GS_THREADS) pre[v] = L.vowner[v] >= 0 ? 1u : 0u;
        __syncthreads();
        wg_excl_scan3(pre, nv, L.xe + Lds::CMAX);
        const uint64_t mask = a.width == 64 ? ~0ULL : ((1ULL << a.width) - 1);
        for (uint32_t k = threadIdx.x; k < cnt; k += GS_THREADS) {
            const uint64_t r = lo + pre[L.hinge[k]];
            if (a.rank_out) a.rank_out[a.pay[lo - a.e0 + k]] = (int64_t)r;
            if (a.index_out) {
                const uint64_t p = a.pay[lo - a.e0 + k];
                a.index_out[r - a.idx_lo] = __builtin_bswap64(a.addr ? a.addr[p] : a.addr_base + a.addr_stride * p);
            }
            if (a.width) {
                const uint64_t val = sig[k].x & mask, bit = r * a.width, word = bit >> 6;
                const uint32_t off = (uint32_t)(bit & 63);
                if (val) {
                    atomicOr((unsigned long long *)(a.sigbits + word), (unsigned long long)(val << off));
                    if (off + a.width > 64)
                        atomicOr((unsigned long long *)(a.sigbits + word + 1), (unsigned long long)(val >> (64 - off)));
                }
            }
        }
    }
    __syncthreads();
    pc.lap(GP_STORE);
}

__device__ __forceinline__ uint32_t ld_agent(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_agent64(const unsigned long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// all seeds below s of local bucket lb failed
__device__ __forceinline__ bool lower_seeds_failed(const SeedLedger &g, uint32_t lb, uint32_t s) {
    for (uint32_t w = 0; w * 64 < s; ++w) {
        const unsigned long long want = s >= (w + 1) * 64 ? ~0ULL : ((1ULL << (s - w * 64)) - 1);
        if ((ld_agent64(g.fail + 4 * (size_t)lb + w) & want) != want) return false;
    }
    return true;
}

template <bool PROF>
__global__ __launch_bounds__(GS_THREADS, GS_THREADS * GS_PER_CU / 256) void k_gov_solve(SolveArgs a) {
    __shared__ SolveLds L;
    uint64_t *scr = a.scratch + (size_t)blockIdx.x * solve_scratch_words<SolveLds>();
    PhaseClock<PROF> pc{PROF && a.prof ? a.prof + (size_t)blockIdx.x * GP_N : nullptr, 0};
    const SeedLedger &g = a.led;
    const uint32_t nb = (uint32_t)(a.m - a.b0);
    // buckets from a queue (status[2], zeroed with the status word): seed
    // retries make per-bucket cost uneven, a static stride left the slowest
    // workgroup ~13 % (C2) to ~40 % (1e7 keys) behind the mean.  A workgroup
    // stays on its bucket until it is done; with the queue empty it tries
    // the next seeds of other workgroups' buckets (the seed ledger).
    __shared__ uint32_t sh_lb, sh_s, sh_win;
    uint32_t cur = 0xFFFFFFFFu;  // (thread 0) this workgroup's bucket
    bool queue_open = true;      // (thread 0)
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t lb = 0xFFFFFFFFu, sd = 0;
            // 1. more seeds of my own bucket
            if (cur != 0xFFFFFFFFu && !ld_agent(g.done + cur) && ld_agent(g.won + cur) == 0) {
                sd = atomicAdd(g.claim + cur, 1u);
                if (sd < 256) lb = cur;
            }
            // 2. a new bucket from the queue
            while (lb == 0xFFFFFFFFu && queue_open) {
                const uint32_t q = atomicAdd(a.status + 2, 1u);
                if (q >= nb) {
                    queue_open = false;
                    break;
                }
                const uint64_t b = a.b0 + q;
                if ((a.E[b + 1] & OFFSET_MASK) - (a.E[b] & OFFSET_MASK) > (uint64_t)GS_CMAX) continue;  // k_gov_solve_big
                cur = q;
                __hip_atomic_store(g.active + blockIdx.x, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                sd = atomicAdd(g.claim + q, 1u);
                if (sd < 256) lb = q;
            }
            // 3. the next seed of a bucket another workgroup still solves
            // (with fewer than spec & 0xFF of its seeds in flight)
            const uint32_t cap = a.spec & 0xFFu;
            for (uint32_t k = 0; lb == 0xFFFFFFFFu && !queue_open && k < gridDim.x; ++k) {
                const uint32_t o = ld_agent(g.active + (blockIdx.x + k) % gridDim.x);
                if (o == 0xFFFFFFFFu || ld_agent(g.done + o) || ld_agent(g.won + o)) continue;
                if (cap) {
                    const uint32_t cl = ld_agent(g.claim + o);
                    uint32_t nf = 0;
                    for (uint32_t w = 0; w * 64 < cl && w < 4; ++w) nf += (uint32_t)__builtin_popcountll(ld_agent64(g.fail + 4 * (size_t)o + w));
                    if (cl - nf >= cap) continue;
                }
                sd = atomicAdd(g.claim + o, 1u);
                if (sd < 256) lb = o;
            }
            sh_lb = lb;
            sh_s = sd;
            sh_win = lb != cur;  // (a speculative attempt)
        }
        __syncthreads();
        const uint32_t lb = uni(sh_lb), sd = uni(sh_s);
        if (lb == 0xFFFFFFFFu) break;
        if (a.spec & 0x100u) {
            if (sh_win) __builtin_amdgcn_s_setprio(0);
            else __builtin_amdgcn_s_setprio(2);
        }
        const uint64_t b = a.b0 + lb;
        // (the bucket's bounds as scalars: every phase's loops are bounded by them)
        const uint64_t lo = readfirstlane64(a.E[b] & OFFSET_MASK), hi = readfirstlane64(a.E[b + 1] & OFFSET_MASK);
        const uint32_t cnt = (uint32_t)(hi - lo);
        const uint32_t nv = (uint32_t)(vertex_offset(hi) - vertex_offset(lo));
        if (cnt == 0) {  // nothing to solve: seed 0, no values
            if (threadIdx.x == 0 && sd == 0) __hip_atomic_store(g.done + lb, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            continue;
        }
        if (nv > (uint32_t)SolveLds::NVMAX) {
            if (threadIdx.x == 0) {
                atomicOr(a.status, (uint32_t)GOV_TOO_BIG);
                __hip_atomic_store(g.done + lb, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            continue;
        }
        const ulonglong2 *sig = reinterpret_cast<const ulonglong2 *>(a.sig) + (lo - a.e0);
        const uint64_t t_try = pc.on() ? clock64() : 0;
        const bool ok = try_seed(L, sig, cnt, nv, (uint64_t)sd << 56, scr, pc, a.fvs_max);
        if (threadIdx.x == 0) {
            uint32_t win = 0;
            if (!ok) {
                atomicOr(g.fail + 4 * (size_t)lb + sd / 64, 1ULL << (sd & 63));
                if (lower_seeds_failed(g, lb, 256)) {  // every seed failed (GOV:431); the last to fail sees it
                    atomicOr(a.status, (uint32_t)GOV_SEEDS);
                    __hip_atomic_store(g.done + lb, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            } else {
                atomicMax(g.won + lb, 256u - sd);
                for (;;) {  // the bucket's seed only when every lower seed failed
                    if (ld_agent(g.won + lb) > 256u - sd) break;  // a lower seed solved it
                    if (lower_seeds_failed(g, lb, sd)) {
                        win = 1;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(4);
                }
            }
            sh_win = win;
        }
        __syncthreads();
        if (!ok) {
            if (pc.on()) pc.add(GP_FAILED_CYCLES, clock64() - t_try);
            continue;
        }
        if (!sh_win) {
            pc.add(GP_N_SPEC_LOST, 1);
            continue;
        }
        pc.start();
        store_bucket(L, a, b, sd, pc);
        if (threadIdx.x == 0) {
            __threadfence();
            __hip_atomic_store(g.done + lb, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// whether oversized bucket b fits k_gov_solve_mid's LDS state
__device__ __forceinline__ bool mid_bucket(const SolveArgs &a, uint64_t b) {
    const uint64_t lo = a.E[b] & OFFSET_MASK, hi = a.E[b + 1] & OFFSET_MASK;
    return hi - lo <= (uint64_t)GM_CMAX && vertex_offset(hi) - vertex_offset(lo) <= (uint64_t)SolveMid::NVMAX;
}

// The oversized buckets of k_big_list that fit GM_CMAX: state in LDS (one
// workgroup per CU), dense scratch per workgroup in global memory.
__global__ __launch_bounds__(GS_THREADS) void k_gov_solve_mid(SolveArgs a, const uint32_t *list, uint32_t nbig,
                                                              uint64_t *scratch) {
    __shared__ SolveMid L;
    uint64_t *scr = scratch + (size_t)blockIdx.x * solve_scratch_words<SolveMid>();
    PhaseClock<false> pc{nullptr, 0};
    for (uint32_t li = blockIdx.x; li < nbig; li += gridDim.x)
        if (mid_bucket(a, a.b0 + list[li])) solve_bucket(L, a, a.b0 + list[li], scr, pc);
}

// The rest of them: one per workgroup at a time, solver state in a global
// slab (slabs[blockIdx.x]), dense scratch after it.
__global__ __launch_bounds__(GS_THREADS) void k_gov_solve_big(SolveArgs a, const uint32_t *list, uint32_t nbig,
                                                              uint8_t *slabs, size_t slab_bytes) {
    SolveBig &L = *reinterpret_cast<SolveBig *>(slabs + (size_t)blockIdx.x * slab_bytes);
    uint64_t *scr = reinterpret_cast<uint64_t *>(slabs + (size_t)blockIdx.x * slab_bytes + ((sizeof(SolveBig) + 255) & ~(size_t)255));
    PhaseClock<false> pc{nullptr, 0};
    for (uint32_t li = blockIdx.x; li < nbig; li += gridDim.x)
        if (!mid_bucket(a, a.b0 + list[li])) solve_bucket(L, a, a.b0 + list[li], scr, pc);
}

// bytes of one k_gov_solve_big workgroup slab (state + dense scratch)
constexpr size_t big_slab_bytes() {
    return ((sizeof(SolveBig) + 255) & ~(size_t)255) + solve_scratch_words<SolveBig>() * 8;
}

// ---- keys straight into one bucket range (sequential range builds) ----------
// The build of a bucket range from the keys themselves (resident in HBM): the
// range's buckets are counted, then its keys re-hashed and scattered to their
// bucket's cursor with their input position -- no signature array for the
// whole key set.  KIND 0: 13-byte keys (dword-aligned 16-byte windows), 1:
// fixed key_len, 2: variable length (offsets).
struct SelArgs {
    const uint8_t *keys;
    const uint64_t *off;     // KIND 2
    uint64_t blob_bytes, n;
    uint32_t key_len;        // KIND 0/1
    uint32_t mult;           // 2m
    uint32_t b_lo, nb;       // the range [b_lo, b_lo + nb)
    uint32_t *counts;        // MODE 0: per bucket of the range
    unsigned long long *cursor;  // MODE 1: next slot of each bucket (range-local positions)
    uint64_t *sorted;        // MODE 1: (sig0, sig1) pairs
    uint64_t *pay;           // MODE 1: input positions
};

__device__ __forceinline__ uint64_t sel_gload64(const uint8_t *base, uint64_t limit, uint64_t pos) {
    const uint64_t a = pos & ~3ULL;
    const uint32_t sh = (uint32_t)(pos & 3) * 8;
    auto ld = [&](uint64_t x) -> uint32_t {
        if (x + 4 <= limit) return *reinterpret_cast<const uint32_t *>(base + x);
        uint32_t w = 0;
        for (int b = 0; b < 4; ++b)
            if (x + b < limit) w |= (uint32_t)base[x + b] << (8 * b);
        return w;
    };
    return funnel64(ld(a), ld(a + 4), ld(a + 8), sh);
}

template <int MODE, int KIND>
__global__ __launch_bounds__(256) void k_sel(SelArgs a) {
    typedef unsigned int u32x4w __attribute__((ext_vector_type(4), aligned(4)));
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < a.n; i += stride) {
        uint64_t s0, s1;
        if (KIND == 0) {
            const uint64_t byte = i * 13, al = byte & ~3ULL;
            if (al + 16 <= a.blob_bytes) {
                const u32x4w w = __builtin_nontemporal_load(reinterpret_cast<const u32x4w *>(a.keys + al));
                W64 x0, x1;
                spooky13_u(w.x, w.y, w.z, w.w, (uint32_t)(byte & 3) * 8, 0, x0, x1);
                s0 = u64(x0);
                s1 = u64(x1);
            } else {
                auto rd = [&](uint32_t o) -> uint64_t { return sel_gload64(a.keys, a.blob_bytes, byte + o); };
                spooky_short(rd, 13, 0, s0, s1);
            }
        } else {
            const uint64_t pos = KIND == 2 ? a.off[i] : i * a.key_len;
            const uint32_t len = KIND == 2 ? (uint32_t)(a.off[i + 1] - pos) : a.key_len;
            auto rd = [&](uint32_t o) -> uint64_t { return sel_gload64(a.keys, a.blob_bytes, pos + o); };
            spooky_short(rd, len, 0, s0, s1);
        }
        const uint32_t rb = bucket_of_w(w64(s0), a.mult) - a.b_lo;  // (wraps below the range)
        if (rb >= a.nb) continue;
        if (MODE == 0) {
            atomicAdd(a.counts + rb, 1u);
        } else {
            const uint64_t p = atomicAdd(a.cursor + rb, 1ULL);
            reinterpret_cast<ulonglong2 *>(a.sorted)[p] = make_ulonglong2(s0, s1);
            a.pay[p] = i;
        }
    }
}

// ---- checks and E4 ownership -------------------------------------------------
// bsdb_set_verify: every local key's rank lies in [e0, e0 + n) and is hit once
// (bitmap of n bits, zeroed); with n keys that is a bijection onto the range.
__global__ __launch_bounds__(256) void k_verify_ranks(MphView v, const uint64_t *sig, uint64_t n, uint64_t e0,
                                                      unsigned long long *bitmap, uint32_t *status) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const ulonglong2 s = reinterpret_cast<const ulonglong2 *>(sig)[i];
        const uint64_t r = mph_rank(v, s.x, s.y) - e0;
        if (r >= n) {
            atomicOr(status, (uint32_t)GOV_VERIFY);
            continue;
        }
        const unsigned long long bit = 1ULL << (r & 63);
        if (atomicOr(bitmap + (r >> 6), bit) & bit) atomicOr(status, (uint32_t)GOV_VERIFY);
    }
}

// Rank g of G owns buckets [g*m/G, (g+1)*m/G): the owner of bucket b is
// floor(((b+1)*G - 1) / m).
__device__ __forceinline__ uint32_t owner_of(uint32_t b, uint64_t m, uint32_t G) {
    return (uint32_t)((((uint64_t)b + 1) * G - 1) / m);
}

constexpr int OWN_MAXR = 64;

__global__ __launch_bounds__(256) void k_owner_count(const uint64_t *sig, uint64_t n, uint32_t mult, uint64_t m,
                                                     uint32_t G, unsigned long long *counts) {
    __shared__ uint32_t h[OWN_MAXR];
    if (threadIdx.x < OWN_MAXR) h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
        atomicAdd(&h[owner_of(bucket_of_w(w64(sig[2 * i]), mult), m, G)], 1u);
    __syncthreads();
    if (threadIdx.x < G && h[threadIdx.x]) atomicAdd(counts + threadIdx.x, (unsigned long long)h[threadIdx.x]);
}

// cursor[g] starts at rank g's offset in the output.  A workgroup takes
// tiles of 1024 keys: ranks within the tile per owner from an LDS histogram,
// then ONE global atomic per owner and tile (per-key atomics on G words are
// serialised at the memory side: ~10x slower at G = 1 or 2).
__global__ __launch_bounds__(256) void k_owner_scatter(const uint64_t *sig, const uint64_t *payload, uint64_t n,
                                                       uint32_t mult, uint64_t m, uint32_t G,
                                                       unsigned long long *cursor, uint64_t *out,
                                                       uint64_t *payload_out) {
    constexpr int K = 4;
    constexpr uint64_t TILE = 256 * K;
    __shared__ uint32_t h[OWN_MAXR];
    __shared__ unsigned long long base[OWN_MAXR];
    const uint32_t tid = threadIdx.x;
    for (uint64_t t0 = (uint64_t)blockIdx.x * TILE; t0 < n; t0 += (uint64_t)gridDim.x * TILE) {
        if (tid < OWN_MAXR) h[tid] = 0;
        __syncthreads();
        ulonglong2 s[K];
        uint32_t o[K], r[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t i = t0 + k * 256 + tid;
            o[k] = G;  // none
            if (i < n) {
                s[k] = reinterpret_cast<const ulonglong2 *>(sig)[i];
                o[k] = owner_of(bucket_of_w(w64(s[k].x), mult), m, G);
                r[k] = atomicAdd(&h[o[k]], 1u);
            }
        }
        __syncthreads();
        if (tid < G && h[tid]) base[tid] = atomicAdd(cursor + tid, (unsigned long long)h[tid]);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (o[k] < G) {
                const uint64_t pos = base[o[k]] + r[k];
                reinterpret_cast<ulonglong2 *>(out)[pos] = s[k];
                if (payload) payload_out[pos] = payload[t0 + k * 256 + tid];
            }
        }
        __syncthreads();  // h and base are reused by the next tile
    }
}

}  // namespace bsdb
