// fused_kernels.hip -- the single-pass histogram of 13-byte keys
// (k_hist13_fused): hash -> bucket -> bucket-occupancy counts with the
// partition ids exchanged between CUs through a small ring that stays in the
// Infinity Cache instead of a full id stream written to and re-read from HBM
// (the two-pass design of hash_kernels.hip).  Reference loop replaced: the
// same as pass 1 + pass 2 (CBHS:360-395, GOV:385-402).  DESIGN.md §4.6.
//
// Layout: one 1024-thread workgroup per CU, grid = 256 = the bucket OWNERS.
// Owner w holds the counts of buckets [floor(w m/256), floor((w+1) m/256)]
// -- the keys whose x = sig0 >>> 1 has top byte w -- as u16 pairs in LDS
// (72 KiB), for the whole launch.  Per half-tile of 8192 keys (a ROUND):
//  * produce: hash the keys; a key's 2-byte id (bucket & 0xFFFF) goes into
//    the LDS bin of its owner (256 bins, double-buffered by round parity),
//    rank from the bin counter (slot 0 of a bin is its count header);
//  * publish: during the next round the producer writes its region of the
//    ring slot as ONE contiguous write-through (sc1) stream of 16-B chunks:
//    a 1 KiB header (per owner: first chunk << 16 | ids), then every bin's
//    ids padded to whole chunks in owner order;
//    every storing wave drains (vmcnt), a workgroup barrier, then ONE lane
//    adds 1 to the round's counter (8 shards by blockIdx % 8, u64: the high
//    word counts bin overflows);
//  * consume: lag - 1 rounds later the workgroup's poll of the round's
//    counter has matched (MI355X_MICROARCH.md § visibility, table row 1)
//    and it reads its header entry in all 256 regions (sc1); one round later
//    its bin's chunks (sc1) and adds each id into its LDS table.
// Ring slots: a round's slot is reused 2 lag - 3 rounds later; a workgroup
// writes round y only after its poll saw every workgroup finish the
// iteration that consumed round y - (2 lag - 3) (derivation in DESIGN.md).
// End: one agreement word (every workgroup adds 1 + its overflow bit); with
// no overflow anywhere every owner adds its table into counts[] (atomics:
// the two boundary buckets of a range are shared with the neighbour);
// otherwise nothing is added and the context's overflow flag makes
// k_overflow_fallback recount the keys with direct atomics.  Every spin is
// bounded (FU_SPIN_MAX polls) and a timeout aborts every workgroup
// (error word, results not added).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bsdb {

constexpr int FU_NT = 1024;
constexpr int FU_NW = FU_NT / 64;
constexpr int FU_OWNERS = 256;                 // = gridDim.x
constexpr int FU_TILE = FU_NT * 16;            // keys per super-tile (4 quarters of 4 keys per thread)
constexpr int FU_HALF = FU_TILE / 2;           // keys per round
constexpr int FU_CAPB = 80;                    // ids per LDS bin (round share 32 +- 5.7)
constexpr int FU_TCAP = 36864;                 // table buckets per owner (u16, packed in pairs): m <= 256 (FU_TCAP - 2)
constexpr int FU_LAG = 5;                      // round y is consumed in iteration y + FU_LAG
constexpr int FU_SLOTS = 8;                    // ring slots (>= 2 FU_LAG - 3; a power of two)
static_assert(FU_SLOTS >= 2 * FU_LAG - 3 && (FU_SLOTS & (FU_SLOTS - 1)) == 0, "ring slots");
constexpr int FU_SHARDS = 8;                   // counter shards (blockIdx % 8: one XCD each under round-robin placement)
constexpr int FU_LINE_U64 = 16;                // one 128-B line per counter
constexpr uint32_t FU_SPIN_MAX = 1u << 21;     // polls before a wait gives up (~seconds)
constexpr uint32_t FU_HDR_BYTES = FU_OWNERS * 4;  // a region's header: (chunk offset << 16 | ids) per owner
constexpr uint32_t FU_CHUNKS_MAX = FU_OWNERS * (FU_CAPB / 8);
constexpr uint32_t FU_REGION_BYTES = FU_HDR_BYTES + FU_CHUNKS_MAX * 16;  // 41 984 (= 328 lines)
constexpr size_t FU_SLOT_BYTES = (size_t)FU_OWNERS * FU_REGION_BYTES;   // 10.7 MB
// sync words (u64): pub[FU_SLOTS][FU_SHARDS] lines, then fin, abort and the
// end decision (0 open, FU_COMMIT, FU_ABORT: set once, by one CAS)
constexpr size_t FU_SYNC_U64 = ((size_t)FU_SLOTS * FU_SHARDS + 3) * FU_LINE_U64;
constexpr uint64_t FU_COMMIT = 1, FU_ABORT = 2;

struct FusedArgs {
    const uint8_t *keys;   // 13-byte keys, the super-tiles [0, nsuper * 256)
    uint64_t nsuper;       // super-tiles per workgroup (every workgroup the same)
    uint64_t seed;
    uint32_t mult;         // 2 m
    uint32_t m;
    uint8_t *ring;         // FU_SLOTS * FU_SLOT_BYTES
    uint64_t *sync;        // FU_SYNC_U64 words, zeroed before the launch
    uint32_t *overflow;    // [0]: the context's overflow flag (k_overflow_fallback), [3]: launches that timed out
    uint32_t *counts;      // += this launch's counts
};

typedef __attribute__((address_space(1))) uint64_t fu_gu64;

__device__ __forceinline__ uint64_t fu_load_relaxed(const uint64_t *p) {
    return __hip_atomic_load((fu_gu64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void fu_add_relaxed(uint64_t *p, uint64_t v) {
    (void)__hip_atomic_fetch_add((fu_gu64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t fu_fetch_add_relaxed(uint64_t *p, uint64_t v) {
    return __hip_atomic_fetch_add((fu_gu64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// sets *p from 0 to v unless another value got there first
__device__ __forceinline__ void fu_decide(uint64_t *p, uint64_t v) {
    uint64_t expect = 0;
    (void)__hip_atomic_compare_exchange_strong((fu_gu64 *)p, &expect, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
}

// VAR 0 is production.  Profiling only (results invalid unless noted): bit 0
// no consumer (no polls, loads or table adds), bit 1 no run stores, bit 2 no
// waits on the round counters, bit 3 per-wave phase cycles (s_memtime)
// over counts[8 (16 p + wave) + k] (nothing else added).
template <bool SEED0, int VAR = 0>
__global__ __launch_bounds__(FU_NT, 1) void k_hist13_fused(FusedArgs a) {
    constexpr bool NO_CONS = VAR & 1, NO_STORE = VAR & 2, NO_WAIT = VAR & 4, STAMP = VAR & 8;
    constexpr int NT = FU_NT, TILE = FU_TILE, L = 13, CAPB = FU_CAPB;
    const uint64_t seed = SEED0 ? 0ull : a.seed;
    __shared__ uint32_t table[FU_TCAP / 2];
    __shared__ __align__(16) uint16_t bins[2][FU_OWNERS * CAPB];
    __shared__ uint32_t cnt[3][FU_OWNERS];  // rank counters, round h in cnt[h % 3]
    __shared__ uint32_t ovf_round[2];
    __shared__ uint64_t red[FU_NW];
    __shared__ uint64_t fin_word;

    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63;
    const uint32_t p = blockIdx.x;  // producer id = owner id
    const uint32_t mult = a.mult;
    const uint64_t H = 2 * a.nsuper;  // rounds
    constexpr uint32_t LAG = FU_LAG, SLOTS = FU_SLOTS;
    const uint32_t lo = (uint32_t)(((uint64_t)p * a.m) >> 8);  // first bucket I own
    const uint32_t hi_b = (uint32_t)min((uint64_t)a.m - 1, (((uint64_t)p + 1) * a.m) >> 8);
    const uint32_t nent = hi_b - lo + 1;  // <= FU_TCAP (host plan)

    for (int i = tid; i < FU_TCAP / 2; i += NT) table[i] = 0;
    for (int i = tid; i < 3 * FU_OWNERS; i += NT) (&cnt[0][0])[i] = 0;
    if (tid < 2) ovf_round[tid] = 0;

    // owner lane of bin d = 16 w + l (l < 16)
    const bool owner = l < 16;

    u32x4a S[4][D13_Q];
    const uint32_t lane_off = ((uint32_t)tid * L) & ~3u;
    const uint32_t sh = (((uint32_t)tid * L) & 3u) * 8u;
    auto load_q = [&](auto qc, uint64_t tt) {
        constexpr int q = decltype(qc)::value;
        const uint8_t *tb = a.keys + tt * ((uint64_t)TILE * L);
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(tb), 0, TILE * L + 16, 0x00020000);
#pragma unroll
        for (int j = 0; j < D13_Q; ++j) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, lane_off, (q * D13_Q + j) * NT * L, 2);
            S[q][j] = u32x4a{v[0], v[1], v[2], v[3]};
        }
    };
    auto hash_q = [&](auto qc, uint32_t *cn, uint32_t bsel) {
        constexpr int q = decltype(qc)::value;
        uint32_t b[D13_Q], o[D13_Q], r[D13_Q];
#pragma unroll
        for (int j = 0; j < D13_Q; ++j)
            b[j] = spooky13_bucket_owner(S[q][j].x, S[q][j].y, S[q][j].z, S[q][j].w, sh, seed, mult, o[j]);
#pragma unroll
        for (int j = 0; j < D13_Q; ++j) r[j] = atomicAdd(&cn[o[j]], 1u);
#pragma unroll
        for (int j = 0; j < D13_Q; ++j) {
            const uint32_t slot = __umul24(o[j], (uint32_t)CAPB) + min(r[j], (uint32_t)CAPB - 1u);
            __builtin_assume(slot < (uint32_t)(FU_OWNERS * CAPB));
            bins[bsel][slot] = (uint16_t)b[j];
        }
    };

    // ---- publish: round y's bins (buffer y & 1) -> region (slot y % SLOTS,
    // producer p): the header, then every bin's ids as whole 16-B chunks in
    // owner order, one contiguous write-through stream.  Owner lane l < 16 of
    // wave w holds bin 16 w + l's ids (o_cnt), its first chunk (o_off) and
    // the wave's first chunk (w_off, uniform), set after the round's barrier.
    uint32_t o_cnt = 0, o_off = 0, w_off = 0;
    auto write_out = [&](uint64_t y) {
        const uint32_t buf = (uint32_t)(y & 1);
        const uint32_t slot = (uint32_t)(y % SLOTS);
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
            a.ring + (size_t)slot * FU_SLOT_BYTES + (size_t)p * FU_REGION_BYTES, 0, FU_REGION_BYTES, 0x00020000);
        if (owner) {
            const uint32_t hv = (o_off << 16) | o_cnt;
            __builtin_amdgcn_raw_buffer_store_b32(hv, rsrc, 4u * ((uint32_t)w * 16 + (uint32_t)l), 0, 16);  // sc1
        }
        const uint32_t nch = owner ? (o_cnt + 7) >> 3 : 0;
        const uint32_t st = o_off - w_off;  // owner lanes: first chunk within the wave's range
        const uint32_t total = __builtin_amdgcn_readlane(st + nch, 15);
        for (uint32_t i0 = 0; i0 < total; i0 += 64) {
            const uint32_t i = i0 + l;
            int j = 0;
#pragma unroll
            for (int step = 8; step >= 1; step >>= 1) {
                const uint32_t s_try = __shfl(st, j + step, 64);
                if (s_try <= i) j += step;
            }
            const uint32_t k = i - __shfl(st, j, 64);
            const uint32_t d = (uint32_t)w * 16 + (uint32_t)j;
            if (i < total) {
                const uint4 v = *reinterpret_cast<const uint4 *>(&bins[buf][d * CAPB + 8 * k]);
                __builtin_amdgcn_raw_buffer_store_b128(u32x4{v.x, v.y, v.z, v.w}, rsrc,
                                                       FU_HDR_BYTES + 16u * (w_off + i), 0, 16);  // sc1
            }
        }
    };
    // after round h's barrier: every wave scans all 256 bin counts (chunk
    // offsets in owner order); owner lanes keep their bin's, lane 0 the wave's
    auto plan_round = [&](uint32_t *cn) -> bool {
        uint32_t c4[4], n4[4], s = 0;
        bool ovf = false;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            c4[e] = cn[4 * l + e];
            ovf |= c4[e] > (uint32_t)CAPB;
            c4[e] = min(c4[e], (uint32_t)CAPB);
            n4[e] = (c4[e] + 7) >> 3;
            s += n4[e];
        }
        uint32_t x = s;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t yv = __shfl_up(x, d, 64);
            if (l >= d) x += yv;
        }
        const uint32_t ex = x - s;  // chunks before bin 4 l
        // bin 16 w + l (owner lanes) sits in lane 4 w + l / 4, element l & 3
        const int src = 4 * w + (l >> 2);
        const uint32_t e = (uint32_t)l & 3;
        const uint32_t pre = __shfl(ex, src, 64);
        const uint32_t c0 = __shfl(c4[0], src, 64), c1 = __shfl(c4[1], src, 64), c2 = __shfl(c4[2], src, 64),
                       c3 = __shfl(c4[3], src, 64);
        const uint32_t n0 = (c0 + 7) >> 3, n1 = (c1 + 7) >> 3, n2 = (c2 + 7) >> 3;
        o_cnt = e == 0 ? c0 : e == 1 ? c1 : e == 2 ? c2 : c3;
        o_off = pre + (e > 0 ? n0 : 0) + (e > 1 ? n1 : 0) + (e > 2 ? n2 : 0);
        w_off = __builtin_amdgcn_readfirstlane(o_off);  // lane 0 = bin 16 w
        return ovf;
    };

    // STAMP: wait, write-out, hash, consume, drain+barrier, iterations, spinning (in wait), store drain (in drain+barrier)
    uint64_t st[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ts = 0;
    // ---- consume: my bins of round y from every producer's region
    // thread t reads producer t >> 2, chunks (t & 3) + 4 i of my bin
    const uint32_t cprod = (uint32_t)tid >> 2, csub = (uint32_t)tid & 3;
    u32x4 cv[2];
    uint32_t hdr = 0;   // my bin's header in producer cprod's region, the round whose headers were read last
    uint32_t hdr_c = 0; // the same for the round being consumed (its chunks in flight)
    uint64_t poll = 0;  // this wave's poll (sum of the shards follows)
    bool dead = false;
    uint32_t consumed = 0;  // ids this thread added (table check at the end)
    uint64_t *const pub = a.sync;
    uint64_t *const fin = a.sync + (size_t)FU_SLOTS * FU_SHARDS * FU_LINE_U64;
    uint64_t *const abort_w = fin + FU_LINE_U64;
    uint64_t *const decide = abort_w + FU_LINE_U64;
    auto region_rsrc = [&](uint64_t y) {
        const uint32_t slot = (uint32_t)(y % SLOTS);
        return __builtin_amdgcn_make_buffer_rsrc(a.ring + (size_t)slot * FU_SLOT_BYTES, 0, (uint32_t)FU_SLOT_BYTES,
                                                 0x00020000);
    };
    auto issue_poll = [&](uint64_t y) {
        const uint32_t slot = (uint32_t)(y % SLOTS);
        uint64_t v = 0;
        if (l < FU_SHARDS) v = fu_load_relaxed(pub + ((size_t)slot * FU_SHARDS + l) * FU_LINE_U64);
        poll = v;
    };
    auto poll_sum = [&]() -> uint64_t {
        uint64_t v = poll;
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 4, 64);
        return __builtin_amdgcn_readfirstlane((uint32_t)v) | ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32);
    };
    bool any_ovf = false;  // a bin overflow was signalled in a round I waited for
    auto wait_round = [&](uint64_t y) {
        // every workgroup's signal of round y: 256 per use of the slot
        const uint32_t expect = (uint32_t)(FU_OWNERS * (y / SLOTS + 1));
        uint64_t v = poll_sum();
        uint32_t spins = 0;
        uint64_t t_spin = 0;
        if constexpr (STAMP) t_spin = __builtin_amdgcn_s_memtime();
        while (!dead && (uint32_t)v != expect) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > FU_SPIN_MAX || fu_load_relaxed(abort_w) != 0) {
                dead = true;
                if (l == 0) fu_add_relaxed(abort_w, 1);
                break;
            }
            issue_poll(y);
            v = poll_sum();
        }
        if constexpr (STAMP) st[6] += __builtin_amdgcn_s_memtime() - t_spin;
        any_ovf |= (v >> 32) != 0;
    };
    auto load_hdr = [&](uint64_t y) {
        hdr = __builtin_amdgcn_raw_buffer_load_b32(region_rsrc(y), cprod * FU_REGION_BYTES + 4u * p, 0, 16);  // sc1
    };
    auto chunk_off = [&](uint32_t k) { return cprod * FU_REGION_BYTES + FU_HDR_BYTES + 16u * ((hdr_c >> 16) + k); };
    auto consume_load = [&](uint64_t y) {
        hdr_c = hdr;
        const auto rsrc = region_rsrc(y);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, chunk_off(csub + 4 * i), 0, 16);  // sc1
            cv[i] = u32x4{v[0], v[1], v[2], v[3]};
        }
    };
    auto add_chunk = [&](const u32x4 &v, uint32_t chunk, uint32_t c) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const uint32_t pos = 8 * chunk + e;
            const uint32_t wv = e < 2 ? v.x : e < 4 ? v.y : e < 6 ? v.z : v.w;
            const uint32_t id = (e & 1) ? wv >> 16 : wv & 0xFFFFu;
            if (pos < c) {
                const uint32_t off = min((id - lo) & 0xFFFFu, (uint32_t)FU_TCAP - 1);
                atomicAdd(&table[off >> 1], 1u << ((off & 1) << 4));
                ++consumed;
            }
        }
    };
    auto consume_add = [&](uint64_t y) {
        const uint32_t c = min(hdr_c & 0xFFFFu, (uint32_t)CAPB);
        add_chunk(cv[0], csub, c);
        add_chunk(cv[1], csub + 4, c);
        // chunks 8, 9 (ids 64..79: a round share of 32 +- 5.7 rarely reaches them)
        const bool far = csub < 2 && c > 8 * (csub + 8);
        if (__any(far)) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(region_rsrc(y), chunk_off(csub + 8), 0, 16);  // sc1
            if (far) add_chunk(u32x4{v[0], v[1], v[2], v[3]}, csub + 8, c);
        }
    };

    // ---- one iteration h: round h hashed (h < H), round h - 1 published,
    // round h - lag consumed, round h - lag + 1's headers read, round
    // h - lag + 2 polled
    auto stamp = [&](int k) {
        if constexpr (STAMP) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            st[k] += now - ts;
            ts = now;
        }
    };
    uint32_t h3_next = 0;
    auto iter = [&](auto qc, uint64_t h, uint64_t next_t) {
        constexpr int QA = decltype(qc)::value;  // 0: quarters 0, 1; 2: quarters 2, 3; -1: drain (no hash)
        const int64_t yc = (int64_t)h - LAG, yh = yc + 1, yp = yc + 2;
        // counters of round h + 1 (last read after round h - 2's barrier)
        const uint32_t h3 = h3_next;  // h % 3
        h3_next = h3 == 2 ? 0 : h3 + 1;
        if (h + 1 < H && tid < FU_OWNERS) cnt[h3_next][tid] = 0;
        if (!NO_CONS) {
            if (yc >= 0) consume_load((uint64_t)yc);  // headers read last iteration
            if (yh >= 0 && (uint64_t)yh < H) {
                if (!NO_WAIT) wait_round((uint64_t)yh);
                load_hdr((uint64_t)yh);
            }
            if (yp >= 0 && (uint64_t)yp < H) issue_poll((uint64_t)yp);
        }
        stamp(0);
        if (!NO_STORE && h >= 1 && h - 1 < H) write_out(h - 1);
        asm volatile("" ::: "memory");  // the stores stay older than the prefetch below
        stamp(1);
        if constexpr (QA >= 0) {
            uint32_t *const cn = cnt[h3];
            const uint32_t bsel = (uint32_t)(h & 1);
            hash_q(std::integral_constant<int, QA>{}, cn, bsel);
            load_q(std::integral_constant<int, QA>{}, next_t);
            hash_q(std::integral_constant<int, QA + 1>{}, cn, bsel);
            load_q(std::integral_constant<int, QA + 1>{}, next_t);
        }
        stamp(2);
        if (!NO_CONS && yc >= 0 && !dead) consume_add((uint64_t)yc);
        stamp(3);
        // drain this wave's stores (everything but the 8 prefetch loads):
        // the signal below covers them
        if constexpr (QA >= 0)
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if constexpr (STAMP) st[7] += __builtin_amdgcn_s_memtime() - ts;
        __syncthreads();
        stamp(4);
        ++st[5];
        if (h < H) {
            const bool ovf = plan_round(cnt[h3]);
            if (ovf) ovf_round[h & 1] = 1;
        }
        if (h >= 1 && h - 1 < H && tid == 0) {
            const uint32_t pb = (uint32_t)((h - 1) & 1);
            const uint64_t ov = ovf_round[pb];
            ovf_round[pb] = 0;
            fu_add_relaxed(pub + ((size_t)((h - 1) % SLOTS) * FU_SHARDS + (p & (FU_SHARDS - 1))) * FU_LINE_U64,
                           1ull + (ov << 32));
        }
    };

    const uint64_t t0 = p;
    load_q(std::integral_constant<int, 0>{}, t0);
    load_q(std::integral_constant<int, 1>{}, t0);
    load_q(std::integral_constant<int, 2>{}, t0);
    load_q(std::integral_constant<int, 3>{}, t0);
    __syncthreads();  // table, counters zeroed
    if constexpr (STAMP) ts = __builtin_amdgcn_s_memtime();
    for (uint64_t k = 0; k < a.nsuper; ++k) {
        // past the last super-tile the loads re-read tile t0 (unconditional)
        const uint64_t nt = k + 1 < a.nsuper ? (k + 1) * FU_OWNERS + p : t0;
        iter(std::integral_constant<int, 0>{}, 2 * k, nt);
        iter(std::integral_constant<int, 2>{}, 2 * k + 1, nt);
    }
    for (uint64_t h = H; h < H + LAG; ++h) iter(std::integral_constant<int, -1>{}, h, t0);
    if constexpr (STAMP) {
        // over counts[] (results invalid): cycles / 16 per phase, iterations
        if (l == 0)
            for (int k = 0; k < 8; ++k) a.counts[((size_t)p * FU_NW + w) * 8 + k] = (uint32_t)(k != 5 ? st[k] >> 4 : st[k]);
        return;
    }

    // ---- end: my table's total against the ids I added, then the agreement
    uint64_t tsum = 0;
    for (int i = tid; i < FU_TCAP / 2; i += NT) tsum += (table[i] & 0xFFFFu) + (table[i] >> 16);
    uint64_t diff = (uint64_t)consumed - tsum;  // 0 unless a u16 count wrapped
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) diff += __shfl_xor(diff, d, 64);
    if (l == 0) red[w] = diff;
    const int any_dead = __syncthreads_or(dead ? 1 : 0);
    if (tid == 0) {
        uint64_t dsum = 0;
        for (int i = 0; i < FU_NW; ++i) dsum += red[i];
        // any_ovf of wave 0 covers every round (each wave waited on every round)
        const bool bad = dsum != 0 || any_dead || any_ovf || fu_load_relaxed(abort_w) != 0;
        // commit or abort is ONE decision for the whole grid: the
        // last workgroup to arrive sets it from every arrival's bad bit; a
        // workgroup that times out waiting sets abort instead; whichever CAS
        // lands first holds, and every workgroup acts on that value
        const uint64_t now = fu_fetch_add_relaxed(fin, 1ull + ((uint64_t)bad << 32)) + 1ull + ((uint64_t)bad << 32);
        if ((uint32_t)now == (uint32_t)gridDim.x) fu_decide(decide, (now >> 32) ? FU_ABORT : FU_COMMIT);
        uint64_t d = fu_load_relaxed(decide);
        uint32_t spins = 0;
        while (d == 0) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > FU_SPIN_MAX || fu_load_relaxed(abort_w) != 0) {
                fu_add_relaxed(abort_w, 1);
                fu_decide(decide, FU_ABORT);
            }
            d = fu_load_relaxed(decide);
        }
        fin_word = d;
        if (d == FU_ABORT) atomicOr(a.overflow, 1u);  // nothing added anywhere: the fallback recounts
        if (fu_load_relaxed(abort_w) != 0 && p == 0) atomicAdd(a.overflow + 3, 1u);  // timeouts
    }
    __syncthreads();
    if (fin_word != FU_COMMIT) return;
    for (uint32_t i = tid; i < nent; i += NT) {
        const uint32_t v = (table[i >> 1] >> ((i & 1) << 4)) & 0xFFFFu;
        if (v) atomicAdd(a.counts + lo + i, v);
    }
}

}  // namespace bsdb
