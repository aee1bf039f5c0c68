// mph_kernels.hip -- MPHF evaluation on gfx950: lookup (A12), signing (A11),
// index scatter (A13).  Arithmetic follows GOV:557-580 / mph.c:63-96:
// bucket -> edgeOffsetAndSeed -> vertexOffset -> signatureToEquation (rehash
// + multiply-shift) -> three 2-bit values -> h = sum % 3 -> rank = offset +
// nonzero 2-bit fields in [vo, vo + e[h]).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "spooky_dev.hpp"

namespace bsdb {

// spooky.c:86-92 + mph.c:63-71.  nv == 0 gives e = 0 (Java shift semantics).
__device__ __forceinline__ void sig_to_equation(uint64_t sig0, uint64_t sig1, uint64_t seed_bits, uint32_t nv,
                                                uint32_t e[3]) {
    if (nv == 0) {
        e[0] = e[1] = e[2] = 0;
        return;
    }
    uint64_t h0 = seed_bits, h1 = SC + sig0, h2 = SC + sig1, h3 = SC;
    short_mix(h0, h1, h2, h3);
    const int shift = __clzll((long long)nv);
    const uint64_t mask = (1ULL << shift) - 1;
    e[0] = (uint32_t)(((h0 & mask) * nv) >> shift);
    e[1] = (uint32_t)(((h1 & mask) * nv) >> shift);
    e[2] = (uint32_t)(((h2 & mask) * nv) >> shift);
}

__device__ __forceinline__ uint32_t two_bit(const uint64_t *a, uint64_t pos) {
    return (uint32_t)(a[pos >> 5] >> ((pos & 31) * 2)) & 3u;
}

__device__ __forceinline__ uint32_t nz_pairs(uint64_t x) { return __popcll((x | (x >> 1)) & 0x5555555555555555ULL); }

// GOV:183-197
__device__ __forceinline__ uint64_t count_nonzero_pairs(uint64_t start, uint64_t end, const uint64_t *a) {
    uint64_t blk = start >> 5;
    const uint64_t end_blk = end >> 5;
    const uint32_t so = (uint32_t)(start & 31), eo = (uint32_t)(end & 31);
    if (blk == end_blk) return nz_pairs((a[blk] & ((1ULL << (eo * 2)) - 1)) >> (so * 2));
    uint64_t pairs = 0;
    if (so) pairs += nz_pairs(a[blk++] >> (so * 2));
    while (blk < end_blk) pairs += nz_pairs(a[blk++]);
    if (eo) pairs += nz_pairs(a[blk] & ((1ULL << (eo * 2)) - 1));
    return pairs;
}

struct MphView {
    const uint64_t *E;        // edgeOffsetAndSeed[m+1]
    const uint64_t *values;   // 2-bit values
    const uint64_t *sigs;     // checksum bit list (width bits per rank), or null
    uint64_t n;               // keys
    uint32_t mult;            // 2m (< 2^32)
    uint32_t width;           // hash.checksum.bits
};

// getLongBySignatureNoCheck (GOV:573-580)
__device__ __forceinline__ uint64_t mph_rank(const MphView &v, uint64_t sig0, uint64_t sig1) {
    const uint32_t b = bucket_of_w(w64(sig0), v.mult);
    const uint64_t eos = v.E[b];
    const uint64_t vo = vertex_offset(eos);
    const uint32_t nv = (uint32_t)(vertex_offset(v.E[b + 1]) - vo);
    uint32_t e[3];
    sig_to_equation(sig0, sig1, eos & ~OFFSET_MASK, nv, e);
    const uint32_t h = (two_bit(v.values, vo + e[0]) + two_bit(v.values, vo + e[1]) + two_bit(v.values, vo + e[2])) % 3;
    return (eos & OFFSET_MASK) + count_nonzero_pairs(vo, vo + e[h], v.values);
}

__device__ __forceinline__ uint64_t bitlist_get(const uint64_t *w, uint64_t i, uint32_t width) {
    const uint64_t bit = i * width, word = bit >> 6;
    const uint32_t off = (uint32_t)(bit & 63);
    const uint64_t mask = width == 64 ? ~0ULL : ((1ULL << width) - 1);
    uint64_t x = w[word] >> off;
    if (off + width > 64) x |= w[word + 1] << (64 - off);
    return x & mask;
}

// getLongBySignature (GOV:557-569): -1 when out of range or the checksum differs
__device__ __forceinline__ int64_t mph_lookup(const MphView &v, uint64_t sig0, uint64_t sig1) {
    const uint64_t r = mph_rank(v, sig0, sig1);
    if (r >= v.n) return -1;
    if (v.width) {
        const uint64_t mask = v.width == 64 ? ~0ULL : ((1ULL << v.width) - 1);
        if (bitlist_get(v.sigs, r, v.width) != (sig0 & mask)) return -1;
    }
    return (int64_t)r;
}

__global__ __launch_bounds__(256) void k_lookup(MphView v, const uint64_t *sig, uint64_t nq, int check, int64_t *out) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < nq; i += stride) {
        const ulonglong2 s = reinterpret_cast<const ulonglong2 *>(sig)[i];
        out[i] = check ? mph_lookup(v, s.x, s.y) : (int64_t)mph_rank(v, s.x, s.y);
    }
}

// A11 signing (GOV:492-508): signatures[rank(sig)] = sig0 & mask, a packed
// width-bit list; fields of adjacent ranks share words -> 64-bit atomic OR
// into a zeroed list.
__global__ __launch_bounds__(256) void k_sign(MphView v, const uint64_t *sig, uint64_t n, uint64_t *out) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    const uint64_t mask = v.width == 64 ? ~0ULL : ((1ULL << v.width) - 1);
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const ulonglong2 s = reinterpret_cast<const ulonglong2 *>(sig)[i];
        const uint64_t r = mph_rank(v, s.x, s.y);
        const uint64_t val = s.x & mask;
        const uint64_t bit = r * v.width, word = bit >> 6;
        const uint32_t off = (uint32_t)(bit & 63);
        atomicOr((unsigned long long *)(out + word), (unsigned long long)(val << off));
        if (off + v.width > 64) atomicOr((unsigned long long *)(out + word + 1), (unsigned long long)(val >> (64 - off)));
    }
}

// A13 index scatter (W:129-145): for records with rank in [start, start+len),
// index[rank-start] = reverseBytes(addr) (REVERSE_ORDER on little-endian hosts,
// Common.java:61), and for index.approximate the first min(len,8) value bytes.
__global__ __launch_bounds__(256) void k_index_scatter(const int64_t *rank, const uint64_t *addr, uint64_t count,
                                                       uint64_t start, uint64_t len, uint64_t *index,
                                                       const uint64_t *value8, const uint8_t *value_len,
                                                       uint8_t *index_a) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < count; i += stride) {
        const int64_t r = rank[i];
        if (r < 0) continue;
        const uint64_t idx = (uint64_t)r - start;
        if ((uint64_t)r < start || idx >= len) continue;
        index[idx] = __builtin_bswap64(addr[i]);
        if (index_a) {
            const uint32_t l = value_len[i] < 8 ? value_len[i] : 8;
            const uint64_t vb = value8[i];
            for (uint32_t b = 0; b < l; ++b) index_a[idx * 8 + b] = (uint8_t)(vb >> (8 * b));
        }
    }
}

}  // namespace bsdb
