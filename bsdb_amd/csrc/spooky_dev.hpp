// spooky_dev.hpp -- SpookyHash-short, bucket map and GOV helpers as CDNA4
// device functions.  Behaviour follows the reference's C spec
// (src/main/c/spooky.c:55-175) and GOV's bucket map
// (GOVMinimalPerfectHashFunctionModified.java:559, 315-317); the code is laid
// out for 64-wide wavefronts: every 64-bit op lowers to a pair of 32-bit VALU
// ops (rotates -> v_alignbit_b32 x2, adds -> v_lshl_add_u64 / add+addc).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bsdb {

constexpr uint64_t SC = 0x9e3779b97f4a7c13ULL;  // spooky.c:39
constexpr uint64_t OFFSET_MASK = ~0ULL >> 8;    // GOV:157
#ifndef BSDB_PROBE_BUCKET_SIZE
constexpr uint32_t BUCKET_SIZE = 1500;          // GOV:281
#else
// (measurement builds only, tools/build_variant.sh: a different mean bucket
// to price the solver's LDS footprint; never the product library)
constexpr uint32_t BUCKET_SIZE = BSDB_PROBE_BUCKET_SIZE;
#endif

// 64-bit rotate by a constant as two v_alignbit_b32 (the generic shift/or form
// costs 2 v_lshl*_b64 + 2 v_or_b32).
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int k) {
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    uint32_t nhi, nlo;
    if (k < 32) {
        nhi = __builtin_amdgcn_alignbit(hi, lo, 32 - k);
        nlo = __builtin_amdgcn_alignbit(lo, hi, 32 - k);
    } else if (k == 32) {
        nhi = lo;
        nlo = hi;
    } else {
        nhi = __builtin_amdgcn_alignbit(lo, hi, 64 - k);
        nlo = __builtin_amdgcn_alignbit(hi, lo, 64 - k);
    }
    return ((uint64_t)nhi << 32) | nlo;
}

// spooky.c:55-68
__device__ __forceinline__ void short_mix(uint64_t &h0, uint64_t &h1, uint64_t &h2, uint64_t &h3) {
    h2 = rotl64(h2, 50); h2 += h3; h0 ^= h2;
    h3 = rotl64(h3, 52); h3 += h0; h1 ^= h3;
    h0 = rotl64(h0, 30); h0 += h1; h2 ^= h0;
    h1 = rotl64(h1, 41); h1 += h2; h3 ^= h1;
    h2 = rotl64(h2, 54); h2 += h3; h0 ^= h2;
    h3 = rotl64(h3, 48); h3 += h0; h1 ^= h3;
    h0 = rotl64(h0, 38); h0 += h1; h2 ^= h0;
    h1 = rotl64(h1, 37); h1 += h2; h3 ^= h1;
    h2 = rotl64(h2, 62); h2 += h3; h0 ^= h2;
    h3 = rotl64(h3, 34); h3 += h0; h1 ^= h3;
    h0 = rotl64(h0, 5);  h0 += h1; h2 ^= h0;
    h1 = rotl64(h1, 36); h1 += h2; h3 ^= h1;
}

// spooky.c:72-84
__device__ __forceinline__ void short_end(uint64_t &h0, uint64_t &h1, uint64_t &h2, uint64_t &h3) {
    h3 ^= h2; h2 = rotl64(h2, 15); h3 += h2;
    h0 ^= h3; h3 = rotl64(h3, 52); h0 += h3;
    h1 ^= h0; h0 = rotl64(h0, 26); h1 += h0;
    h2 ^= h1; h1 = rotl64(h1, 51); h2 += h1;
    h3 ^= h2; h2 = rotl64(h2, 28); h3 += h2;
    h0 ^= h3; h3 = rotl64(h3, 9);  h0 += h3;
    h1 ^= h0; h0 = rotl64(h0, 47); h1 += h0;
    h2 ^= h1; h1 = rotl64(h1, 54); h2 += h1;
    h3 ^= h2; h2 = rotl64(h2, 32); h3 += h2;
    h0 ^= h3; h3 = rotl64(h3, 25); h0 += h3;
    h1 ^= h0; h0 = rotl64(h0, 63); h1 += h0;
}

// Keys of 8..15 bytes have no ShortMix: h2 = SC + bytes[0..8), h3 = SC + bytes[8..len)
// (spooky.c:132-149), h0 = seed + 8*len (spooky.c:170).
__device__ __forceinline__ void spooky_8_15(uint64_t w0, uint64_t w1, uint32_t len, uint64_t seed,
                                            uint64_t &sig0, uint64_t &sig1) {
    uint64_t h0 = seed + (uint64_t)len * 8, h1 = seed, h2 = SC + w0, h3 = SC + w1;
    short_end(h0, h1, h2, h3);
    sig0 = h0;
    sig1 = h1;
}

__device__ __forceinline__ uint64_t low_bytes_mask(uint32_t k) {  // k in 0..8
    return k >= 8 ? ~0ULL : ((1ULL << (8 * k)) - 1);
}

// Generic SpookyHash-short over a key read through `rd(off)`, which returns the
// little-endian u64 at byte offset `off` of the key (bytes past the key end may
// be garbage: they are masked here).  spooky.c:94-175.
template <class Reader>
__device__ __forceinline__ void spooky_short(const Reader &rd, uint32_t len, uint64_t seed,
                                             uint64_t &sig0, uint64_t &sig1) {
    uint64_t h0 = seed, h1 = seed, h2 = SC, h3 = SC;
    uint32_t rem = len & 31, off = 0;
    if (len > 15) {
        const uint32_t nblk = len >> 5;
        for (uint32_t b = 0; b < nblk; ++b, off += 32) {
            h2 += rd(off);
            h3 += rd(off + 8);
            short_mix(h0, h1, h2, h3);
            h0 += rd(off + 16);
            h1 += rd(off + 24);
        }
        if (rem >= 16) {
            h2 += rd(off);
            h3 += rd(off + 8);
            short_mix(h0, h1, h2, h3);
            off += 16;
            rem -= 16;
        }
    }
    if (rem == 0) {
        h2 += SC;
        h3 += SC;
    } else if (rem >= 8) {
        h2 += rd(off);
        h3 += rd(off + 8) & low_bytes_mask(rem - 8);
    } else {
        h2 += rd(off) & low_bytes_mask(rem);
    }
    h0 += (uint64_t)len * 8;
    short_end(h0, h1, h2, h3);
    sig0 = h0;
    sig1 = h1;
}

// GOV:559 / CBHS:965 -- Math.multiplyHigh(sig0 >>> 1, 2m); sig0>>>1 < 2^63 so the
// signed and unsigned high products agree.
__device__ __forceinline__ uint32_t bucket_of(uint64_t sig0, uint64_t multiplier) {
    return (uint32_t)__umul64hi(sig0 >> 1, multiplier);
}

// GOV:315-317 (C_TIMES_256 = 281)
__device__ __forceinline__ uint64_t vertex_offset(uint64_t eos) { return ((eos & OFFSET_MASK) * 281) >> 8; }

// Funnel read of 8 bytes at byte offset `o` of a dword-addressed buffer.
__device__ __forceinline__ uint64_t funnel64(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t sh) {
    const uint32_t lo = __builtin_amdgcn_alignbit(d1, d0, sh);
    const uint32_t hi = __builtin_amdgcn_alignbit(d2, d1, sh);
    return ((uint64_t)hi << 32) | lo;
}

// ---- 32-bit-half formulation --------------------------------------------
// The same arithmetic with every 64-bit word held as two VGPRs: xor = 2
// v_xor_b32, rotate = 2 v_alignbit_b32, add = v_add_co_u32 + v_addc_co_u32.
// Unlike v_lshl_add_u64 this needs no even-aligned register pairs, so the
// allocator inserts no v_mov_b32 shuffles (measured: ~34 moves/key saved).
struct W64 {
    uint32_t lo, hi;
};

__device__ __forceinline__ W64 w64(uint64_t x) { return W64{(uint32_t)x, (uint32_t)(x >> 32)}; }
__device__ __forceinline__ uint64_t u64(W64 x) { return ((uint64_t)x.hi << 32) | x.lo; }

__device__ __forceinline__ W64 add(W64 a, W64 b) {
    unsigned int c;
    W64 r;
    r.lo = __builtin_addc(a.lo, b.lo, 0u, &c);
    r.hi = __builtin_addc(a.hi, b.hi, c, &c);
    return r;
}
__device__ __forceinline__ W64 xor_(W64 a, W64 b) { return W64{a.lo ^ b.lo, a.hi ^ b.hi}; }
template <int K>
__device__ __forceinline__ W64 rotl(W64 x) {
    if (K < 32) return W64{__builtin_amdgcn_alignbit(x.lo, x.hi, 32 - K), __builtin_amdgcn_alignbit(x.hi, x.lo, 32 - K)};
    if (K == 32) return W64{x.hi, x.lo};
    return W64{__builtin_amdgcn_alignbit(x.hi, x.lo, 64 - K), __builtin_amdgcn_alignbit(x.lo, x.hi, 64 - K)};
}

#define BSDB_END_STEP(D, C, K) D = xor_(D, C); C = rotl<K>(C); D = add(D, C);
// spooky.c:72-84 on W64 halves.
__device__ __forceinline__ void short_end_w(W64 &h0, W64 &h1, W64 &h2, W64 &h3) {
    BSDB_END_STEP(h3, h2, 15) BSDB_END_STEP(h0, h3, 52) BSDB_END_STEP(h1, h0, 26)
    BSDB_END_STEP(h2, h1, 51) BSDB_END_STEP(h3, h2, 28) BSDB_END_STEP(h0, h3, 9)
    BSDB_END_STEP(h1, h0, 47) BSDB_END_STEP(h2, h1, 54) BSDB_END_STEP(h3, h2, 32)
    BSDB_END_STEP(h0, h3, 25) BSDB_END_STEP(h1, h0, 63)
}
#undef BSDB_END_STEP

// ---- 64-bit-pair formulation -------------------------------------------
// Same arithmetic with the adds as one v_lshl_add_u64 (measured on gfx950:
// one issue slot, the same rate as a 32-bit op, where v_add_co + v_addc take
// two); xors and rotates stay on the 32-bit halves.
__device__ __forceinline__ uint64_t add_u(uint64_t a, uint64_t b) {
    uint64_t r;
    asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
template <int K>
__device__ __forceinline__ uint64_t rotl_u(uint64_t x) {
    const W64 r = rotl<K>(W64{(uint32_t)x, (uint32_t)(x >> 32)});
    return ((uint64_t)r.hi << 32) | r.lo;
}
#define BSDB_END_STEP_U(D, C, K) D ^= C; C = rotl_u<K>(C); D = add_u(D, C);
// D += C rotated by 32 with the halves crossed in the carry chain (2 VALU)
// instead of swapping C into a register pair first (2 moves + the add)
__device__ __forceinline__ uint64_t add_swapped(uint64_t d, uint64_t c) {
    unsigned int cy;
    const uint32_t lo = __builtin_addc((uint32_t)d, (uint32_t)(c >> 32), 0u, &cy);
    const uint32_t hi = __builtin_addc((uint32_t)(d >> 32), (uint32_t)c, cy, &cy);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ void short_end_u(uint64_t &h0, uint64_t &h1, uint64_t &h2, uint64_t &h3) {
    BSDB_END_STEP_U(h3, h2, 15) BSDB_END_STEP_U(h0, h3, 52) BSDB_END_STEP_U(h1, h0, 26)
    BSDB_END_STEP_U(h2, h1, 51) BSDB_END_STEP_U(h3, h2, 28) BSDB_END_STEP_U(h0, h3, 9)
    BSDB_END_STEP_U(h1, h0, 47) BSDB_END_STEP_U(h2, h1, 54)
    h3 ^= h2;  // step 9, K = 32
    h3 = add_swapped(h3, h2);
    h2 = rotl_u<32>(h2);
    BSDB_END_STEP_U(h0, h3, 25) BSDB_END_STEP_U(h1, h0, 63)
}
#undef BSDB_END_STEP_U

// spooky.c:55-68 with the adds as v_lshl_add_u64.
#define BSDB_MIX_STEP_U(A, K, B, C) A = rotl_u<K>(A); A = add_u(A, B); C ^= A;
__device__ __forceinline__ void short_mix_u(uint64_t &h0, uint64_t &h1, uint64_t &h2, uint64_t &h3) {
    BSDB_MIX_STEP_U(h2, 50, h3, h0) BSDB_MIX_STEP_U(h3, 52, h0, h1) BSDB_MIX_STEP_U(h0, 30, h1, h2)
    BSDB_MIX_STEP_U(h1, 41, h2, h3) BSDB_MIX_STEP_U(h2, 54, h3, h0) BSDB_MIX_STEP_U(h3, 48, h0, h1)
    BSDB_MIX_STEP_U(h0, 38, h1, h2) BSDB_MIX_STEP_U(h1, 37, h2, h3) BSDB_MIX_STEP_U(h2, 62, h3, h0)
    BSDB_MIX_STEP_U(h3, 34, h0, h1) BSDB_MIX_STEP_U(h0, 5, h1, h2)  BSDB_MIX_STEP_U(h1, 36, h2, h3)
}
#undef BSDB_MIX_STEP_U

// spooky_short (spooky.c:94-175) in the v_lshl_add_u64 formulation, sig0 only
// (the bucket needs nothing else).
template <class Reader>
__device__ __forceinline__ uint64_t spooky_short_sig0_u(const Reader &rd, uint32_t len, uint64_t seed) {
    uint64_t h0 = seed, h1 = seed, h2 = SC, h3 = SC;
    uint32_t rem = len & 31, off = 0;
    if (len > 15) {
        const uint32_t nblk = len >> 5;
        for (uint32_t b = 0; b < nblk; ++b, off += 32) {
            h2 = add_u(h2, rd(off));
            h3 = add_u(h3, rd(off + 8));
            short_mix_u(h0, h1, h2, h3);
            h0 = add_u(h0, rd(off + 16));
            h1 = add_u(h1, rd(off + 24));
        }
        if (rem >= 16) {
            h2 = add_u(h2, rd(off));
            h3 = add_u(h3, rd(off + 8));
            short_mix_u(h0, h1, h2, h3);
            off += 16;
            rem -= 16;
        }
    }
    if (rem == 0) {
        h2 = add_u(h2, SC);
        h3 = add_u(h3, SC);
    } else if (rem >= 8) {
        h2 = add_u(h2, rd(off));
        h3 = add_u(h3, rd(off + 8) & low_bytes_mask(rem - 8));
    } else {
        h2 = add_u(h2, rd(off) & low_bytes_mask(rem));
    }
    h0 = add_u(h0, (uint64_t)len * 8);
    short_end_u(h0, h1, h2, h3);
    return h0;
}

// spooky_short (spooky.c:94-175) of a key of len <= 64 bytes held in
// registers: d[0..16] are the dwords from the key's first byte rounded down
// to 4, sh = 8 * (that byte's offset in d[0]).  With c_k = bytes [16k, 16k+16):
//   len >= 16: h2 += c0, mix          len >= 32: h0,h1 += c1 (block 0 done)
//   len >= 48: h2 += c2, mix          len == 64: h0,h1 += c3 (block 1 done)
// then the tail is c_{len/16} masked to len % 16 bytes (SC twice when empty).
__device__ __forceinline__ uint64_t spooky_le64_sig0(const uint32_t (&d)[17], uint32_t sh, uint32_t len,
                                                     uint64_t seed) {
    auto W = [&](int k) -> uint64_t { return funnel64(d[2 * k], d[2 * k + 1], d[2 * k + 2], sh); };
    uint64_t h0 = seed, h1 = seed, h2 = SC, h3 = SC;
    if (len >= 16) {
        h2 = add_u(h2, W(0));
        h3 = add_u(h3, W(1));
        short_mix_u(h0, h1, h2, h3);
        if (len >= 32) {
            h0 = add_u(h0, W(2));
            h1 = add_u(h1, W(3));
        }
        if (len >= 48) {
            h2 = add_u(h2, W(4));
            h3 = add_u(h3, W(5));
            short_mix_u(h0, h1, h2, h3);
            if (len >= 64) {
                h0 = add_u(h0, W(6));
                h1 = add_u(h1, W(7));
            }
        }
    }
    const uint32_t ci = len >> 4, r = len & 15;  // tail chunk (ci = 4: len 64, r = 0)
    const uint64_t t0 = ci == 0 ? W(0) : ci == 1 ? W(2) : ci == 2 ? W(4) : W(6);
    const uint64_t t1 = ci == 0 ? W(1) : ci == 1 ? W(3) : ci == 2 ? W(5) : W(7);
    uint64_t x0, x1;
    if (r == 0) {
        x0 = SC;
        x1 = SC;
    } else if (r >= 8) {
        x0 = t0;
        x1 = t1 & low_bytes_mask(r - 8);
    } else {
        x0 = t0 & low_bytes_mask(r);
        x1 = 0;
    }
    h2 = add_u(h2, x0);
    h3 = add_u(h3, x1);
    h0 = add_u(h0, (uint64_t)len * 8);
    short_end_u(h0, h1, h2, h3);
    return h0;
}

// The same for a key of len < 16 bytes: d[0..4] only, no ShortMix.
__device__ __forceinline__ uint64_t spooky_lt16_sig0(const uint32_t (&d)[5], uint32_t sh, uint32_t len,
                                                     uint64_t seed) {
    const uint64_t t0 = funnel64(d[0], d[1], d[2], sh), t1 = funnel64(d[2], d[3], d[4], sh);
    uint64_t x0, x1;
    if (len == 0) {
        x0 = SC;
        x1 = SC;
    } else if (len >= 8) {
        x0 = t0;
        x1 = t1 & low_bytes_mask(len - 8);
    } else {
        x0 = t0 & low_bytes_mask(len);
        x1 = 0;
    }
    uint64_t h0 = add_u(seed, (uint64_t)len * 8), h1 = seed, h2 = add_u(SC, x0), h3 = add_u(SC, x1);
    short_end_u(h0, h1, h2, h3);
    return h0;
}

__device__ __forceinline__ void spooky13_u(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3, uint32_t sh,
                                           uint64_t seed, W64 &sig0, W64 &sig1) {
    const uint64_t w0 = ((uint64_t)__builtin_amdgcn_alignbit(d2, d1, sh) << 32) | __builtin_amdgcn_alignbit(d1, d0, sh);
    const uint64_t w1 = ((uint64_t)((d3 >> sh) & 0xFFu) << 32) | __builtin_amdgcn_alignbit(d3, d2, sh);
    uint64_t h0 = seed + 13 * 8, h1 = seed, h2 = add_u(SC, w0), h3 = add_u(SC, w1);
    short_end_u(h0, h1, h2, h3);
    sig0 = w64(h0);
    sig1 = w64(h1);
}

// 13-byte key given as its first 16 little-endian bytes d0..d3 shifted by sh
// bits (the key starts at byte sh/8 of d0): spooky.c tail case 13 + ShortEnd.
__device__ __forceinline__ void spooky13_w(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3, uint32_t sh,
                                           W64 seed, W64 &sig0, W64 &sig1) {
    const W64 w0{__builtin_amdgcn_alignbit(d1, d0, sh), __builtin_amdgcn_alignbit(d2, d1, sh)};
    const W64 w1{__builtin_amdgcn_alignbit(d3, d2, sh), (d3 >> sh) & 0xFFu};
    const W64 sc = w64(SC);
    W64 h0 = add(seed, W64{13 * 8, 0}), h1 = seed, h2 = add(sc, w0), h3 = add(sc, w1);
    short_end_w(h0, h1, h2, h3);
    sig0 = h0;
    sig1 = h1;
}

// GOV:559 bucket with the multiplier 2m < 2^32 (GOV:349 caps m at
// Integer.MAX_VALUE): hi64((sig0>>>1) * M) = (xh*M + hi32(xl*M)) >> 32.
__device__ __forceinline__ uint32_t bucket_of_w(W64 sig0, uint32_t mult) {
    const uint32_t xl = __builtin_amdgcn_alignbit(sig0.hi, sig0.lo, 1);
    const uint32_t xh = sig0.hi >> 1;
    const uint64_t t = (uint64_t)xh * mult + __umulhi(xl, mult);
    return (uint32_t)(t >> 32);
}

__device__ __forceinline__ uint32_t short_end_bucket(uint64_t h0, uint64_t h1, uint64_t h2, uint64_t h3, uint32_t mult);

// The bucket of a 13-byte key straight from the hash (the histogram needs
// nothing else): spooky.c's tail case 13, then short_end_bucket.

__device__ __forceinline__ uint32_t spooky13_bucket(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3, uint32_t sh,
                                                    uint64_t seed, uint32_t mult) {
    const uint64_t w0 = ((uint64_t)__builtin_amdgcn_alignbit(d2, d1, sh) << 32) | __builtin_amdgcn_alignbit(d1, d0, sh);
    const uint64_t w1 = ((uint64_t)((d3 >> sh) & 0xFFu) << 32) | __builtin_amdgcn_alignbit(d3, d2, sh);
    return short_end_bucket(seed + 13 * 8, seed, add_u(SC, w0), add_u(SC, w1), mult);
}

// The bucket of a fixed-length key of L in {8, 12, 16} bytes given as the
// 16 little-endian bytes d0..d3 from its (4-byte aligned) first byte:
// spooky.c's tail cases 8 and 12 (h3 += the masked second word, 0 or the
// 4 bytes 8..11) and, for 16, the one 16-byte ShortMix step with the empty
// tail (h2, h3 += SC) -- spooky.c:97-170.
template <int L>
__device__ __forceinline__ uint32_t spooky_fix_bucket(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3, uint64_t seed,
                                                      uint32_t mult) {
    static_assert(L == 8 || L == 12 || L == 16, "aligned fixed lengths");
    const uint64_t w0 = ((uint64_t)d1 << 32) | d0;
    if (L == 16) {
        uint64_t h0 = seed, h1 = seed, h2 = add_u(SC, w0), h3 = add_u(SC, ((uint64_t)d3 << 32) | d2);
        short_mix_u(h0, h1, h2, h3);
        return short_end_bucket(add_u(h0, 16 * 8), h1, add_u(h2, SC), add_u(h3, SC), mult);
    }
    return short_end_bucket(seed + L * 8, seed, add_u(SC, w0), L == 12 ? add_u(SC, (uint64_t)d2) : SC, mult);
}

// ShortEnd (spooky.c:72-84) up to h0's last rotation, then the bucket
// (GOV:559) from the unrotated word h (sig0 = rotl(h, 63) = h >>> 1 | h << 63,
// so x = sig0 >>> 1 = h >>> 2 | (h & 1) << 62): 3 VALU instead of the
// rotation's 2 plus 2.
__device__ __forceinline__ uint32_t short_end_bucket(uint64_t h0, uint64_t h1, uint64_t h2, uint64_t h3, uint32_t mult) {
#define BSDB_END_STEP_U(D, C, K) D ^= C; C = rotl_u<K>(C); D = add_u(D, C);
    BSDB_END_STEP_U(h3, h2, 15) BSDB_END_STEP_U(h0, h3, 52) BSDB_END_STEP_U(h1, h0, 26)
    BSDB_END_STEP_U(h2, h1, 51) BSDB_END_STEP_U(h3, h2, 28) BSDB_END_STEP_U(h0, h3, 9)
    BSDB_END_STEP_U(h1, h0, 47) BSDB_END_STEP_U(h2, h1, 54)
    h3 ^= h2;
    h3 = add_swapped(h3, h2);
    BSDB_END_STEP_U(h0, h3, 25)
#undef BSDB_END_STEP_U
    const uint32_t hl = (uint32_t)h0, hh = (uint32_t)(h0 >> 32);
    const uint32_t xl = __builtin_amdgcn_alignbit(hh, hl, 2);
    const uint32_t xh = __builtin_amdgcn_alignbit(hl, hh, 2) & 0x7FFFFFFFu;
    const uint64_t t = (uint64_t)xh * mult + __umulhi(xl, mult);  // GOV:559, as bucket_of_w
    return (uint32_t)(t >> 32);
}

// short_end_bucket that also returns the top 8 bits of x = sig0 >>> 1 (the
// fused histogram's bucket owner, k_hist13_fused): buckets are monotone in x,
// so owner w's buckets are [floor(w m / 256), floor((w + 1) m / 256)].
__device__ __forceinline__ uint32_t short_end_bucket_owner(uint64_t h0, uint64_t h1, uint64_t h2, uint64_t h3,
                                                           uint32_t mult, uint32_t &owner) {
#define BSDB_END_STEP_U(D, C, K) D ^= C; C = rotl_u<K>(C); D = add_u(D, C);
    BSDB_END_STEP_U(h3, h2, 15) BSDB_END_STEP_U(h0, h3, 52) BSDB_END_STEP_U(h1, h0, 26)
    BSDB_END_STEP_U(h2, h1, 51) BSDB_END_STEP_U(h3, h2, 28) BSDB_END_STEP_U(h0, h3, 9)
    BSDB_END_STEP_U(h1, h0, 47) BSDB_END_STEP_U(h2, h1, 54)
    h3 ^= h2;
    h3 = add_swapped(h3, h2);
    BSDB_END_STEP_U(h0, h3, 25)
#undef BSDB_END_STEP_U
    const uint32_t hl = (uint32_t)h0, hh = (uint32_t)(h0 >> 32);
    const uint32_t xl = __builtin_amdgcn_alignbit(hh, hl, 2);
    const uint32_t xh = __builtin_amdgcn_alignbit(hl, hh, 2) & 0x7FFFFFFFu;
    owner = xh >> 23;
    const uint64_t t = (uint64_t)xh * mult + __umulhi(xl, mult);  // GOV:559, as bucket_of_w
    return (uint32_t)(t >> 32);
}

__device__ __forceinline__ uint32_t spooky13_bucket_owner(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3,
                                                          uint32_t sh, uint64_t seed, uint32_t mult, uint32_t &owner) {
    const uint64_t w0 = ((uint64_t)__builtin_amdgcn_alignbit(d2, d1, sh) << 32) | __builtin_amdgcn_alignbit(d1, d0, sh);
    const uint64_t w1 = ((uint64_t)((d3 >> sh) & 0xFFu) << 32) | __builtin_amdgcn_alignbit(d3, d2, sh);
    return short_end_bucket_owner(seed + 13 * 8, seed, add_u(SC, w0), add_u(SC, w1), mult, owner);
}

// SURVEY.md §8(d) D2 synthetic keys (bench input generator only).
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9e3779b97f4a7c15ULL;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

}  // namespace bsdb
