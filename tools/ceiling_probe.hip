// Ceiling probe for the headline (measurement tool, not product code): what
// any histogram design for BASELINE C4 must at least spend on this chip.
// At the C4 size (13 193 787 549 x 13 B = 171.5 GB resident):
//   k16     every key byte read once, perfectly coalesced 16-B nontemporal
//           loads, no compute: the HBM read ceiling of the key stream
//   k13     the same bytes as each key's dword-aligned 16-B window (the
//           production front end's load pattern)
//   hash    k13's loads + SpookyHash-short (spooky.c tail case 13 + ShortEnd,
//           seed 0) + the bucket multiplyHigh: the hash stage alone, with no
//           histogram at all (a xor of the buckets keeps it live)
//   lds     hash + ONE LDS atomic increment per key into a per-workgroup
//           8192-counter table (bucket mod 8192): the cheapest on-chip count
//           any histogram design needs, with no id exchange at all (a
//           lower bound: the real 35 MB table fits no LDS)
//   ldscf   the same count with a bank-conflict-free address (row = bucket
//           bits, column = the lane: every lane of a wave on its own bank)
//   ldsrtn  the random count with the returned old value used (ds_add_rtn,
//           the pass-1 kernel's rank atomic)
// Each kernel is timed with HIP events (best of 3).  The keys are random
// bytes (a splitmix64 fill): the hash's cost does not depend on the values,
// but the LDS atomics' does -- with a constant fill (round 3's first runs)
// every key has one of four buckets, so a wave's 64 atomics hit ~4 words and
// serialise; those 'lds' rows measured same-word contention, not random
// banks.
//   ldsu16  hash + one u16-packed LDS count per key into a 34 360-bucket
//           table (68.7 KB, ds_add_u32 of 1 or 1<<16): the consumer side of
//           the fused single-pass design
//   hipcc --offload-arch=gfx950 -O3 -I bsdb_amd/csrc tools/ceiling_probe.hip -o tools/ceiling_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "spooky_dev.hpp"

using namespace bsdb;
typedef unsigned int u32x4a __attribute__((ext_vector_type(4), aligned(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int NT = 512, KPT = 16;

__global__ __launch_bounds__(NT) void k16(const uint8_t *p, uint64_t nvec, uint32_t *out) {
    uint32_t x = 0;
    const uint64_t stride = (uint64_t)gridDim.x * NT * KPT;
    for (uint64_t base = (uint64_t)blockIdx.x * NT * KPT; base < nvec; base += stride) {
        u32x4 w[KPT];
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint64_t v = base + threadIdx.x + (uint64_t)j * NT;
            w[j] = v < nvec ? __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p) + v) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int j = 0; j < KPT; ++j) x ^= w[j].x ^ w[j].y ^ w[j].z ^ w[j].w;
    }
    if (x == 0x12345678u) out[threadIdx.x] = x;
}

constexpr int LDS_BINS = 8192;

constexpr int U16_BUCKETS = 34360, U16_WORDS = U16_BUCKETS / 2;

__global__ void k_fill(uint64_t *p, uint64_t nwords) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nwords; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

// LDS: 0 none, 1 random ds_add, 2 conflict-free ds_add, 3 random ds_add_rtn,
// 4 u16-packed count into a 34 360-bucket table
template <bool HASH, int LDS = 0>
__global__ __launch_bounds__(NT) void k13(const uint8_t *p, uint64_t nkeys, uint32_t mult, uint32_t *out) {
    constexpr int TAB = LDS == 4 ? U16_WORDS : LDS ? LDS_BINS : 1;
    __shared__ uint32_t tab[TAB];
    if (LDS) {
        for (int i = threadIdx.x; i < TAB; i += NT) tab[i] = 0;
        __syncthreads();
    }
    uint32_t x = 0;
    const uint64_t stride = (uint64_t)gridDim.x * NT * KPT;
    for (uint64_t base = (uint64_t)blockIdx.x * NT * KPT; base < nkeys; base += stride) {
        u32x4a w[KPT];
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint64_t k = base + threadIdx.x + (uint64_t)j * NT;
            const uint64_t byte = (k < nkeys ? k : 0) * 13;
            w[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4a *>(p + (byte & ~3ULL)));
        }
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint64_t k = base + threadIdx.x + (uint64_t)j * NT;
            if (HASH) {
                const uint32_t sh = (uint32_t)((k * 13) & 3) * 8;
                W64 s0, s1;
                spooky13_u(w[j].x, w[j].y, w[j].z, w[j].w, sh, 0, s0, s1);
                const uint32_t b = bucket_of_w(s0, mult);
                if (LDS == 1) {
                    if (k < nkeys) atomicAdd(&tab[b & (LDS_BINS - 1)], 1u);
                } else if (LDS == 2) {
                    if (k < nkeys) atomicAdd(&tab[((b >> 6) & (LDS_BINS / 64 - 1)) * 64 + (threadIdx.x & 63)], 1u);
                } else if (LDS == 3) {
                    if (k < nkeys) x += atomicAdd(&tab[b & (LDS_BINS - 1)], 1u);
                } else if (LDS == 4) {
                    const uint32_t o = __umulhi(b, 0x80000000u / U16_BUCKETS * 2) ;  // (b mod-ish table slot)
                    const uint32_t t = b - o * U16_BUCKETS;
                    if (k < nkeys) atomicAdd(&tab[(t >> 1) % U16_WORDS], 1u << ((t & 1) << 4));
                } else {
                    x ^= b;
                }
            } else {
                x ^= w[j].x ^ w[j].y ^ w[j].z ^ w[j].w;
            }
        }
    }
    if (LDS) {
        __syncthreads();
        for (int i = threadIdx.x; i < TAB; i += NT) x ^= tab[i] * (uint32_t)(i + 1);
    }
    if (x == 0x12345678u) out[threadIdx.x] = x;
}

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 13193787549ULL;
    const uint64_t bytes = n * 13, m = n / 1500 + 1;
    uint8_t *p = nullptr;
    uint32_t *o = nullptr;
    if (hipMalloc(&p, bytes + 64) != hipSuccess || hipMalloc(&o, 4096) != hipSuccess) {
        fprintf(stderr, "allocation of %.1f GB failed\n", bytes / 1e9);
        return 1;
    }
    (void)hipMemset(p, 0x5b, bytes + 64);
    k_fill<<<4096, 256>>>(reinterpret_cast<uint64_t *>(p), bytes / 8);
    (void)hipDeviceSynchronize();
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    printf("{\"n_keys\": %llu, \"key_bytes\": %.1f, \"cus\": %d", (unsigned long long)n, bytes / 1e9, cus);
    const int kind0 = argc > 2 ? atoi(argv[2]) : 0;
    for (int kind = kind0; kind < 7; ++kind) {
        for (int per_cu : {2, 4}) {
            const int grid = cus * per_cu;
            float best = 1e30f;
            for (int rep = 0; rep < 4; ++rep) {
                (void)hipEventRecord(a);
                if (kind == 0) k16<<<grid, NT>>>(p, bytes / 16, o);
                else if (kind == 1) k13<false><<<grid, NT>>>(p, n, (uint32_t)(2 * m), o);
                else if (kind == 2) k13<true><<<grid, NT>>>(p, n, (uint32_t)(2 * m), o);
                else if (kind == 3) k13<true, 1><<<grid, NT>>>(p, n, (uint32_t)(2 * m), o);
                else if (kind == 4) k13<true, 2><<<grid, NT>>>(p, n, (uint32_t)(2 * m), o);
                else if (kind == 5) k13<true, 3><<<grid, NT>>>(p, n, (uint32_t)(2 * m), o);
                else k13<true, 4><<<grid, NT>>>(p, n, (uint32_t)(2 * m), o);
                (void)hipEventRecord(b);
                (void)hipEventSynchronize(b);
                float ms = 0;
                (void)hipEventElapsedTime(&ms, a, b);
                if (rep && ms < best) best = ms;
            }
            const char *name = kind == 0 ? "k16" : kind == 1 ? "k13" : kind == 2 ? "hash" : kind == 3 ? "lds" : kind == 4 ? "ldscf" : kind == 5 ? "ldsrtn" : "ldsu16";
            printf(", \"%s_wg%d\": {\"ms\": %.3f, \"TBps\": %.3f, \"Gkeys_per_s\": %.1f, \"roofline_frac\": %.3f}", name,
                   per_cu, best, bytes / best / 1e9, n / best / 1e6, bytes / best / 1e9 / 8.0);
            fflush(stdout);
        }
    }
    printf("}\n");
    return hipGetLastError() == hipSuccess ? 0 : 2;
}
