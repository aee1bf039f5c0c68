// Standalone probe (not product code): does a buffer written by one kernel stay
// in the Infinity Cache (MALL) while another kernel streams key bytes with
// nontemporal / plain loads?  Decides whether the partition-id stream of the
// two-pass histogram can be kept on-die by chunking.
//   hipcc --offload-arch=gfx950 -O3 -o tools/mall_probe tools/mall_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(512) void k_write(u32x4 *p, uint64_t nvec, uint32_t v) {
    for (uint64_t i = (uint64_t)blockIdx.x * 512 + threadIdx.x; i < nvec; i += (uint64_t)gridDim.x * 512)
        p[i] = u32x4{v, v + 1, v + 2, (uint32_t)i};
}

template <int NT>
__global__ __launch_bounds__(512) void k_read(const u32x4 *p, uint64_t nvec, uint32_t *out) {
    uint32_t x = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 512 * 8;
    for (uint64_t b = (uint64_t)blockIdx.x * 512 * 8; b + 512 * 8 <= nvec; b += stride) {
        u32x4 w[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) w[j] = NT ? __builtin_nontemporal_load(p + b + threadIdx.x + j * 512) : p[b + threadIdx.x + j * 512];
#pragma unroll
        for (int j = 0; j < 8; ++j) x ^= w[j].x ^ w[j].y ^ w[j].z ^ w[j].w;
    }
    if (x == 0x12345678) out[threadIdx.x] = x;
}

static float timeit(hipEvent_t a, hipEvent_t b) {
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    const uint64_t big = 8ULL << 30;  // 8 GiB streamed buffer
    u32x4 *A, *B;
    uint32_t *o;
    hipMalloc(&A, big);
    hipMalloc(&B, 256ULL << 20);
    hipMalloc(&o, 4096);
    hipMemset(A, 1, big);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int G = 2048;
    // 1. read-only streaming bandwidth
    for (int nt = 0; nt < 2; ++nt)
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(a);
            if (nt) k_read<1><<<G, 512>>>(A, big / 16, o); else k_read<0><<<G, 512>>>(A, big / 16, o);
            hipEventRecord(b);
            float ms = timeit(a, b);
            if (rep == 2) printf("stream read 8 GiB nt=%d: %.3f ms  %.2f TB/s\n", nt, ms, big / ms / 1e9);
        }
    // 2. residency of a buffer B (S bytes) written by a kernel, after X bytes of streaming
    for (uint64_t S : {32ULL << 20, 64ULL << 20, 128ULL << 20})
        for (int nt = 0; nt < 2; ++nt)
            for (uint64_t X : {0ULL, 256ULL << 20, 1ULL << 30, 4ULL << 30}) {
                float best = 1e9;
                for (int rep = 0; rep < 3; ++rep) {
                    k_read<0><<<G, 512>>>(A + (big - (2ULL << 30)) / 16, (2ULL << 30) / 16, o);  // flush-ish
                    k_write<<<G, 512>>>(B, S / 16, rep);
                    if (X) {
                        if (nt) k_read<1><<<G, 512>>>(A, X / 16, o); else k_read<0><<<G, 512>>>(A, X / 16, o);
                    }
                    hipEventRecord(a);
                    k_read<1><<<G, 512>>>(B, S / 16, o);
                    hipEventRecord(b);
                    float ms = timeit(a, b);
                    best = ms < best ? ms : best;
                }
                printf("B=%3llu MiB after %5llu MiB stream (nt=%d): re-read %.4f ms  %.2f TB/s\n",
                       (unsigned long long)(S >> 20), (unsigned long long)(X >> 20), nt, best, S / best / 1e9);
            }
    // 3. cold reference: B after an 8 GiB plain stream
    for (uint64_t S : {32ULL << 20, 64ULL << 20, 128ULL << 20}) {
        k_read<0><<<G, 512>>>(A, big / 16, o);
        hipEventRecord(a);
        k_read<1><<<G, 512>>>(B, S / 16, o);
        hipEventRecord(b);
        float ms = timeit(a, b);
        printf("B=%3llu MiB cold: %.4f ms  %.2f TB/s\n", (unsigned long long)(S >> 20), ms, S / ms / 1e9);
    }
    return 0;
}
