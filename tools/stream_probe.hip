// Standalone HBM read probe for the 13-byte-key access pattern (not product code).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef unsigned int u32x4a __attribute__((ext_vector_type(4), aligned(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// lane reads the dword-aligned 16-byte window of key k (13-byte stride), 16 keys/thread
__global__ __launch_bounds__(512) void k13(const uint8_t *p, uint64_t nkeys, uint32_t *out, int nt) {
    uint32_t x = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 512 * 16;
    for (uint64_t base = (uint64_t)blockIdx.x * 512 * 16; base + 512 * 16 <= nkeys; base += stride) {
        u32x4a w[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint64_t byte = (base + threadIdx.x + j * 512) * 13;
            const u32x4a *q = reinterpret_cast<const u32x4a *>(p + (byte & ~3ULL));
            w[j] = nt ? __builtin_nontemporal_load(q) : *q;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) x ^= w[j].x ^ w[j].y ^ w[j].z ^ w[j].w;
    }
    if (x == 0x12345678) out[threadIdx.x] = x;
}

// lane reads 16 contiguous bytes (perfect coalescing), same total bytes
__global__ __launch_bounds__(512) void k16(const uint8_t *p, uint64_t nbytes, uint32_t *out, int nt) {
    uint32_t x = 0;
    const uint64_t nvec = nbytes / 16;
    const uint64_t stride = (uint64_t)gridDim.x * 512 * 16;
    for (uint64_t base = (uint64_t)blockIdx.x * 512 * 16; base + 512 * 16 <= nvec; base += stride) {
        u32x4 w[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const u32x4 *q = reinterpret_cast<const u32x4 *>(p) + base + threadIdx.x + j * 512;
            w[j] = nt ? __builtin_nontemporal_load(q) : *q;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) x ^= w[j].x ^ w[j].y ^ w[j].z ^ w[j].w;
    }
    if (x == 0x12345678) out[threadIdx.x] = x;
}

int main() {
    const uint64_t nkeys = 2147483648ULL, nbytes = nkeys * 13 + 64;
    uint8_t *p; uint32_t *o;
    hipMalloc(&p, nbytes); hipMalloc(&o, 4096);
    hipMemset(p, 1, nbytes);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (int grid : {512, 1024, 2048, 4096}) for (int nt = 0; nt < 2; ++nt) {
        for (int kind = 0; kind < 2; ++kind) {
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(a);
                if (kind == 0) k13<<<grid, 512>>>(p, nkeys, o, nt); else k16<<<grid, 512>>>(p, nkeys * 13, o, nt);
                hipEventRecord(b); hipEventSynchronize(b);
                float ms; hipEventElapsedTime(&ms, a, b);
                if (rep) printf("%s grid=%d nt=%d: %.3f ms  %.2f TB/s\n", kind ? "k16" : "k13", grid, nt, ms, nkeys * 13 / ms / 1e9);
            }
        }
    }
    return 0;
}
