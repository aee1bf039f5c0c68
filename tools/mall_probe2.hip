// Standalone probe (not product code): does the Infinity Cache (MALL) absorb
// writes to a small ring that is rewritten continuously, and serve a re-read
// of just-written data, when a 13-byte-key stream runs beside it?  Decides
// whether the partition-id exchange of the two-pass histogram can stay on-die.
//   hipcc --offload-arch=gfx950 -O3 -o tools/mall_probe2 tools/mall_probe2.hip
// Each workgroup writes its share of TOTAL bytes as 16-B stores into a ring
// of R bytes (wrapping); optional concurrent stream of S bytes of nt loads.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int SC1>
__global__ __launch_bounds__(1024) void k_ring_write(u32x4 *ring, uint64_t ring_vec, uint64_t total_vec,
                                                     const u32x4 *stream, uint64_t stream_vec, uint32_t *out) {
    const uint64_t G = (uint64_t)gridDim.x * 1024, t = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    uint32_t x = 0;
    uint64_t s = t;
    for (uint64_t i = t; i < total_vec; i += G) {
        const u32x4 v = {(uint32_t)i, (uint32_t)(i >> 32), x, 7u};
        u32x4 *p = ring + (i % ring_vec);
        if (SC1) {  // write-through (agent-scope) 8-byte stores, 16 B per lane
            __hip_atomic_store(reinterpret_cast<uint64_t *>(p), (uint64_t)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(reinterpret_cast<uint64_t *>(p) + 1, (uint64_t)x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            *p = v;
        }
        if (stream_vec) {
            // ~6.5 stream vectors per ring vector: 13 B of keys per 2 B of ids
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const u32x4 w = __builtin_nontemporal_load(stream + (s % stream_vec));
                x ^= w.x ^ w.w;
                s += G;
            }
        }
    }
    if (x == 0x12345678) out[0] = x;
}

__global__ __launch_bounds__(1024) void k_ring_read(const u32x4 *ring, uint64_t ring_vec, uint64_t total_vec,
                                                    uint32_t *out) {
    const uint64_t G = (uint64_t)gridDim.x * 1024, t = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    uint32_t x = 0;
    for (uint64_t i = t; i < total_vec; i += G) {
        const u32x4 w = ring[(i + ring_vec / 2) % ring_vec];  // another workgroup's writes
        x ^= w.x ^ w.z;
    }
    if (x == 0x12345678) out[0] = x;
}

static float ms_between(hipEvent_t a, hipEvent_t b) {
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    const uint64_t big = 24ULL << 30;
    u32x4 *buf, *stream;
    uint32_t *o;
    if (hipMalloc(&buf, big) != hipSuccess || hipMalloc(&stream, 16ULL << 30) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    hipMemset(buf, 1, big);
    hipMemset(stream, 2, 16ULL << 30);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int G = 256;
    const uint64_t total = 32ULL << 30;  // bytes written per run
    for (int with_stream = 0; with_stream < 2; ++with_stream)
        for (int sc1 = 0; sc1 < 2; ++sc1)
            for (uint64_t R : {16ULL << 20, 64ULL << 20, 160ULL << 20, 512ULL << 20, 16ULL << 30}) {
                float best = 1e9;
                for (int rep = 0; rep < 3; ++rep) {
                    hipEventRecord(a);
                    if (sc1)
                        k_ring_write<1><<<G, 1024>>>(buf, R / 16, total / 16, stream, with_stream ? (16ULL << 30) / 16 : 0, o);
                    else
                        k_ring_write<0><<<G, 1024>>>(buf, R / 16, total / 16, stream, with_stream ? (16ULL << 30) / 16 : 0, o);
                    hipEventRecord(b);
                    const float ms = ms_between(a, b);
                    best = ms < best ? ms : best;
                }
                const double gb = total / 1e9, sgb = with_stream ? total * 6.0 / 1e9 : 0;
                printf("write ring %6llu MiB sc1=%d stream=%d: %8.2f ms  ring %.2f TB/s  (+stream %.2f TB/s)\n",
                       (unsigned long long)(R >> 20), sc1, with_stream, best, gb / best, sgb / best);
            }
    // re-read right after a write kernel (kernel boundary = hand-off)
    for (uint64_t R : {64ULL << 20, 160ULL << 20, 512ULL << 20, 8ULL << 30}) {
        float best = 1e9;
        for (int rep = 0; rep < 3; ++rep) {
            k_ring_write<0><<<G, 1024>>>(buf, R / 16, R / 16, stream, 0, o);
            hipEventRecord(a);
            k_ring_read<<<G, 1024>>>(buf, R / 16, R / 16, o);
            hipEventRecord(b);
            const float ms = ms_between(a, b);
            best = ms < best ? ms : best;
        }
        printf("re-read %6llu MiB just written: %8.3f ms  %.2f TB/s\n", (unsigned long long)(R >> 20), best,
               R / 1e9 / best);
    }
    return 0;
}
