// VALU issue-rate probe for the instructions the 13-byte hash is built from.
// hipcc --offload-arch=gfx950 -O3 tools/alu_probe.hip -o tools/alu_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../bsdb_amd/csrc/spooky_dev.hpp"

constexpr int ITER = 4096;
constexpr int CH = 8;

__global__ void k_addc(uint32_t *out, uint32_t s) {
    uint32_t lo[CH], hi[CH];
    for (int c = 0; c < CH; c++) { lo[c] = threadIdx.x + c; hi[c] = s + c; }
    for (int i = 0; i < ITER; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++)
            asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %2, vcc" : "+v"(lo[c]), "+v"(hi[c]) : "v"(s) : "vcc");
    }
    uint32_t r = 0;
    for (int c = 0; c < CH; c++) r ^= lo[c] ^ hi[c];
    if (r == 0x12345) out[0] = r;
}

__global__ void k_lshladd(uint32_t *out, uint32_t s) {
    uint64_t a[CH];
    uint64_t b = ((uint64_t)s << 32) | s;
    for (int c = 0; c < CH; c++) a[c] = threadIdx.x + c;
    for (int i = 0; i < ITER; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a[c]) : "v"(b));
    }
    uint64_t r = 0;
    for (int c = 0; c < CH; c++) r ^= a[c];
    if (r == 0x12345) out[0] = (uint32_t)r;
}

__global__ void k_xor(uint32_t *out, uint32_t s) {
    uint32_t a[CH];
    for (int c = 0; c < CH; c++) a[c] = threadIdx.x + c;
    for (int i = 0; i < ITER; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[c]) : "v"(s));
    }
    uint32_t r = 0;
    for (int c = 0; c < CH; c++) r ^= a[c];
    if (r == 0x12345) out[0] = r;
}

__global__ void k_alignbit(uint32_t *out, uint32_t s) {
    uint32_t a[CH];
    for (int c = 0; c < CH; c++) a[c] = threadIdx.x + c;
    for (int i = 0; i < ITER; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_alignbit_b32 %0, %0, %1, 13" : "+v"(a[c]) : "v"(s));
    }
    uint32_t r = 0;
    for (int c = 0; c < CH; c++) r ^= a[c];
    if (r == 0x12345) out[0] = r;
}

__global__ void k_bitop3(uint32_t *out, uint32_t s) {
    uint32_t a[CH];
    for (int c = 0; c < CH; c++) a[c] = threadIdx.x + c;
    for (int i = 0; i < ITER; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(a[c]) : "v"(s));
    }
    uint32_t r = 0;
    for (int c = 0; c < CH; c++) r ^= a[c];
    if (r == 0x12345) out[0] = r;
}

__global__ void k_pkadd(uint32_t *out, uint32_t s) {   // packed fp32 add: dual-rate check
    float2 a[CH];
    for (int c = 0; c < CH; c++) a[c] = make_float2(threadIdx.x + c, c);
    uint64_t b = ((uint64_t)s << 32) | s;
    for (int i = 0; i < ITER; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[c]) : "v"(b));
    }
    float r = 0;
    for (int c = 0; c < CH; c++) r += a[c].x + a[c].y;
    if (r == 1.2345f) out[0] = 1;
}

// the 13-byte hash's ShortEnd on NK independent keys per lane (the
// production formulation), 55 VALU per key per round
template <int NK>
__global__ void k_spooky(uint32_t *out, uint32_t s) {
    uint64_t h[NK][4];
    for (int c = 0; c < NK; c++) for (int q = 0; q < 4; q++) h[c][q] = threadIdx.x * 77 + c * 5 + q + s;
    for (int i = 0; i < ITER / 8; i++) {
#pragma unroll
        for (int c = 0; c < NK; c++) bsdb::short_end_u(h[c][0], h[c][1], h[c][2], h[c][3]);
    }
    uint64_t r = 0;
    for (int c = 0; c < NK; c++) r ^= h[c][0] ^ h[c][1];
    if (r == 0x12345) out[0] = (uint32_t)r;
}

template <typename K>
void run(const char *name, K k, int ops_per, uint32_t *d, int wpc = 32, double iters = ITER * CH) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    int dev;
    hipGetDevice(&dev);
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, dev);
    const int blocks = p.multiProcessorCount * (wpc / 4);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 7u);
    hipEventRecord(a);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 7u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double instr = 5.0 * blocks * 256.0 * iters * ops_per;
    printf("%-12s %8.3f ms  %7.2f T lane-instr/s  (%.1f instr/clk/CU at %d MHz)\n", name, ms / 5, instr / (ms * 1e-3) / 1e12,
           instr / (ms * 1e-3) / (p.multiProcessorCount * (double)p.clockRate * 1e3), p.clockRate / 1000);
}

int main() {
    uint32_t *d;
    hipMalloc(&d, 64);
    run("addc(2)", k_addc, 2, d);
    for (int wpc : {8, 16, 32}) {
        char nm[64];
        snprintf(nm, sizeof nm, "spooky1 w%d", wpc);
        run(nm, k_spooky<1>, 55, d, wpc, ITER / 8 * 1.0);
        snprintf(nm, sizeof nm, "spooky2 w%d", wpc);
        run(nm, k_spooky<2>, 55, d, wpc, ITER / 8 * 2.0);
        snprintf(nm, sizeof nm, "spooky4 w%d", wpc);
        run(nm, k_spooky<4>, 55, d, wpc, ITER / 8 * 4.0);
    }
    run("lshl_add64", k_lshladd, 1, d);
    run("xor", k_xor, 1, d);
    run("alignbit", k_alignbit, 1, d);
    run("bitop3", k_bitop3, 1, d);
    run("pk_add_f32", k_pkadd, 1, d);
    return 0;
}
