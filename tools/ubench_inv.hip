// Cost of a per-lane Fq inversion in the MSM's radix-2^29 arithmetic, in units of the 29-bit
// Montgomery product (the denominator of the batch-affine estimate in DESIGN.md section 10):
// every lane inverts its own element by Fermat (a^(q-2), square-and-multiply), with 4 waves per SIMD,
// against the same kernel doing only products.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/ubench_inv.hip -o tools/ubench_inv
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../plonky3_eon_amd/csrc/field29.h"

using namespace eon;

__device__ __forceinline__ F29 inv29(const F29& a) {
    // a^(q-2), binary MSB first: 253 squarings + 128 products (q - 2 has 129 set bits); the bit is
    // the same in every lane (uniform branch)
    constexpr uint32_t E[8] = {0xd87cfd45u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                               0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
    F29 r = a;
    for (int bit = 252; bit >= 0; bit--) {
        r = sqr29<FqP>(r);
        if ((E[bit >> 5] >> (bit & 31)) & 1) r = mul29<FqP>(r, a);
    }
    return r;
}

__global__ void __launch_bounds__(256) k_inv(uint32_t* out, uint32_t reps) {
    F29 a;
    for (int i = 0; i < 9; i++) a.l[i] = (threadIdx.x * 2654435761u + i * 40503u + blockIdx.x) & M29;
    a.l[8] &= 0xfffff;
    for (uint32_t r = 0; r < reps; r++) {
        pin29(a);
        a = inv29(a);
        a.l[0] ^= 1;
    }
    uint32_t x = 0;
    for (int i = 0; i < 9; i++) x ^= a.l[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__global__ void __launch_bounds__(256) k_mul(uint32_t* out, uint32_t reps) {
    F29 a, b;
    for (int i = 0; i < 9; i++) {
        a.l[i] = (threadIdx.x * 2654435761u + i * 40503u + blockIdx.x) & M29;
        b.l[i] = (threadIdx.x * 97u + i * 7u) & M29;
    }
    a.l[8] &= 0xfffff;
    b.l[8] &= 0xfffff;
    for (uint32_t r = 0; r < reps; r++) {
        pin29(a);
        a = mul29<FqP>(a, b);
    }
    uint32_t x = 0;
    for (int i = 0; i < 9; i++) x ^= a.l[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

int main() {
    int dev = 0, ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const uint32_t blocks = ncu * 4, threads = 256;  // 4 waves per SIMD
    uint32_t* out;
    hipMalloc(&out, blocks * threads * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float ms_inv = 0, ms_mul = 0;
    const uint32_t reps_inv = 8, reps_mul = 4096;
    for (int it = 0; it < 3; it++) {
        hipEventRecord(a);
        hipLaunchKernelGGL(k_inv, dim3(blocks), dim3(threads), 0, 0, out, reps_inv);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms_inv, a, b);
        hipEventRecord(a);
        hipLaunchKernelGGL(k_mul, dim3(blocks), dim3(threads), 0, 0, out, reps_mul);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms_mul, a, b);
    }
    const double lanes = (double)blocks * threads;
    const double inv_s = lanes * reps_inv / (ms_inv * 1e-3), mul_s = lanes * reps_mul / (ms_mul * 1e-3);
    printf("{\"inversions_per_s\": %.4e, \"mul29_per_s\": %.4e, \"inversion_in_products\": %.1f, \"cus\": %d}\n", inv_s,
           mul_s, mul_s / inv_s, ncu);
    return 0;
}
