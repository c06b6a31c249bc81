// Multiply-add chain throughput on gfx950: one v_mad_u64_u32 per inline asm statement (field29.h's
// mad29_vv, after each of which the compiler places an s_nop, as it does after any inline asm that
// writes an SGPR) against the same instructions eight to a statement (no s_nop inside) and
// against the compiler's own chain (C++ acc += a * b, no asm at all).  Same operands, same
// results; printed as lane multiply-adds per ns.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/ubench_mad_nop.hip -o tools/ubench_mad_nop
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ __forceinline__ void mad1(uint64_t& acc, uint32_t a, uint32_t b) {
    uint64_t c;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(c) : "v"(a), "v"(b));
}

__device__ __forceinline__ void mad8(uint64_t& acc, const uint32_t (&a)[8], const uint32_t (&b)[8]) {
    uint64_t c;
    asm("v_mad_u64_u32 %0, %1, %2, %10, %0\n\t"
        "v_mad_u64_u32 %0, %1, %3, %11, %0\n\t"
        "v_mad_u64_u32 %0, %1, %4, %12, %0\n\t"
        "v_mad_u64_u32 %0, %1, %5, %13, %0\n\t"
        "v_mad_u64_u32 %0, %1, %6, %14, %0\n\t"
        "v_mad_u64_u32 %0, %1, %7, %15, %0\n\t"
        "v_mad_u64_u32 %0, %1, %8, %16, %0\n\t"
        "v_mad_u64_u32 %0, %1, %9, %17, %0"
        : "+v"(acc), "=s"(c)
        : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]),
          "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]));
}

// MODE 0: one asm per multiply-add; 1: eight per asm; 2: plain C++
template <int MODE, int CHAINS>
__global__ void __launch_bounds__(256) k_chain(uint32_t* out, uint32_t steps) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t a[8], b[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        a[i] = (t * 2654435761u + i * 40503u) & 0x1fffffff;
        b[i] = (t * 97u + i * 1013904223u) & 0x1fffffff;
    }
    uint64_t acc[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; c++) acc[c] = c;
    for (uint32_t s = 0; s < steps; s++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) {
            if (MODE == 0) {
#pragma unroll
                for (int i = 0; i < 8; i++) mad1(acc[c], a[i], b[i]);
            } else if (MODE == 1) {
                mad8(acc[c], a, b);
            } else {
#pragma unroll
                for (int i = 0; i < 8; i++) acc[c] += (uint64_t)a[i] * b[i];
            }
            acc[c] >>= 29;  // a column step: keeps the chain dependent and bounded
        }
        a[0] ^= (uint32_t)acc[0] & 0xfff;
    }
    uint64_t r = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; c++) r += acc[c];
    out[t] = (uint32_t)r ^ (uint32_t)(r >> 32);
}

template <int MODE, int CHAINS>
static void run(const char* name, uint32_t blocks, uint32_t threads, uint32_t steps, uint32_t* d,
                uint32_t* ref) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k_chain<MODE, CHAINS>), dim3(blocks), dim3(threads), 0, 0, d, steps);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0, 0);
    const int reps = 5;
    for (int r = 0; r < reps; r++)
        hipLaunchKernelGGL((k_chain<MODE, CHAINS>), dim3(blocks), dim3(threads), 0, 0, d, steps);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    const double n = (double)blocks * threads;
    bool same = true;
    if (ref) {
        uint32_t* h = new uint32_t[(size_t)n];
        uint32_t* g = new uint32_t[(size_t)n];
        (void)hipMemcpy(h, d, (size_t)n * 4, hipMemcpyDeviceToHost);
        (void)hipMemcpy(g, ref, (size_t)n * 4, hipMemcpyDeviceToHost);
        for (size_t i = 0; i < (size_t)n; i++) same &= h[i] == g[i];
        delete[] h;
        delete[] g;
    }
    const double mads = n * steps * CHAINS * 8;
    printf("{\"kernel\": \"%s\", \"blocks\": %u, \"threads\": %u, \"chains\": %d, \"ms\": %.3f, "
           "\"lane_mads_per_ns\": %.1f, \"same_as_asm1\": %s}\n",
           name, blocks, threads, CHAINS, ms, mads / (ms * 1e6), same ? "true" : "false");
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
}

int main() {
    const uint32_t steps = 4096;
    for (uint32_t cfg = 0; cfg < 2; cfg++) {
        // full chip at 8 waves per SIMD, then one wave per SIMD
        const uint32_t blocks = cfg == 0 ? 8192 : 1024, threads = cfg == 0 ? 256 : 64;
        const size_t n = (size_t)blocks * threads;
        uint32_t *d0, *d1;
        if (hipMalloc(&d0, n * 4) != hipSuccess || hipMalloc(&d1, n * 4) != hipSuccess) return 1;
        run<0, 1>("asm1_chain1", blocks, threads, steps, d0, nullptr);
        run<1, 1>("asm8_chain1", blocks, threads, steps, d1, d0);
        run<2, 1>("cxx_chain1", blocks, threads, steps, d1, d0);
        run<0, 2>("asm1_chain2", blocks, threads, steps, d0, nullptr);
        run<1, 2>("asm8_chain2", blocks, threads, steps, d1, d0);
        run<2, 2>("cxx_chain2", blocks, threads, steps, d1, d0);
        (void)hipFree(d0);
        (void)hipFree(d1);
    }
    return 0;
}
