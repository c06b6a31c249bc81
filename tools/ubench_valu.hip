// VALU issue cost (gfx950) of the instructions a wide-integer product can be built from:
// v_fma_f64, v_mad_u64_u32, v_lshl_add_u64 (64-bit add), v_mul_lo_u32, v_mul_hi_u32, v_fma_f32.
// Eight independent chains per thread (inline asm, exact instruction), 32 waves per CU.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr int CH = 8, IT = 4096;

#define KERNEL(NAME, T, INIT, ASM, CONS)                                                   \
    __global__ void __launch_bounds__(256) NAME(T* out, T s) {                            \
        T x[CH];                                                                           \
        for (int c = 0; c < CH; c++) x[c] = INIT;                                          \
        for (int i = 0; i < IT; i++) {                                                     \
            _Pragma("unroll") for (int c = 0; c < CH; c++) asm volatile(ASM : "+v"(x[c]) : "v"(s) CONS); \
        }                                                                                  \
        T r = 0;                                                                           \
        for (int c = 0; c < CH; c++) r += x[c];                                            \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r;                                    \
    }

KERNEL(k_fma_f64, double, threadIdx.x * 1e-3 + c, "v_fma_f64 %0, %0, %1, %1", )
KERNEL(k_mul_f64, double, threadIdx.x * 1e-3 + c, "v_mul_f64 %0, %0, %1", )
KERNEL(k_add_f64, double, threadIdx.x * 1e-3 + c, "v_add_f64 %0, %0, %1", )
KERNEL(k_fma_f32, float, threadIdx.x * 1e-3f + c, "v_fma_f32 %0, %0, %1, %1", )
__global__ void __launch_bounds__(256) k_mad_u64(uint64_t* out, uint64_t s) {
    uint64_t x[CH];
    const uint32_t a = (uint32_t)s, b = (uint32_t)(s >> 7);
    for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c;
    for (int i = 0; i < IT; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(x[c]) : "v"(a), "v"(b) : "vcc");
    }
    uint64_t r = 0;
    for (int c = 0; c < CH; c++) r += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
KERNEL(k_lshl_add_u64, uint64_t, threadIdx.x + c, "v_lshl_add_u64 %0, %0, 0, %1", )
KERNEL(k_mul_lo_u32, uint32_t, threadIdx.x + c, "v_mul_lo_u32 %0, %0, %1", )
KERNEL(k_mul_hi_u32, uint32_t, threadIdx.x + c, "v_mul_hi_u32 %0, %0, %1", )
KERNEL(k_add_co_u32, uint32_t, threadIdx.x + c, "v_add_co_u32 %0, vcc, %0, %1", : "vcc")
KERNEL(k_addc_co_u32, uint32_t, threadIdx.x + c, "v_addc_co_u32 %0, vcc, %0, %1, vcc", : "vcc")
KERNEL(k_mad_u32_u24, uint32_t, threadIdx.x + c, "v_mad_u32_u24 %0, %0, %1, %0", )

template <class T>
static void run(const char* name, void (*k)(T*, T), T s, void* buf) {
    const int blocks = 256 * 8;  // 8 workgroups (32 waves) per CU
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    k<<<blocks, 256>>>((T*)buf, s);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    for (int r = 0; r < 5; r++) k<<<blocks, 256>>>((T*)buf, s);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    const double waves = blocks * 4.0, winstr = 5.0 * waves * IT * CH;
    const double cyc = (ms * 1e-3 * 2.4e9 * 1024) / winstr;  // per SIMD, 1024 SIMDs, 2.4 GHz
    printf("%-16s %8.3f ms  %.2f cycles per wave64 instruction per SIMD at 2.4 GHz\n", name, ms / 5, cyc);
}

int main() {
    void* buf;
    (void)hipMalloc(&buf, (size_t)256 * 8 * 256 * 8);
    run("v_fma_f64", k_fma_f64, 1.0000001, buf);
    run("v_mul_f64", k_mul_f64, 1.0000001, buf);
    run("v_add_f64", k_add_f64, 1.0000001, buf);
    run("v_fma_f32", k_fma_f32, 1.0000001f, buf);
    run("v_mad_u64_u32", k_mad_u64, (uint64_t)12345, buf);
    run("v_lshl_add_u64", k_lshl_add_u64, (uint64_t)12345, buf);
    run("v_mul_lo_u32", k_mul_lo_u32, 12345u, buf);
    run("v_mul_hi_u32", k_mul_hi_u32, 12345u, buf);
    run("v_add_co_u32", k_add_co_u32, 12345u, buf);
    run("v_addc_co_u32", k_addc_co_u32, 12345u, buf);
    run("v_mad_u32_u24", k_mad_u32_u24, 12345u, buf);
    (void)hipFree(buf);
    return 0;
}
