// Microbenchmark: issue cost of the instructions in the Montgomery product stream on gfx950
// (v_mad_u64_u32, its v_addc_co_u32 carry capture, a plain v_add_u32, v_mul_lo_u32 and the
// v_lshl_add_u64 column shift), each as 8 independent chains per wave at 4 and 8 waves per SIMD.
// Prints cycles per wave-instruction per SIMD at the measured kernel time and a 2.4 GHz clock.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ void __launch_bounds__(256) k_isa(unsigned* out, int iters, unsigned seed) {
    unsigned x = threadIdx.x ^ seed, y = blockIdx.x | 1u;
    uint64_t a[8];
    unsigned o[8];
#pragma unroll
    for (int c = 0; c < 8; c++) {
        a[c] = (uint64_t)(x + c) << 7;
        o[c] = c;
    }
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
            for (int c = 0; c < 8; c++) {
                if (MODE == 0) {
                    asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(a[c]) : "v"(x), "v"(y) : "s40", "s41");
                } else if (MODE == 1) {
                    uint64_t cc;
                    asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(a[c]), "=s"(cc) : "v"(x), "v"(y));
                    asm volatile("v_addc_co_u32_e64 %0, %1, %0, 0, %2" : "+v"(o[c]), "=s"(cc) : "s"(cc));
                } else if (MODE == 2) {
                    asm volatile("v_add_u32 %0, %0, %1" : "+v"(o[c]) : "v"(x));
                } else if (MODE == 3) {
                    asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(o[c]) : "v"(y));
                } else if (MODE == 4) {
                    asm volatile("v_lshl_add_u64 %0, %0, 32, %1" : "+v"(a[c]) : "v"(a[(c + 1) & 7]));
                } else if (MODE == 5) {
                    uint64_t cc;
                    asm volatile("v_add_co_u32_e64 %0, %1, %0, %2" : "+v"(o[c]), "=s"(cc) : "v"(x));
                } else if (MODE == 6) {
                    // VOP2 forms: carry in/out through VCC
                    asm volatile("v_add_co_u32_e32 %0, vcc, %0, %1\n\tv_addc_co_u32_e32 %2, vcc, 0, %2, vcc"
                                 : "+v"(o[c]), "+v"(o[(c + 4) & 7]) : "v"(x) : "vcc");
                } else if (MODE == 7) {
                    asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0\n\tv_addc_co_u32_e32 %3, vcc, 0, %3, vcc"
                                 : "+v"(a[c]), "+v"(o[c]) : "v"(x), "v"(y) : "vcc");
                } else if (MODE == 8) {
                    uint64_t cc;
                    asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(a[c]), "=s"(cc) : "v"(x), "v"(y));
                    asm volatile("v_cndmask_b32_e64 %0, 0, 1, %1" : "=v"(o[c]) : "s"(cc));
                } else if (MODE == 9) {
                    asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(o[c]) : "v"(x), "v"(y));
                } else if (MODE == 10) {
                    asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(o[c]) : "v"(y));
                }
            }
    }
    unsigned s = 0;
#pragma unroll
    for (int c = 0; c < 8; c++) s += (unsigned)a[c] + (unsigned)(a[c] >> 32) + o[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE>
void run(const char* name, unsigned* d, int waves_per_simd, int iters) {
    const int blocks = 256 * waves_per_simd;  // 256 CUs x 4 SIMDs x w waves / 4 waves per block
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k_isa<MODE>, dim3(blocks), dim3(256), 0, 0, d, 64, 1u);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_isa<MODE>, dim3(blocks), dim3(256), 0, 0, d, iters, 2u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double instr_per_wave = (double)iters * 16;  // counted instructions per wave
    const double cyc = ms * 1e-3 * 2.4e9 / (waves_per_simd * instr_per_wave);
    printf("{\"op\":\"%s\",\"waves_per_simd\":%d,\"ms\":%.3f,\"simd_cycles_per_wave_instr\":%.3f}\n", name,
           waves_per_simd, ms, cyc);
}

int main() {
    unsigned* d;
    hipMalloc(&d, 256 * 8 * 256 * sizeof(unsigned));
    for (int w : {4, 8}) {
        run<0>("v_mad_u64_u32", d, w, 1 << 14);
        run<1>("v_mad_u64_u32+v_addc", d, w, 1 << 14);
        run<2>("v_add_u32", d, w, 1 << 14);
        run<3>("v_mul_lo_u32", d, w, 1 << 14);
        run<4>("v_lshl_add_u64", d, w, 1 << 14);
        run<5>("v_add_co_u32", d, w, 1 << 14);
        run<6>("v_add_co_u32_e32+v_addc_co_u32_e32 (vcc)", d, w, 1 << 14);
        run<7>("v_mad_u64_u32(vcc)+v_addc_co_u32_e32", d, w, 1 << 14);
        run<8>("v_mad_u64_u32+v_cndmask_b32", d, w, 1 << 14);
        run<9>("v_add3_u32", d, w, 1 << 14);
        run<10>("v_mul_hi_u32", d, w, 1 << 14);
    }
    return 0;
}
