// Microbenchmark (round 6): issue cost per wave-instruction on one SIMD of the non-product VALU
// instructions of the radix-2^29 products and field additions (v_lshrrev_b64 column shift,
// v_and_b32 mask, v_mul_lo_u32, v_add3_u32, v_sub_u32, v_ashrrev_i32, v_cndmask_b32, v_alignbit_b32,
// v_mov_b32 / v_mov_b64) next to v_mad_u64_u32, at 4 and 8 waves per SIMD.  Unlike
// tools/ubench_isa.hip, each repetition's 8 independent instructions are ONE asm statement, so no
// compiler wait-state pad sits between them.  The in-kernel clock (s_memtime / s_memrealtime, as
// eon_diag_clock_probe) converts the time to cycles.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_isa2.hip -o tools/ubench_isa2 && tools/ubench_isa2
#include <hip/hip_runtime.h>

#include <cstdio>

#define R8(I) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7)

template <int MODE>
__global__ void __launch_bounds__(256) k_isa(unsigned* out, unsigned long long* clk, int iters, unsigned seed) {
    unsigned x = threadIdx.x ^ seed, y = blockIdx.x | 1u;
    uint64_t a0 = x, a1 = x + 1, a2 = x + 2, a3 = x + 3, a4 = x + 4, a5 = x + 5, a6 = x + 6, a7 = x + 7;
    unsigned o0 = 1, o1 = 2, o2 = 3, o3 = 4, o4 = 5, o5 = 6, o6 = 7, o7 = 8;
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it++) {
#define A64 "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
#define A32 "+v"(o0), "+v"(o1), "+v"(o2), "+v"(o3), "+v"(o4), "+v"(o5), "+v"(o6), "+v"(o7)
        if constexpr (MODE == 0) {
#define I(c) "v_mad_u64_u32 %" #c ", vcc, %8, %9, %" #c "\n\t"
            asm volatile(R8(I) : A64 : "v"(x), "v"(y) : "vcc");
#undef I
        } else if constexpr (MODE == 1) {
#define I(c) "v_lshrrev_b64 %" #c ", 29, %" #c "\n\t"
            asm volatile(R8(I) : A64);
#undef I
        } else if constexpr (MODE == 2) {
#define I(c) "v_and_b32 %" #c ", 0x1fffffff, %" #c "\n\t"
            asm volatile(R8(I) : A32);
#undef I
        } else if constexpr (MODE == 3) {
#define I(c) "v_mul_lo_u32 %" #c ", %" #c ", %8\n\t"
            asm volatile(R8(I) : A32 : "v"(y));
#undef I
        } else if constexpr (MODE == 4) {
#define I(c) "v_add3_u32 %" #c ", %" #c ", %8, %9\n\t"
            asm volatile(R8(I) : A32 : "v"(x), "v"(y));
#undef I
        } else if constexpr (MODE == 5) {
#define I(c) "v_sub_u32 %" #c ", %" #c ", %8\n\t"
            asm volatile(R8(I) : A32 : "v"(x));
#undef I
        } else if constexpr (MODE == 6) {
#define I(c) "v_ashrrev_i32 %" #c ", 29, %" #c "\n\t"
            asm volatile(R8(I) : A32);
#undef I
        } else if constexpr (MODE == 7) {
#define I(c) "v_cndmask_b32 %" #c ", %" #c ", %8, vcc\n\t"
            asm volatile(R8(I) : A32 : "v"(x));
#undef I
        } else if constexpr (MODE == 8) {
#define I(c) "v_alignbit_b32 %" #c ", %8, %" #c ", 29\n\t"
            asm volatile(R8(I) : A32 : "v"(x));
#undef I
        } else if constexpr (MODE == 9) {
#define I(c) "v_mov_b32 %" #c ", %8\n\t"
            asm volatile(R8(I) : A32 : "v"(x));
#undef I
        } else if constexpr (MODE == 10) {
#define I(c) "v_mov_b64 %" #c ", %8\n\t"
            asm volatile(R8(I) : A64 : "v"((uint64_t)y << 3));
#undef I
        } else if constexpr (MODE == 11) {
#define I(c) "v_lshl_or_b32 %" #c ", %" #c ", 3, %8\n\t"
            asm volatile(R8(I) : A32 : "v"(x));
#undef I
        } else if constexpr (MODE == 12) {
#define I(c) "v_bfe_u32 %" #c ", %" #c ", 3, 29\n\t"
            asm volatile(R8(I) : A32);
#undef I
        } else if constexpr (MODE == 13) {
            // the product's column tail as it runs: mad, mul_lo, mad, shift on 8 chains
#define I(c) "v_mad_u64_u32 %" #c ", vcc, %8, %9, %" #c "\n\t"
            asm volatile(R8(I) : A64 : "v"(x), "v"(y) : "vcc");
#undef I
#define I(c) "v_lshrrev_b64 %" #c ", 29, %" #c "\n\t"
            asm volatile(R8(I) : A64);
#undef I
        }
#undef A64
#undef A32
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] =
        (unsigned)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7) + o0 + o1 + o2 + o3 + o4 + o5 + o6 + o7;
}

template <int MODE>
void run(const char* name, unsigned* d, unsigned long long* clk, int waves_per_simd, int iters, int per_iter) {
    const int blocks = 256 * waves_per_simd;  // 256 CUs x 4 SIMDs x w waves / 4 waves per block
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k_isa<MODE>, dim3(blocks), dim3(256), 0, 0, d, clk, 64, 1u);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_isa<MODE>, dim3(blocks), dim3(256), 0, 0, d, clk, iters, 2u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[2];
    hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost);
    const double mhz = h[1] ? (double)h[0] / (double)h[1] * 100.0 : 0.0;
    const double instr_per_wave = (double)iters * per_iter;
    const double cyc = ms * 1e-3 * mhz * 1e6 / (waves_per_simd * instr_per_wave);
    printf("{\"op\":\"%s\",\"waves_per_simd\":%d,\"ms\":%.3f,\"clock_mhz\":%.0f,\"simd_cycles_per_wave_instr\":%.3f}\n",
           name, waves_per_simd, ms, mhz, cyc);
}

int main() {
    unsigned* d;
    unsigned long long* clk;
    hipMalloc(&d, 256 * 8 * 256 * sizeof(unsigned));
    hipMalloc(&clk, 16);
    const int it = 1 << 15;
    for (int w : {4, 8}) {
        run<0>("v_mad_u64_u32", d, clk, w, it, 8);
        run<1>("v_lshrrev_b64", d, clk, w, it, 8);
        run<2>("v_and_b32 (literal)", d, clk, w, it, 8);
        run<3>("v_mul_lo_u32", d, clk, w, it, 8);
        run<4>("v_add3_u32", d, clk, w, it, 8);
        run<5>("v_sub_u32", d, clk, w, it, 8);
        run<6>("v_ashrrev_i32", d, clk, w, it, 8);
        run<7>("v_cndmask_b32 (vcc)", d, clk, w, it, 8);
        run<8>("v_alignbit_b32", d, clk, w, it, 8);
        run<9>("v_mov_b32", d, clk, w, it, 8);
        run<10>("v_mov_b64", d, clk, w, it, 8);
        run<11>("v_lshl_or_b32", d, clk, w, it, 8);
        run<12>("v_bfe_u32", d, clk, w, it, 8);
        run<13>("v_mad_u64_u32 + v_lshrrev_b64 (8 + 8)", d, clk, w, it, 16);
    }
    return 0;
}
