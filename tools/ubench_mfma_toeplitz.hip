// Round-6 research: a 256 x 256-bit product by a FIXED operand w (a twiddle,
// the modulus of a Montgomery reduction) on the integer matrix cores -- v_mfma_i32_16x16x64_i8 --
// as a Toeplitz GEMM, against the radix-2^29 VALU schoolbook it would replace.  Both compute the
// full 512-bit y w of 64 lanes' y (9 normalised 29-bit limbs each, one y per lane, as the MSM /
// NTT code holds them) and return it as 18 normalised 29-bit limbs, checked equal lane by lane.
//
// MFMA path, per wave (64 products):
//   1. digit split: y -> 38 unsigned 7-bit digits (i8 operands are signed; 7-bit digits keep every
//      column sum positive: <= 38 * 127^2 < 2^20), 4 per VGPR;
//   2. operand layout through LDS: group g (products 16g .. 16g+15) is the B operand, lane l holding
//      digits 16(l>>4) .. +15 of product 16g + (l & 15) (one ds_read_b128 per group);
//   3. 5 MFMAs per group: A_t[m][k] = wd[16t + m - k] (Toeplitz of w, constant, built once), so
//      D_t[m][n] = column 16t + m of product n; 75 columns used of 80;
//   4. recombination: D back through LDS to the product's lane, then sum_o c_o 2^(7o) carried into
//      29-bit limbs (one v_mad_u64_u32 per column -- c_o times 2^(7o - base) into a 64-bit running
//      sum -- plus a mask and a shift per limb).
// VALU path: 81 v_mad_u64_u32 against the SGPR limbs of w, a mask and a 64-bit shift per column.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/ubench_mfma_toeplitz.hip -o tools/ubench_mfma_toeplitz
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t M29 = (1u << 29) - 1;
constexpr int ND = 38;  // 7-bit digits of a value < 2^266
constexpr int NC = 2 * ND - 1;  // 75 product columns
constexpr int TILES = 5;        // 16 columns each

struct W {
    uint32_t l[9];    // w in 29-bit limbs
    uint8_t d[64];    // w's 7-bit digits (zero-padded)
};

__device__ __forceinline__ void digits7(const uint32_t* y, uint32_t* packed /* 10 words */) {
    // y (9 x 29) -> 9 32-bit words, then 7-bit digits packed 4 per word
    uint32_t w[9];
#pragma unroll
    for (int i = 0; i < 9; i++) {
        const int bit = 32 * i;
        const int li = bit / 29, s = bit % 29;
        uint64_t v = (uint64_t)y[li] >> s;
        if (li + 1 < 9) v |= (uint64_t)y[li + 1] << (29 - s);
        if (li + 2 < 9 && 58 - s < 64) v |= (uint64_t)y[li + 2] << (58 - s);
        w[i] = (uint32_t)v;
    }
#pragma unroll
    for (int q = 0; q < 10; q++) {
        uint32_t p = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int d = 4 * q + j;
            uint32_t dig = 0;
            if (d < ND) {
                const int bit = 7 * d, wi = bit >> 5, s = bit & 31;
                uint64_t v = w[wi];
                if (wi + 1 < 9) v |= (uint64_t)w[wi + 1] << 32;
                dig = (uint32_t)(v >> s) & 127u;
            }
            p |= dig << (8 * j);
        }
        packed[q] = p;
    }
}

// VALU schoolbook y w -> 18 limbs (w's limbs uniform: SGPR operands)
__global__ void __launch_bounds__(256) k_valu(const uint32_t* ys, W w, uint32_t* out, int reps) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t y[9];
#pragma unroll
    for (int i = 0; i < 9; i++) y[i] = ys[t * 9 + i];
    uint32_t r[18];
    for (int it = 0; it < reps; it++) {
        uint64_t acc = 0;
#pragma unroll
        for (int k = 0; k < 17; k++) {
#pragma unroll
            for (int i = 0; i < 9; i++)
                if (k - i >= 0 && k - i < 9) acc += (uint64_t)y[i] * w.l[k - i];
            r[k] = (uint32_t)acc & M29;
            acc >>= 29;
        }
        r[17] = (uint32_t)acc;
        // the next repetition multiplies the high half of this product: every limb depends on the
        // previous one (a single-bit feedback let the compiler hoist the other limbs' products)
#pragma unroll
        for (int i = 0; i < 9; i++) y[i] = r[9 + i] & (i == 8 ? 0x3fffffu : M29);
    }
#pragma unroll
    for (int i = 0; i < 18; i++) out[t * 18 + i] = r[i];
}

// MFMA path: one wave = 64 products; 256 threads = 4 waves per block
__global__ void __launch_bounds__(256) k_mfma(const uint32_t* ys, W w, uint32_t* out, int reps) {
    __shared__ uint32_t dig_lds[4][64][16];  // per wave: each lane's digit words (10 used, rest 0)
    __shared__ int32_t cols[4][64][TILES * 16 + 1];  // per wave: each product's 80 column sums
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6, blk = lane >> 4;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t y[9];
#pragma unroll
    for (int i = 0; i < 9; i++) y[i] = ys[t * 9 + i];
    for (int q = 10; q < 16; q++) dig_lds[wv][lane][q] = 0;
    // the Toeplitz A tiles of w: lane l holds A_t[row l&15][k = 16(l>>4) + j], j = 0..15
    i32x4 A[TILES];
#pragma unroll
    for (int tt = 0; tt < TILES; tt++) {
        uint32_t q[4];
#pragma unroll
        for (int r4 = 0; r4 < 4; r4++) {
            uint32_t p = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int k = 16 * (int)blk + 4 * r4 + j;
                const int idx = 16 * tt + (int)(lane & 15) - k;
                const uint32_t dv = (idx >= 0 && idx < ND) ? w.d[idx] : 0u;
                p |= dv << (8 * j);
            }
            q[r4] = p;
        }
        A[tt] = i32x4{(int)q[0], (int)q[1], (int)q[2], (int)q[3]};
    }
    uint32_t r[18];
    for (int it = 0; it < reps; it++) {
        uint32_t pk[10];
        digits7(y, pk);
#pragma unroll
        for (int q = 0; q < 10; q++) dig_lds[wv][lane][q] = pk[q];
        __syncthreads();
#pragma unroll
        for (int g = 0; g < 4; g++) {
            // B: lane l holds digits 16(l>>4) .. +15 of product 16g + (l & 15)
            const uint32_t* p = &dig_lds[wv][16 * g + (lane & 15)][4 * blk];
            const i32x4 B = i32x4{(int)p[0], (int)p[1], (int)p[2], (int)p[3]};
#pragma unroll
            for (int tt = 0; tt < TILES; tt++) {
                i32x4 acc = i32x4{0, 0, 0, 0};
                acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[tt], B, acc, 0, 0, 0);
                // D[row 4(l>>4) + i][col l & 15] = column 16 tt + 4(l>>4) + i of product 16g + (l & 15)
#pragma unroll
                for (int i = 0; i < 4; i++) cols[wv][16 * g + (lane & 15)][16 * tt + 4 * blk + i] = acc[i];
            }
        }
        __syncthreads();
        // recombination: sum_o c_o 2^(7o) -> 18 limbs of 29 bits
        uint64_t acc = 0;
        int base = 0, outi = 0;
#pragma unroll
        for (int o = 0; o < NC; o++) {
            acc += (uint64_t)(uint32_t)cols[wv][lane][o] << (7 * o - base);
            while (7 * (o + 1) - base >= 29 && outi < 17) {
                r[outi++] = (uint32_t)acc & M29;
                acc >>= 29;
                base += 29;
            }
        }
        while (outi < 17) {
            r[outi++] = (uint32_t)acc & M29;
            acc >>= 29;
        }
        r[17] = (uint32_t)acc;
#pragma unroll
        for (int i = 0; i < 9; i++) y[i] = r[9 + i] & (i == 8 ? 0x3fffffu : M29);
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 18; i++) out[t * 18 + i] = r[i];
}

int main() {
    const int blocks = 4096, n = blocks * 256;
    std::vector<uint32_t> hy((size_t)n * 9);
    uint64_t s = 88172645463325252ull;
    auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (uint32_t)s; };
    for (auto& v : hy) v = rnd() & M29;
    for (int i = 0; i < n; i++) hy[(size_t)i * 9 + 8] &= 0x3fffff;  // y < 2^254
    W w{};
    for (int i = 0; i < 9; i++) w.l[i] = rnd() & M29;
    w.l[8] &= 0x3fffff;
    // w's 7-bit digits from its bits
    for (int d = 0; d < 64; d++) {
        uint32_t v = 0;
        for (int b = 0; b < 7; b++) {
            const int bit = 7 * d + b, li = bit / 29, s2 = bit % 29;
            if (li < 9) v |= ((w.l[li] >> s2) & 1u) << b;
        }
        w.d[d] = d < ND ? (uint8_t)v : 0;
    }
    uint32_t *dy, *o1, *o2;
    hipMalloc(&dy, hy.size() * 4);
    hipMalloc(&o1, (size_t)n * 18 * 4);
    hipMalloc(&o2, (size_t)n * 18 * 4);
    hipMemcpy(dy, hy.data(), hy.size() * 4, hipMemcpyHostToDevice);
    // correctness: one repetition each
    hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(256), 0, 0, dy, w, o1, 3);
    hipLaunchKernelGGL(k_mfma, dim3(blocks), dim3(256), 0, 0, dy, w, o2, 3);
    hipDeviceSynchronize();
    std::vector<uint32_t> h1((size_t)n * 18), h2((size_t)n * 18);
    hipMemcpy(h1.data(), o1, h1.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(h2.data(), o2, h2.size() * 4, hipMemcpyDeviceToHost);
    size_t bad = 0;
    for (int i = 0; i < n; i++)
        for (int j = 0; j < 18; j++)
            if (h1[(size_t)i * 18 + j] != h2[(size_t)i * 18 + j]) {
                bad++;
                break;
            }
    printf("{\"check\":\"mfma product == valu product\",\"lanes\":%d,\"mismatching_lanes\":%zu}\n", n, bad);
    const int reps = 256;
    for (int k = 0; k < 2; k++) {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        if (k == 0)
            hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(256), 0, 0, dy, w, o1, reps);
        else
            hipLaunchKernelGGL(k_mfma, dim3(blocks), dim3(256), 0, 0, dy, w, o2, reps);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        printf("{\"path\":\"%s\",\"products\":%.0f,\"ms\":%.3f,\"products_per_s\":%.4g}\n",
               k == 0 ? "valu radix-2^29 schoolbook (81 v_mad_u64_u32)" : "mfma i32_16x16x64_i8 Toeplitz + split + recombine",
               (double)n * reps, ms, (double)n * reps / (ms * 1e-3));
    }
    return 0;
}
