// Bucket-addition throughput on gfx950: the piece sums' XYZZ mixed addition (madd29_unchecked,
// one accumulator chain per lane) against affine additions batched by Montgomery's trick over K
// independent chains per lane (lambda = dy / dx with one Fermat inversion per K additions: K - 1
// prefix products, the inversion, 2 (K - 1) backward products, then lambda, lambda^2 and
// lambda (x1 - x3) per addition), every chain in registers, the same cheap operand generator in
// both (values in range rather than curve points: the arithmetic is identical).  This is the
// measurement behind DESIGN.md section 10 item 0.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/ubench_batch_affine.hip -o tools/ubench_batch_affine
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../plonky3_eon_amd/csrc/ec29.h"

using namespace eon;

__device__ __forceinline__ F29 gen(uint32_t s) {
    F29 r;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        s = s * 1664525u + 1013904223u;
        r.l[i] = s & M29;
    }
    r.l[8] &= 0xfffff;  // below p
    return r;
}

// a - q p with q = floor(a_8 / (p_8 + 1)): below 2p for any normalised a (as ntt.hip's
// reduce_top29, for Fq)
__device__ __forceinline__ F29 reduce29_below2p(const F29& a) {
    const uint32_t q = a.l[8] / (R29<FqP>::P[8] + 1);
    F29 r;
    int64_t c = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        const int64_t t = (int64_t)a.l[i] - (int64_t)q * R29<FqP>::P[i] + c;
        r.l[i] = (uint32_t)t & M29;
        c = t >> 29;
    }
    return r;
}

// a^(p - 2) in the 29-Montgomery form (square-and-multiply, MSB first; uniform bits)
__device__ __forceinline__ F29 inv29(const F29& a) {
    constexpr uint32_t E[8] = {0xd87cfd45u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                               0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
    F29 r = a;
    for (int bit = 252; bit >= 0; bit--) {
        r = sqr29<FqP>(r);
        if ((E[bit >> 5] >> (bit & 31)) & 1) r = mul29<FqP>(r, a);
    }
    return r;
}

__global__ void __launch_bounds__(256) k_xyzz(uint32_t* out, uint32_t steps) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    G1X29 acc;
    acc.X = gen(t);
    acc.Y = gen(t ^ 0x5bd1e995u);
    acc.ZZ = const29<FqP>(R29<FqP>::ONE);
    acc.ZZZ = acc.ZZ;
    for (uint32_t s = 0; s < steps; s++) {
        F29 px = gen(t * 31u + s), py = gen(t * 17u + s * 7u);
        pin29(px);
        pin29(py);
        madd29_unchecked(acc, px, py);
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) x ^= acc.X.l[i] ^ acc.Y.l[i] ^ acc.ZZ.l[i];
    out[t] = x;
}

template <int K>
__global__ void __launch_bounds__(256) k_affine(uint32_t* out, uint32_t steps) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    F29 ax[K], ay[K];
#pragma unroll
    for (int j = 0; j < K; j++) {
        ax[j] = gen(t * 13u + j);
        ay[j] = gen(t * 29u + j * 3u);
    }
    for (uint32_t s = 0; s < steps; s++) {
        F29 dx[K], pre[K];
#pragma unroll
        for (int j = 0; j < K; j++) {
            F29 px = gen(t * 31u + s * K + j);
            pin29(px);
            dx[j] = sub29<FqP, 2>(px, ax[j]);  // x2 - x1 (x1 < 2p)
            pre[j] = j == 0 ? dx[0] : mul29<FqP>(pre[j - 1], dx[j]);
        }
        F29 inv = inv29(pre[K - 1]);
#pragma unroll
        for (int j = K - 1; j >= 0; j--) {
            const F29 ij = j == 0 ? inv : mul29<FqP>(inv, pre[j - 1]);
            if (j > 0) inv = mul29<FqP>(inv, dx[j]);
            F29 px = gen(t * 31u + s * K + j), py = gen(t * 17u + s * K + j);
            pin29(px);
            pin29(py);
            const F29 lam = mul29<FqP>(sub29<FqP, 2>(py, ay[j]), ij);                       // < 2p
            const F29 x3 = sub29<FqP, 4>(sqr29<FqP>(lam), add29_lazy(ax[j], px));           // < 6p
            ay[j] = sub29<FqP, 2>(mul29<FqP>(lam, sub29<FqP, 6>(ax[j], x3)), ay[j]);       // < 4p
            ax[j] = reduce29_below2p(x3);
        }
    }
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < K; j++)
#pragma unroll
        for (int i = 0; i < 9; i++) x ^= ax[j].l[i] ^ ay[j].l[i];
    out[t] = x;
}

// ---- round 5: one inversion shared by the W waves of a block ----
// Montgomery's trick over every chain of the block: per lane the K-chain prefix products, per
// wave an inclusive product scan of the 64 lane totals (6 shuffle steps, one product each), per
// block the W wave totals in LDS, ONE Fermat inversion by lane 0 of wave 0 while the other waves
// wait at the barrier, then every wave's inverse from the block inverse and the other waves'
// totals, every lane's from its wave's inverse and the exclusive scans of the lane totals (prefix
// and suffix), and the K chain inverses by the backward pass.  The affine additions are the same
// as k_affine's.  Costs per wave and batch: 6K + ~12 products for 64 K additions, plus 350 / W
// (the inversion) -- against the XYZZ madd's 10 per addition (0.156 wave-products per addition).
__device__ __forceinline__ F29 shfl29(const F29& a, int src) {
    F29 r;
#pragma unroll
    for (int i = 0; i < 9; i++) r.l[i] = (uint32_t)__shfl((int)a.l[i], src, 64);
    return r;
}

template <int K, int W>
__global__ void __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(1, 2))) k_affine_xwave(uint32_t* out, uint32_t steps) {
    __shared__ F29 wtot[W];
    __shared__ F29 winv[W];
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const F29 one = const29<FqP>(R29<FqP>::ONE);
    F29 ax[K], ay[K];
#pragma unroll
    for (int j = 0; j < K; j++) {
        ax[j] = gen(t * 13u + j);
        ay[j] = gen(t * 29u + j * 3u);
    }
    for (uint32_t s = 0; s < steps; s++) {
        F29 dx[K], pre[K];
#pragma unroll
        for (int j = 0; j < K; j++) {
            F29 px = gen(t * 31u + s * K + j);
            pin29(px);
            dx[j] = sub29<FqP, 2>(px, ax[j]);
            pre[j] = j == 0 ? dx[0] : mul29<FqP>(pre[j - 1], dx[j]);
        }
        // inclusive product scan of the lane totals over the wave, and the suffix scan
        F29 inc = pre[K - 1], suf = pre[K - 1];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const F29 lo_v = shfl29(inc, (int)lane - o >= 0 ? (int)lane - o : (int)lane);
            const F29 hi_v = shfl29(suf, (int)lane + o < 64 ? (int)lane + o : (int)lane);
            if ((int)lane - o >= 0) inc = mul29<FqP>(inc, lo_v);
            if ((int)lane + o < 64) suf = mul29<FqP>(suf, hi_v);
        }
        const F29 excl_lo = lane ? shfl29(inc, (int)lane - 1) : one;  // lanes below
        const F29 excl_hi = lane < 63 ? shfl29(suf, (int)lane + 1) : one;  // lanes above
        if (lane == 63) wtot[w] = inc;
        __syncthreads();
        if (threadIdx.x == 0) {  // the block's one inversion, then every wave's inverse
            F29 pw[W];
            pw[0] = wtot[0];
            for (int v = 1; v < W; v++) pw[v] = mul29<FqP>(pw[v - 1], wtot[v]);
            F29 iv = reduce29_below2p(inv29(pw[W - 1]));
            for (int v = W - 1; v >= 1; v--) {
                winv[v] = mul29<FqP>(iv, pw[v - 1]);
                iv = mul29<FqP>(iv, wtot[v]);
            }
            winv[0] = iv;
        }
        __syncthreads();
        // this lane's inverse: the wave's inverse times the other lanes' totals
        F29 inv = mul29<FqP>(mul29<FqP>(winv[w], excl_lo), excl_hi);
#pragma unroll
        for (int j = K - 1; j >= 0; j--) {
            const F29 ij = j == 0 ? inv : mul29<FqP>(inv, pre[j - 1]);
            if (j > 0) inv = mul29<FqP>(inv, dx[j]);
            F29 px = gen(t * 31u + s * K + j), py = gen(t * 17u + s * K + j);
            pin29(px);
            pin29(py);
            const F29 lam = mul29<FqP>(sub29<FqP, 2>(py, ay[j]), ij);
            const F29 x3 = sub29<FqP, 4>(sqr29<FqP>(lam), add29_lazy(ax[j], px));
            ay[j] = sub29<FqP, 2>(mul29<FqP>(lam, sub29<FqP, 6>(ax[j], x3)), ay[j]);
            ax[j] = reduce29_below2p(x3);
        }
    }
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < K; j++)
#pragma unroll
        for (int i = 0; i < 9; i++) x ^= ax[j].l[i] ^ ay[j].l[i];
    out[t] = x;
}

template <class F>
static double rate(F launch, double adds) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float best = 1e30f;
    for (int it = 0; it < 3; it++) {
        (void)hipEventRecord(a);
        launch();
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (it && ms < best) best = ms;
    }
    return adds / (best * 1e-3);
}

int main() {
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t* out;
    (void)hipMalloc(&out, (size_t)ncu * 4 * 1024 * 4 * 8);
    // XYZZ: 4 waves per SIMD (the piece sums' occupancy)
    const uint32_t xb = ncu * 4, xs = 512;
    const double r_xyzz = rate([&] { hipLaunchKernelGGL(k_xyzz, dim3(xb), dim3(256), 0, 0, out, xs); },
                               (double)xb * 256 * xs);
    printf("{\"form\":\"xyzz_madd\",\"adds_per_s\":%.4e,\"cus\":%d}\n", r_xyzz, ncu);
    auto affine = [&](auto kern, int k, uint32_t steps) {
        const uint32_t blocks = ncu * 4;
        const double r = rate([&] { hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, steps); },
                              (double)blocks * 256 * steps * k);
        printf("{\"form\":\"batch_affine\",\"K\":%d,\"adds_per_s\":%.4e,\"vs_xyzz\":%.3f}\n", k, r, r / r_xyzz);
    };
    affine(k_affine<1>, 1, 8);
    affine(k_affine<2>, 2, 8);
    affine(k_affine<4>, 4, 8);
    affine(k_affine<8>, 8, 8);
    affine(k_affine<16>, 16, 4);
    // cross-wave shared inversion (round 5): W waves per block, K chains per lane; the block count
    // fills the CUs at the occupancy the register budget allows
    auto xwave = [&](auto kern, int k, int wv, uint32_t blocks_per_cu, uint32_t steps) {
        const uint32_t blocks = ncu * blocks_per_cu;
        const double r = rate([&] { hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * wv), 0, 0, out, steps); },
                              (double)blocks * 64 * wv * steps * k);
        printf("{\"form\":\"batch_affine_xwave\",\"K\":%d,\"W\":%d,\"adds_per_s\":%.4e,\"vs_xyzz\":%.3f}\n", k, wv, r,
               r / r_xyzz);
    };
    xwave(k_affine_xwave<4, 16>, 4, 16, 1, 8);
    xwave(k_affine_xwave<8, 8>, 8, 8, 1, 8);
    xwave(k_affine_xwave<16, 4>, 16, 4, 1, 4);
    xwave(k_affine_xwave<16, 16>, 16, 16, 1, 2);
    (void)hipFree(out);
    return 0;
}
