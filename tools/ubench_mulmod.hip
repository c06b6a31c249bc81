// Microbenchmark: 256-bit Montgomery multiply throughput on gfx950 (Fr and Fq), with 1/2/4
// independent chains per thread.  Prints mulmod/s so the NTT/MSM rooflines use a measured peak.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../plonky3_eon_amd/csrc/field.h"

using namespace eon;

// Montgomery square in the same column order as mul_fips: the product half of column k is
// 2 * sum_{i<j, i+j=k} a_i a_j (summed in a fresh 96-bit accumulator, then doubled into the column)
// plus a_{k/2}^2, so the product half costs 36 v_mad_u64_u32 instead of 64 (100 per square).
__device__ __forceinline__ void add_doubled(Acc96& acc, const Acc96& off) {
    const uint64_t d = off.lo << 1;
    const uint32_t dov = (off.ov << 1) | (uint32_t)(off.lo >> 63);
    const uint64_t s = acc.lo + d;
    acc.ov += dov + (uint32_t)(s < d);
    acc.lo = s;
}

template <class M>
__device__ __forceinline__ Fe<M> sqr_fips(const Fe<M>& a) {
    uint32_t m[8], t[8];
    Acc96 acc{0, 0};
#pragma unroll
    for (int k = 0; k < 8; k++) {
        if (k >= 1) {
            Acc96 off{0, 0};
#pragma unroll
            for (int i = 0; 2 * i < k; i++)
                if (i != k - i) mac(off, a.v[i], a.v[k - i]);
            add_doubled(acc, off);
        }
        if ((k & 1) == 0) mac(acc, a.v[k / 2], a.v[k / 2]);
#pragma unroll
        for (int i = 0; i < k; i++) mac_s(acc, m[i], M::P[k - i]);
        m[k] = (uint32_t)acc.lo * M::INV;
        mac_s(acc, m[k], M::P[0]);
        acc.lo = (acc.lo >> 32) | ((uint64_t)acc.ov << 32);
        acc.ov = 0;
    }
#pragma unroll
    for (int k = 8; k < 15; k++) {
        if (k <= 13) {
            Acc96 off{0, 0};
#pragma unroll
            for (int i = k - 7; 2 * i < k; i++) mac(off, a.v[i], a.v[k - i]);
            add_doubled(acc, off);
        }
        if ((k & 1) == 0) mac(acc, a.v[k / 2], a.v[k / 2]);
#pragma unroll
        for (int i = k - 7; i < 8; i++) mac_s(acc, m[i], M::P[k - i]);
        t[k - 8] = (uint32_t)acc.lo;
        acc.lo = (acc.lo >> 32) | ((uint64_t)acc.ov << 32);
        acc.ov = 0;
    }
    t[7] = (uint32_t)acc.lo;
    Fe<M> r, d;
    int64_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        r.v[i] = t[i];
        br += (int64_t)t[i] - M::P[i];
        d.v[i] = (uint32_t)br;
        br >>= 32;
    }
    return br < 0 ? r : d;
}


// Variant: the carry of each product goes through VCC and a 4-byte VOP2 v_addc (one asm block,
// with the VALU-SGPR-write -> carry-read wait state spelled out).
__device__ __forceinline__ void mac_vcc(Acc96& acc, uint32_t x, uint32_t y) {
    asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+v"(acc.lo), "+v"(acc.ov) : "v"(x), "v"(y) : "vcc");
}
__device__ __forceinline__ void mac_s_vcc(Acc96& acc, uint32_t x, uint32_t y) {
    asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+v"(acc.lo), "+v"(acc.ov) : "v"(x), "s"(y) : "vcc");
}
template <class M>
__device__ __forceinline__ Fe<M> mul_fips_vcc(const Fe<M>& a, const Fe<M>& b) {
    uint32_t m[8], t[8];
    Acc96 acc{0, 0};
#pragma unroll
    for (int k = 0; k < 8; k++) {
#pragma unroll
        for (int i = 0; i <= k; i++) mac_vcc(acc, a.v[i], b.v[k - i]);
#pragma unroll
        for (int i = 0; i < k; i++) mac_s_vcc(acc, m[i], M::P[k - i]);
        m[k] = (uint32_t)acc.lo * M::INV;
        mac_s_vcc(acc, m[k], M::P[0]);
        acc.lo = (acc.lo >> 32) | ((uint64_t)acc.ov << 32);
        acc.ov = 0;
    }
#pragma unroll
    for (int k = 8; k < 15; k++) {
#pragma unroll
        for (int i = k - 7; i < 8; i++) mac_vcc(acc, a.v[i], b.v[k - i]);
#pragma unroll
        for (int i = k - 7; i < 8; i++) mac_s_vcc(acc, m[i], M::P[k - i]);
        t[k - 8] = (uint32_t)acc.lo;
        acc.lo = (acc.lo >> 32) | ((uint64_t)acc.ov << 32);
        acc.ov = 0;
    }
    t[7] = (uint32_t)acc.lo;
    Fe<M> r, d;
    int64_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        r.v[i] = t[i];
        br += (int64_t)t[i] - M::P[i];
        d.v[i] = (uint32_t)br;
        br >>= 32;
    }
    return br < 0 ? r : d;
}


template <class M, int CH, int FIPS>
__global__ void __launch_bounds__(256) k_mul(const Fe<M>* in, Fe<M>* out, int iters) {
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    Fe<M> x[CH];
    Fe<M> y = in[(tid + 7) & 1023];
#pragma unroll
    for (int c = 0; c < CH; c++) x[c] = in[(tid + c) & 1023];
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int c = 0; c < CH; c++) x[c] = FIPS == 2 ? mul_fips_vcc(x[c], y) : FIPS ? mul_fips(x[c], y) : mul_cios(x[c], y);
    }
    Fe<M> acc = x[0];
#pragma unroll
    for (int c = 1; c < CH; c++) acc = add(acc, x[c]);
    out[tid] = acc;
}

// squaring chains (sqr_fips, 100 v_mad_u64_u32) against the multiply chains above
template <class M>
__global__ void __launch_bounds__(256) k_sqr(const Fe<M>* in, Fe<M>* out, int iters) {
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    Fe<M> x0 = in[tid & 1023], x1 = in[(tid + 1) & 1023];
    for (int it = 0; it < iters; it++) {
        x0 = sqr_fips(x0);
        x1 = sqr_fips(x1);
    }
    out[tid] = add(x0, x1);
}

template <class M>
void run_sqr(const char* name, Fe<M>* d_in, Fe<M>* d_out, int blocks, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k_sqr<M><<<blocks, 256>>>(d_in, d_out, 16);
    hipDeviceSynchronize();
    hipEventRecord(a);
    k_sqr<M><<<blocks, 256>>>(d_in, d_out, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    double n = (double)blocks * 256 * iters * 2;
    printf("{\"field\":\"%s\",\"op\":\"sqr\",\"chains\":2,\"blocks\":%d,\"ms\":%.3f,\"sqr_per_s\":%.4e}\n", name,
           blocks, ms, n / (ms * 1e-3));
}

// the FIPS product followed by 64 extra s_nop 0: prices one s_nop in the mulmod stream
template <class M>
__global__ void __launch_bounds__(256) k_mul_nops(const Fe<M>* in, Fe<M>* out, int iters) {
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    Fe<M> y = in[(tid + 7) & 1023];
    Fe<M> x0 = in[tid & 1023], x1 = in[(tid + 1) & 1023];
    for (int it = 0; it < iters; it++) {
        x0 = mul_fips(x0, y);
        asm volatile(".rept 32\n\ts_nop 0\n\t.endr");
        x1 = mul_fips(x1, y);
        asm volatile(".rept 32\n\ts_nop 0\n\t.endr");
    }
    out[tid] = add(x0, x1);
}

template <class M>
void run_nops(const char* name, Fe<M>* d_in, Fe<M>* d_out, int blocks, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k_mul_nops<M><<<blocks, 256>>>(d_in, d_out, 16);
    hipDeviceSynchronize();
    hipEventRecord(a);
    k_mul_nops<M><<<blocks, 256>>>(d_in, d_out, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    double n = (double)blocks * 256 * iters * 2;
    printf("{\"field\":\"%s\",\"fips\":\"+64nops\",\"chains\":2,\"blocks\":%d,\"ms\":%.3f,\"mulmod_per_s\":%.4e}\n", name,
           blocks, ms, n / (ms * 1e-3));
}

template <class M>
__global__ void k_check(const Fe<M>* a, const Fe<M>* b, int n, unsigned* bad, Fe<M>* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fe<M> x = mul_cios(a[i], b[i]), y = mul_fips(a[i], b[i]);
    if (x != y) atomicAdd(bad, 1u);
    if (mul_fips_vcc(a[i], b[i]) != y || sqr_fips(a[i]) != mul_fips(a[i], a[i]) || sqr_fips(b[i]) != mul_cios(b[i], b[i])) atomicAdd(bad + 1, 1u);
    out[i] = y;
}

template <class M, int CH, int FIPS>
void run(const char* name, Fe<M>* d_in, Fe<M>* d_out, int blocks, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k_mul<M, CH, FIPS><<<blocks, 256>>>(d_in, d_out, 16);
    hipDeviceSynchronize();
    hipEventRecord(a);
    k_mul<M, CH, FIPS><<<blocks, 256>>>(d_in, d_out, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    double n = (double)blocks * 256 * iters * CH;
    printf("{\"field\":\"%s\",\"fips\":%d,\"chains\":%d,\"blocks\":%d,\"ms\":%.3f,\"mulmod_per_s\":%.4e}\n", name, (int)FIPS, CH,
           blocks, ms, n / (ms * 1e-3));
}

int main() {
    std::vector<Fr> h(1024);
    for (int i = 0; i < 1024; i++) h[i] = from_u64<FrP>(0x9e3779b97f4a7c15ull * (i + 1));
    Fr *d_in, *d_out;
    const int maxblocks = 256 * 32;
    hipMalloc(&d_in, 1024 * sizeof(Fr));
    hipMalloc(&d_out, (size_t)maxblocks * 256 * sizeof(Fr));
    hipMemcpy(d_in, h.data(), 1024 * sizeof(Fr), hipMemcpyHostToDevice);
    {
        // correctness: GENERATOR = 5 in Montgomery form (bn254/src/field.rs:372-377)
        Fr g = from_u64<FrP>(5);
        const uint32_t G[8] = {0x9fffffe6u, 0x1b0d0ef9u, 0xa32a913fu, 0xeaba68a3u,
                               0xd8dd0689u, 0x47d8eb76u, 0x20f5bbc3u, 0x15d00855u};
        bool ok = true;
        for (int i = 0; i < 8; i++) ok &= g.v[i] == G[i];
        printf("{\"host_generator_ok\":%d}\n", (int)ok);
        const int n = 1 << 20;
        std::vector<Fr> ha(n), hb(n);
        uint64_t st = 1;
        auto nx = [&]() { st += 0x9e3779b97f4a7c15ull; uint64_t z = st; z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull; z = (z ^ (z >> 27)) * 0x94d049bb133111ebull; return z ^ (z >> 31); };
        for (int i = 0; i < n; i++) {
            ha[i] = from_u64<FrP>(nx()); ha[i] = mul(ha[i], from_u64<FrP>(nx()));
            hb[i] = from_u64<FrP>(nx()); hb[i] = mul(hb[i], hb[i]);
        }
        hb[0] = Fr::zero(); ha[1] = neg(Fr::one()); hb[1] = neg(Fr::one());
        Fr *da, *db, *dout; unsigned* dbad;
        hipMalloc(&da, n * sizeof(Fr)); hipMalloc(&db, n * sizeof(Fr)); hipMalloc(&dout, n * sizeof(Fr));
        hipMalloc(&dbad, 8); hipMemset(dbad, 0, 8);
        hipMemcpy(da, ha.data(), n * sizeof(Fr), hipMemcpyHostToDevice);
        hipMemcpy(db, hb.data(), n * sizeof(Fr), hipMemcpyHostToDevice);
        k_check<FrP><<<n / 256, 256>>>(da, db, n, dbad, dout);
        unsigned bads[2] = {0, 0}; hipMemcpy(bads, dbad, 8, hipMemcpyDeviceToHost);
        const unsigned bad = bads[0];
        std::vector<Fr> ho(n); hipMemcpy(ho.data(), dout, n * sizeof(Fr), hipMemcpyDeviceToHost);
        unsigned badh = 0;
        for (int i = 0; i < n; i += 97) badh += (mul(ha[i], hb[i]) != ho[i]);
        {
            // Fq: the same limbs are valid Fq residues; add -1 and -2 in Fq for the top of the range
            Fq e[2] = {neg(Fq::one()), neg(from_u64<FqP>(2))};
            hipMemcpy(da + 2, e, sizeof(e), hipMemcpyHostToDevice);
            k_check<FqP><<<n / 256, 256>>>((Fq*)da, (Fq*)db, n, dbad, (Fq*)dout);
            hipMemcpy(da + 2, ha.data() + 2, 2 * sizeof(Fr), hipMemcpyHostToDevice);
        }
        hipMemcpy(bads, dbad, 8, hipMemcpyDeviceToHost);
        printf("{\"device_fips_vs_cios_mismatch\":%u,\"device_vs_host_mismatch\":%u,\"sqr_mismatch\":%u,\"fr_fq_fips_vs_cios_mismatch\":%u}\n",
               bad, badh, bads[1], bads[0]);
    }
    for (int blocks : {256 * 4, 256 * 8, 256 * 16}) {
        run<FrP, 1, false>("Fr", d_in, d_out, blocks, 4096);
        run<FrP, 2, false>("Fr", d_in, d_out, blocks, 2048);
        run<FrP, 4, false>("Fr", d_in, d_out, blocks, 1024);
        run<FqP, 2, false>("Fq", (Fq*)d_in, (Fq*)d_out, blocks, 2048);
        run<FrP, 1, true>("Fr", d_in, d_out, blocks, 4096);
        run<FrP, 2, true>("Fr", d_in, d_out, blocks, 2048);
        run<FrP, 4, true>("Fr", d_in, d_out, blocks, 1024);
        run<FrP, 2, 2>("Fr", d_in, d_out, blocks, 2048);
        run<FqP, 2, 2>("Fq", (Fq*)d_in, (Fq*)d_out, blocks, 2048);
        run_nops<FrP>("Fr", d_in, d_out, blocks, 2048);
        run_sqr<FrP>("Fr", d_in, d_out, blocks, 2048);
        run_sqr<FqP>("Fq", (Fq*)d_in, (Fq*)d_out, blocks, 2048);
    }
    return 0;
}
