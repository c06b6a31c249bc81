// Microbenchmark: 256-bit Montgomery product in radix 2^29 (9 limbs, R = 2^261) against the
// radix-2^32 FIPS product of csrc/field.h.  With 29-bit limbs every column sum (at most 18
// products < 2^60 plus the carry) fits one 64-bit accumulator, so the 32x32 multiply-adds need no
// carry capture (the radix-2^32 product spends half its issue slots on v_addc).
//
// Checks: mul29(x, y) * 2^5 == mul_fips(x, y) (mod p) on 2^20 random pairs, including lazy
// inputs (limbs < 2^30, values < 13p).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../plonky3_eon_amd/csrc/field29.h"

using namespace eon;

template <class M, int CH, int V>
__global__ void __launch_bounds__(256) k_mul29(const Fe<M>* in, Fe<M>* out, int iters) {
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    F29 x[CH];
    F29 y = unpack29(in[(tid + 7) & 1023]);
#pragma unroll
    for (int c = 0; c < CH; c++) x[c] = unpack29(in[(tid + c) & 1023]);
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int c = 0; c < CH; c++)
            x[c] =  (V == 1 ? mul29_2acc<M>(x[c], y) : mul29<M>(x[c], y));
    }
    F29 acc = x[0];
#pragma unroll
    for (int c = 1; c < CH; c++) acc = add29_lazy(acc, x[c]);
    out[tid] = pack29<M>(acc);
}

template <class M>
__global__ void __launch_bounds__(256) k_fips(const Fe<M>* in, Fe<M>* out, int iters) {
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    Fe<M> y = in[(tid + 7) & 1023];
    Fe<M> x0 = in[tid & 1023], x1 = in[(tid + 1) & 1023];
    for (int it = 0; it < iters; it++) {
        x0 = mul_fips(x0, y);
        x1 = mul_fips(x1, y);
    }
    out[tid] = add(x0, x1);
}

// subtraction cost: x = sub29<4>(x, y) chains (plus one product per 8 subs to keep values bounded)
template <class M>
__global__ void __launch_bounds__(256) k_sub29(const Fe<M>* in, Fe<M>* out, int iters) {
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    F29 y = unpack29(in[(tid + 7) & 1023]);
    F29 x0 = unpack29(in[tid & 1023]), x1 = unpack29(in[(tid + 1) & 1023]);
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            x0 = sub29<M, 2>(y, x0);
            x1 = sub29<M, 2>(y, x1);
        }
    }
    out[tid] = pack29<M>(add29_lazy(x0, x1));
}

template <class M>
__global__ void k_check(const Fe<M>* a, const Fe<M>* b, int n, unsigned* bad) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    // canonical inputs for either field (the Fq test vectors are squared into [0, p))
    const Fe<M> ai = M::P[7] == FqP::P[7] && M::P[0] == FqP::P[0] ? a[i] : mul_fips(a[i], a[i]);
    const Fe<M> bi = M::P[7] == FqP::P[7] && M::P[0] == FqP::P[0] ? b[i] : mul_fips(b[i], b[i]);
    const Fe<M> want = mul_fips(ai, bi);  // a b 2^-256
    const F29 x = unpack29(ai), y = unpack29(bi);
    // a b 2^-261 (< 2p) -> canonical -> times 2^5
    auto check = [&](const F29& r, int slot) {
        if (!limbs_ok29(r)) atomicAdd(bad + slot, 1u);
        Fe<M> c = pack29<M>(canon29<M>(r));
        for (int k = 0; k < 5; k++) c = add(c, c);
        if (c != want) atomicAdd(bad + slot, 1u);
    };
    check(mul29<M>(x, y), 0);
    check(mul29_2acc<M>(x, y), 1);
    // lazy inputs: x + y (limbs < 2^30), (x + 12p) normalised
    const F29 lx = add29_lazy(x, F29{});  // identity lazy add
    const Fe<M> s = add(ai, bi);
    const Fe<M> want2 = mul_fips(s, bi);
    const F29 r2 = mul29<M>(add29_lazy(x, y), y);
    Fe<M> c2 = pack29<M>(canon29<M>(r2));
    for (int k = 0; k < 5; k++) c2 = add(c2, c2);
    if (c2 != want2) atomicAdd(bad + 2, 1u);
    // sub29: (x - y) * y
    const Fe<M> want3 = mul_fips(sub(ai, bi), bi);
    const F29 r3 = mul29<M>(sub29<M, 2>(x, y), y);
    Fe<M> c3 = pack29<M>(canon29<M>(r3));
    for (int k = 0; k < 5; k++) c3 = add(c3, c3);
    if (c3 != want3) atomicAdd(bad + 3, 1u);
    // 12p-bounded input: x + 12p (value < 13p) times y
    F29 big = add29_norm(x, mulp29<M>(12));
    const F29 r4 = mul29<M>(big, y);
    Fe<M> c4 = pack29<M>(canon29<M>(r4));
    for (int k = 0; k < 5; k++) c4 = add(c4, c4);
    if (c4 != want || !limbs_ok29(lx)) atomicAdd(bad + 4, 1u);
    // sum of two products with one reduction: x y + (x - y + 8p) (2p - y)
    const F29 d = sub29<M, 8>(x, y), e = sub29<M, 2>(F29{}, y);
    const Fe<M> want5 = add(want, mul_fips(sub(ai, bi), neg(bi)));
    Fe<M> c5 = pack29<M>(canon29<M>(mul29_sum2<M>(x, y, d, e)));
    for (int k = 0; k < 5; k++) c5 = add(c5, c5);
    if (c5 != want5) atomicAdd(bad + 5, 1u);
}

template <class M, int CH, int V>
double run(const char* name, Fe<M>* d_in, Fe<M>* d_out, int blocks, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k_mul29<M, CH, V><<<blocks, 256>>>(d_in, d_out, 16);
    hipDeviceSynchronize();
    hipEventRecord(a);
    k_mul29<M, CH, V><<<blocks, 256>>>(d_in, d_out, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double r = (double)blocks * 256 * iters * CH / (ms * 1e-3);
    printf("{\"field\":\"%s\",\"op\":\"mul29\",\"variant\":%d,\"chains\":%d,\"blocks\":%d,\"ms\":%.3f,\"mulmod_per_s\":%.4e}\n",
           name, V, CH, blocks, ms, r);
    return r;
}

template <class M>
void run_fips(const char* name, Fe<M>* d_in, Fe<M>* d_out, int blocks, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k_fips<M><<<blocks, 256>>>(d_in, d_out, 16);
    hipDeviceSynchronize();
    hipEventRecord(a);
    k_fips<M><<<blocks, 256>>>(d_in, d_out, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    printf("{\"field\":\"%s\",\"op\":\"mul_fips\",\"chains\":2,\"blocks\":%d,\"ms\":%.3f,\"mulmod_per_s\":%.4e}\n", name,
           blocks, ms, (double)blocks * 256 * iters * 2 / (ms * 1e-3));
}

template <class M>
void run_sub(const char* name, Fe<M>* d_in, Fe<M>* d_out, int blocks, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k_sub29<M><<<blocks, 256>>>(d_in, d_out, 16);
    hipDeviceSynchronize();
    hipEventRecord(a);
    k_sub29<M><<<blocks, 256>>>(d_in, d_out, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    printf("{\"field\":\"%s\",\"op\":\"sub29\",\"blocks\":%d,\"ms\":%.3f,\"sub_per_s\":%.4e}\n", name, blocks, ms,
           (double)blocks * 256 * iters * 16 / (ms * 1e-3));
}

int main() {
    const int n = 1 << 20;
    std::vector<Fq> ha(n), hb(n);
    uint64_t st = 1;
    auto nx = [&]() {
        st += 0x9e3779b97f4a7c15ull;
        uint64_t z = st;
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        return z ^ (z >> 31);
    };
    for (int i = 0; i < n; i++) {
        ha[i] = mul(from_u64<FqP>(nx()), from_u64<FqP>(nx()));
        hb[i] = mul(from_u64<FqP>(nx()), from_u64<FqP>(nx()));
    }
    ha[0] = Fq::zero();
    ha[1] = neg(Fq::one());
    hb[1] = neg(Fq::one());
    hb[2] = neg(from_u64<FqP>(2));
    ha[3] = hb[3];
    Fq *da, *db, *dout;
    unsigned* dbad;
    hipMalloc(&da, n * sizeof(Fq));
    hipMalloc(&db, n * sizeof(Fq));
    hipMalloc(&dout, (size_t)4096 * 256 * sizeof(Fq));
    hipMalloc(&dbad, 64);
    hipMemset(dbad, 0, 64);
    hipMemcpy(da, ha.data(), n * sizeof(Fq), hipMemcpyHostToDevice);
    hipMemcpy(db, hb.data(), n * sizeof(Fq), hipMemcpyHostToDevice);
    k_check<FqP><<<n / 256, 256>>>(da, db, n, dbad);
    k_check<FrP><<<n / 256, 256>>>((const Fr*)da, (const Fr*)db, n, dbad + 8);
    unsigned bad[16];
    hipMemcpy(bad, dbad, 64, hipMemcpyDeviceToHost);
    printf("{\"fq_mismatch\":[%u,%u,%u,%u,%u,%u],\"fr_mismatch\":[%u,%u,%u,%u,%u,%u]}\n", bad[0], bad[1], bad[2], bad[3], bad[4],
           bad[5], bad[8], bad[9], bad[10], bad[11], bad[12], bad[13]);
    for (int blocks : {256 * 4, 256 * 8, 256 * 16}) {
        run_fips<FqP>("Fq", da, dout, blocks, 2048);
        run<FqP, 1, 0>("Fq", da, dout, blocks, 4096);
        run<FqP, 2, 0>("Fq", da, dout, blocks, 2048);
        run<FqP, 2, 1>("Fq", da, dout, blocks, 2048);
        run<FqP, 4, 0>("Fq", da, dout, blocks, 1024);
        run_sub<FqP>("Fq", da, dout, blocks, 512);
    }
    return 0;
}
