// Diagnostic: the shader clock the chip holds under this VALU load, and the radix-2^29 product
// rate at that clock, measured live on the box that runs the bench (MI355X_MICROARCH.md, "DVFS
// give-back" item 6: the in-kernel clock is delta s_memtime / delta s_memrealtime x 100 MHz,
// stamped around the loop on random data; sysfs pp_dpm_sclk is not that clock).  Not on any
// product path: bench.py calls it after its timed region, so the bench line can say at what clock
// its numbers were taken and compare the piece sums against the product peak of the same box.
//
// The loop is the roofline denominator's own benchmark (tools/ubench_r29.hip: mul29<Fq>, two
// independent chains per thread, 256-thread blocks, 4096 blocks) with both timestamps taken by
// wave 0 of every block around its chain; the result is the median over blocks.
#include <algorithm>
#include <vector>

#include "context.h"
#include "field29.h"

namespace {

using namespace eon;

constexpr uint32_t PROBE_THREADS = 256, PROBE_BLOCKS = 4096;

__global__ void __launch_bounds__(PROBE_THREADS) k_clock_probe(uint32_t iters, uint32_t seed, uint64_t* stamps,
                                                               uint32_t* sink) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t s = (tid ^ seed) * 2654435761u + 0x9e3779b9u;
    auto rnd = [&]() {
        s = s * 1664525u + 1013904223u;
        return s;
    };
    F29 x0, x1, y;  // random values below 2^248 < p, normalised limbs
#pragma unroll
    for (int i = 0; i < 9; i++) {
        const uint32_t m = i == 8 ? 0xffffu : M29;
        x0.l[i] = rnd() & m;
        x1.l[i] = rnd() & m;
        y.l[i] = rnd() & m;
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t it = 0; it < iters; it++) {
        x0 = mul29<FqP>(x0, y);
        x1 = mul29<FqP>(x1, y);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
    uint32_t h = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) h ^= x0.l[i] ^ x1.l[i];
    if (h == 0x5bd1e995u) sink[0] = tid;  // keeps both chains live
}

// The whole-product asm statements (prod_asm.h) against the column-block products of field29.h,
// bit for bit, on n pseudo-random operands per kind at their contracts' limb bounds (mul29 /
// sqr29: limbs < 2^30; mul29_sum2: a, c, d < 2^29, b < 2^31) -- every other thread's limbs all at
// the bound's maximum, the worst column sums.  mism[k] counts the mismatching threads of kind k
// (0 mul, 1 sqr, 2 sum2).
__global__ void __launch_bounds__(256) k_prod_asm_check(uint32_t n, uint32_t seed, uint32_t* mism) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    uint32_t s = (t ^ seed) * 2654435761u + 0x9e3779b9u;
    auto rnd = [&](uint32_t bits) {
        s ^= s << 13;
        s ^= s >> 17;
        s ^= s << 5;
        const uint32_t m = (1u << bits) - 1;
        return (t & 1) ? m : (s * 2654435761u) & m;
    };
    F29 a, b, c, d;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        a.l[i] = rnd(30);
        b.l[i] = rnd(30);
    }
    const F29 m1 = mul29<FqP>(a, b), m2 = mul29_asm<FqP>(a, b);
    const F29 q1 = sqr29<FqP>(a), q2 = sqr29_asm<FqP>(a);
#pragma unroll
    for (int i = 0; i < 9; i++) {
        a.l[i] = rnd(29);
        b.l[i] = rnd(31);
        c.l[i] = rnd(29);
        d.l[i] = rnd(29);
    }
    const F29 s1 = mul29_sum2<FqP>(a, b, c, d), s2 = mul29_sum2_asm<FqP>(a, b, c, d);
    uint32_t e0 = 0, e1 = 0, e2 = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        e0 |= m1.l[i] ^ m2.l[i];
        e1 |= q1.l[i] ^ q2.l[i];
        e2 |= s1.l[i] ^ s2.l[i];
    }
    if (e0) atomicAdd(mism + 0, 1u);
    if (e1) atomicAdd(mism + 1, 1u);
    if (e2) atomicAdd(mism + 2, 1u);
}

int finish(eon_ctx* ctx, const Status& s) {
    if (s.bad()) ctx->last_error = s.msg;
    return s.code;
}

}  // namespace

extern "C" int eon_diag_clock_probe(eon_ctx* ctx, uint32_t launches, uint32_t iters, eon_clock_probe* out) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = [&]() -> Status {
        if (!out) return Status::err(EON_E_ARG, "null argument");
        if (launches == 0 || launches > 100000 || iters == 0 || iters > (1u << 24))
            return Status::err(EON_E_ARG, "1 <= launches <= 1e5, 1 <= iters <= 2^24");
        DevBuf stamps, sink;
        PoolScope ps(ctx->pool, ctx->stream);
        EON_HIP(ps.take(stamps, (size_t)PROBE_BLOCKS * 2 * sizeof(uint64_t)));
        EON_HIP(ps.take(sink, 64));
        // the guard exists before either event is created, and destroys only those that were
        struct Ev {
            hipEvent_t a = nullptr, b = nullptr;
            ~Ev() {
                if (a) (void)hipEventDestroy(a);
                if (b) (void)hipEventDestroy(b);
            }
        } ev;
        EON_HIP(hipEventCreate(&ev.a));
        EON_HIP(hipEventCreate(&ev.b));
        hipEvent_t a = ev.a, b = ev.b;
        // one untimed launch, then `launches` back to back (the clock settles under the load)
        hipLaunchKernelGGL(k_clock_probe, dim3(PROBE_BLOCKS), dim3(PROBE_THREADS), 0, ctx->stream, iters, 0u,
                           stamps.as<uint64_t>(), sink.as<uint32_t>());
        EON_HIP(hipGetLastError());
        EON_HIP(hipEventRecord(a, ctx->stream));
        for (uint32_t k = 0; k < launches; k++)
            hipLaunchKernelGGL(k_clock_probe, dim3(PROBE_BLOCKS), dim3(PROBE_THREADS), 0, ctx->stream, iters, k + 1,
                               stamps.as<uint64_t>(), sink.as<uint32_t>());
        EON_HIP(hipGetLastError());
        EON_HIP(hipEventRecord(b, ctx->stream));
        std::vector<uint64_t> h((size_t)PROBE_BLOCKS * 2);
        EON_HIP(hipMemcpyAsync(h.data(), stamps.p, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, ctx->stream));
        EON_HIP(hipStreamSynchronize(ctx->stream));
        float ms = 0;
        EON_HIP(hipEventElapsedTime(&ms, a, b));
        std::vector<double> mhz;
        mhz.reserve(PROBE_BLOCKS);
        for (uint32_t i = 0; i < PROBE_BLOCKS; i++)
            if (h[2 * i + 1]) mhz.push_back((double)h[2 * i] / (double)h[2 * i + 1] * 100.0);
        if (mhz.empty()) return Status::err(EON_E_DEVICE, "no clock stamps");
        std::sort(mhz.begin(), mhz.end());
        out->clock_mhz_median = mhz[mhz.size() / 2];
        out->clock_mhz_min = mhz.front();
        out->clock_mhz_max = mhz.back();
        out->ms_per_launch = ms / launches;
        out->products_per_s = (double)PROBE_BLOCKS * PROBE_THREADS * 2.0 * iters * launches / (ms * 1e-3);
        return Status::ok();
    }();
    return finish(ctx, s);
}

extern "C" int eon_diag_prod_asm_check(eon_ctx* ctx, uint32_t n, uint32_t seed, uint32_t mismatches[3]) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = [&]() -> Status {
        if (!mismatches) return Status::err(EON_E_ARG, "null argument");
        DevBuf cnt;
        PoolScope ps(ctx->pool, ctx->stream);
        EON_HIP(ps.take(cnt, 64));
        EON_HIP(hipMemsetAsync(cnt.p, 0, 16, ctx->stream));
        if (n) hipLaunchKernelGGL(k_prod_asm_check, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, n, seed,
                                  cnt.as<uint32_t>());
        EON_HIP(hipGetLastError());
        EON_HIP(hipMemcpyAsync(mismatches, cnt.p, 12, hipMemcpyDeviceToHost, ctx->stream));
        EON_HIP(hipStreamSynchronize(ctx->stream));
        return Status::ok();
    }();
    return finish(ctx, s);
}
