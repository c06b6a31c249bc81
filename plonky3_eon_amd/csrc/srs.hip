// Test-SRS generation on device: init_srs_unsafe's g1_powers[i] = alpha^i * G
// (kzg/src/params.rs:123-139).  Setup cost, not prove time; it lets
// the MSM benchmark and tests build 2^20+ bases without a host scalar-multiplication loop.
#include "context.h"
#include "ec.h"
#include "msm.h"

using namespace eon;

namespace {

constexpr uint32_t CHUNK = 4;  // consecutive exponents per thread

__global__ void k_srs_points(uint64_t n, Fr alpha, G1Xyzz* out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t i0 = t * CHUNK;
    if (i0 >= n) return;
    // alpha^i0 by square-and-multiply, then consecutive powers
    Fr s = Fr::one(), b = alpha;
    for (uint64_t e = i0; e; e >>= 1) {
        if (e & 1) s = mul(s, b);
        b = sqr(b);
    }
    G1Affine g;
    g.x = from_u64<FqP>(1);
    g.y = from_u64<FqP>(2);
    const uint64_t i1 = i0 + CHUNK < n ? i0 + CHUNK : n;
    for (uint64_t i = i0; i < i1; i++) {
        const Fr k = to_canonical(s);
        G1Xyzz acc = xyzz_inf();
        for (int w = 7; w >= 0; w--)
            for (int bit = 31; bit >= 0; bit--) {
                acc = xyzz_dbl(acc);
                if ((k.v[w] >> bit) & 1) acc = xyzz_add_affine(acc, g);
            }
        out[i] = acc;
        s = mul(s, alpha);
    }
}

Status srs_dev(eon_ctx* ctx, const eon_fr* alpha, uint64_t n, G1Affine* out) {
    if (!alpha) return Status::err(EON_E_ARG, "null alpha");
    if (n == 0) return Status::ok();
    const Fr a = fr_from_abi(alpha);
    if (!fr_is_canonical(a)) return Status::err(EON_E_ARG, "alpha is not a canonical Fr");
    DevBuf tmp;
    EON_HIP(tmp.ensure(n * sizeof(G1Xyzz)));
    const uint64_t threads = (n + CHUNK - 1) / CHUNK;
    hipLaunchKernelGGL(k_srs_points, dim3((unsigned)((threads + 127) / 128)), dim3(128), 0,
                       ctx->stream, n, a, tmp.as<G1Xyzz>());
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = launch_batch_to_affine(tmp.as<G1Xyzz>(), n, out, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    tmp.release();
    EON_HIP(e);
    return Status::ok();
}

}  // namespace

extern "C" {

int eon_g1_srs_powers_dev(eon_ctx* ctx, const eon_fr* alpha, uint64_t n, eon_g1_affine* out) {
    if (!ctx) return EON_E_ARG;
    if (n && !out) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = srs_dev(ctx, alpha, n, reinterpret_cast<G1Affine*>(out));
    if (s.bad()) ctx->last_error = s.msg;
    return s.code;
}

int eon_g1_srs_powers(eon_ctx* ctx, const eon_fr* alpha, uint64_t n, eon_g1_affine* out) {
    if (!ctx) return EON_E_ARG;
    if (n && !out) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = [&]() -> Status {
        EON_HIP(ctx->stage_out.ensure((n ? n : 1) * sizeof(G1Affine)));
        EON_TRY(srs_dev(ctx, alpha, n, ctx->stage_out.as<G1Affine>()));
        if (n)
            EON_HIP(hipMemcpy(out, ctx->stage_out.p, n * sizeof(G1Affine), hipMemcpyDeviceToHost));
        return Status::ok();
    }();
    if (s.bad()) ctx->last_error = s.msg;
    return s.code;
}

}  // extern "C"
