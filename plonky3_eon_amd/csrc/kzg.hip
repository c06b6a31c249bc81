// KZG opening on device: quotient_and_eval (kzg/src/util.rs:100-111) for every column of a
// row-major coefficient matrix at one point, as KzgPcs::open does per (matrix, point, column)
// (kzg/src/pcs.rs:297-330).
//
// With r_i = sum_{j >= i} c_j z^(j-i) (so r_i = c_i + z * r_(i+1), r_n = 0): f(z) = r_0 and the
// synthetic-division quotient is q_i = r_(i+1), i < n-1.  The recurrence runs as a blocked scan:
//   k_horner_block   per (block of BL rows, column): local suffix Horner total T_b (carry-in 0)
//   k_horner_carry   per column, over blocks top-down: carry_b = T_(b+1) + z^BL * carry_(b+1)
//   k_horner_apply   per (block, column): the local recurrence again from carry_b, writing q
// Two mulmods per coefficient; threads = (n / BL) x width, adjacent threads = adjacent columns.
#include "context.h"

using namespace eon;

namespace {

constexpr uint32_t BL = 256;  // rows per scan block

__device__ __forceinline__ Fr ld(const Fr* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    const uint4 a = q[0], b = q[1];
    Fr x;
    x.v[0] = a.x; x.v[1] = a.y; x.v[2] = a.z; x.v[3] = a.w;
    x.v[4] = b.x; x.v[5] = b.y; x.v[6] = b.z; x.v[7] = b.w;
    return x;
}

__device__ __forceinline__ void st(Fr* p, const Fr& x) {
    uint4* q = reinterpret_cast<uint4*>(p);
    q[0] = make_uint4(x.v[0], x.v[1], x.v[2], x.v[3]);
    q[1] = make_uint4(x.v[4], x.v[5], x.v[6], x.v[7]);
}

__global__ void k_horner_block(const Fr* c, uint64_t n, uint32_t width, Fr z, Fr* totals) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nblk = (n + BL - 1) / BL;
    if (t >= nblk * width) return;
    const uint32_t col = (uint32_t)(t % width);
    const uint64_t b = t / width;
    const uint64_t lo = b * BL, hi = lo + BL < n ? lo + BL : n;
    Fr r = Fr::zero();
    for (uint64_t i = hi; i-- > lo;) r = add(ld(c + i * width + col), mul(z, r));
    st(totals + b * width + col, r);
}

// carries[b] = r at the first row above block b (0 for the top block)
__global__ void k_horner_carry(const Fr* totals, uint64_t nblk, uint32_t width, Fr z_bl, Fr* carries,
                               Fr* values) {
    const uint32_t col = blockIdx.x * blockDim.x + threadIdx.x;
    if (col >= width) return;
    Fr carry = Fr::zero();
    for (uint64_t b = nblk; b-- > 0;) {
        st(carries + b * width + col, carry);
        // r_(lo_b) = T_b + z^(rows in block b) * carry; every block but the top one is full
        carry = add(ld(totals + b * width + col), mul(z_bl, carry));
    }
    st(values + col, carry);  // r_0 = f(z)
}

__global__ void k_horner_apply(const Fr* c, uint64_t n, uint32_t width, Fr z, const Fr* carries,
                               Fr* q) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nblk = (n + BL - 1) / BL;
    if (t >= nblk * width) return;
    const uint32_t col = (uint32_t)(t % width);
    const uint64_t b = t / width;
    const uint64_t lo = b * BL, hi = lo + BL < n ? lo + BL : n;
    Fr r = ld(carries + b * width + col);
    for (uint64_t i = hi; i-- > lo;) {
        if (i < n - 1) st(q + i * width + col, r);  // q_i = r_(i+1)
        r = add(ld(c + i * width + col), mul(z, r));
    }
}

}  // namespace

extern "C" {

int eon_quotient_and_eval_columns_dev(eon_ctx* ctx, const eon_fr* coeffs, uint64_t rows,
                                      uint32_t width, const eon_fr* point, eon_fr* quotient,
                                      eon_fr* values) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = [&]() -> Status {
        if (!point || (width && !values)) return Status::err(EON_E_ARG, "null argument");
        if (width == 0) return Status::ok();
        if (rows == 0) {  // empty column: (empty quotient, 0) (kzg/src/util.rs:101-103)
            EON_HIP(hipMemsetAsync(values, 0, (size_t)width * sizeof(Fr), ctx->stream));
            return Status::ok();
        }
        if (!coeffs) return Status::err(EON_E_ARG, "null argument");
        const Fr z = fr_from_abi(point);
        if (!fr_is_canonical(z)) return Status::err(EON_E_ARG, "point is not a canonical Fr");
        const uint64_t nblk = (rows + BL - 1) / BL;
        EON_HIP(ctx->kzg_tmp.ensure(2 * nblk * width * sizeof(Fr)));
        Fr* totals = ctx->kzg_tmp.as<Fr>();
        Fr* carries = totals + nblk * width;
        const Fr* c = reinterpret_cast<const Fr*>(coeffs);
        const uint64_t threads = nblk * width;
        const unsigned grid = (unsigned)((threads + 127) / 128);
        ctx->prof.begin("k_horner_block", rows * width * 32ull, ctx->stream);
        hipLaunchKernelGGL(k_horner_block, dim3(grid), dim3(128), 0, ctx->stream, c, rows, width, z, totals);
        ctx->prof.end(ctx->stream);
        hipLaunchKernelGGL(k_horner_carry, dim3((width + 63) / 64), dim3(64), 0, ctx->stream, totals, nblk,
                           width, pow_u64(z, BL), carries, reinterpret_cast<Fr*>(values));
        if (!quotient || rows < 2) return Status::ok();  // values only
        ctx->prof.begin("k_horner_apply", rows * width * 64ull, ctx->stream);
        hipLaunchKernelGGL(k_horner_apply, dim3(grid), dim3(128), 0, ctx->stream, c, rows, width, z, carries,
                           reinterpret_cast<Fr*>(quotient));
        ctx->prof.end(ctx->stream);
        EON_HIP(hipGetLastError());
        return Status::ok();
    }();
    if (s.bad()) ctx->last_error = s.msg;
    return s.code;
}

}  // extern "C"
