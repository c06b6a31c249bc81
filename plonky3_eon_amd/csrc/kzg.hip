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
#include "field29.h"
#include "ntt.h"

#include <algorithm>

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

// ---- values only, several points in one pass ------------------------------------------------------
// f(z) = sum_b T_b Z^b with T_b the block totals above and Z = z^BL; the blocks' Horner chain is
// split once more into chunks of CH blocks (P_q = sum over the chunk, then sum_q P_q (Z^CH)^q), so
// no thread walks more than max(BL, CH, n / (BL CH)) steps; one read of the coefficients serves
// every point.
constexpr uint32_t CH = 32;
constexpr uint32_t MAX_PTS = 4;
struct Pts {
    Fr z[MAX_PTS];
};

// the points as Shoup multipliers (plain root z and floor(z 2^261 / p), field29.h mul29_shoup):
// r <- c + z r per coefficient is then 143 multiply-adds with no Montgomery multipliers, the
// running value kept lazy (< 4p) in 29-bit limbs
struct PtsShoup {
    F29 w[MAX_PTS], q[MAX_PTS];
};

__global__ void k_eval_block(const Fr* c, uint64_t n, uint32_t width, PtsShoup zs, uint32_t np, Fr* totals) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nblk = (n + BL - 1) / BL;
    if (t >= nblk * width) return;
    const uint32_t col = (uint32_t)(t % width);
    const uint64_t b = t / width;
    const uint64_t lo = b * BL, hi = lo + BL < n ? lo + BL : n;
    // r[] indexed only by unrolled loops, so it stays in registers (a rolled loop over it kept it in
    // scratch, read and written every coefficient)
    F29 r[MAX_PTS];
#pragma unroll
    for (uint32_t p = 0; p < MAX_PTS; p++) r[p] = unpack29(Fr::zero());
    for (uint64_t i = hi; i-- > lo;) {
        const F29 x = unpack29(ld(c + i * width + col));  // canonical
#pragma unroll
        for (uint32_t p = 0; p < MAX_PTS; p++)
            if (p < np) r[p] = add29_norm(x, mul29_shoup_u<FrP>(r[p], zs.w[p], zs.q[p]));  // < p + 3p; z in SGPRs
    }
#pragma unroll
    for (uint32_t p = 0; p < MAX_PTS; p++)
        if (p < np)
            st(totals + ((uint64_t)p * nblk + b) * width + col, pack29<FrP>(canon29<FrP>(reduce_top29<FrP>(r[p]))));
}

// per (point, chunk of CH blocks, column): P_q = sum_{b in chunk} T_b Z^(b - q CH)
__global__ void k_eval_chunks(const Fr* totals, uint64_t nblk, uint32_t width, Pts zbl, uint32_t np, Fr* part) {
    const uint64_t nq = (nblk + CH - 1) / CH;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)np * nq * width) return;
    const uint32_t col = (uint32_t)(t % width);
    const uint64_t q = (t / width) % nq;
    const uint32_t p = (uint32_t)(t / (width * nq));
    const uint64_t b0 = q * CH, b1 = b0 + CH < nblk ? b0 + CH : nblk;
    Fr acc = Fr::zero();
    for (uint64_t b = b1; b-- > b0;) acc = add(ld(totals + ((uint64_t)p * nblk + b) * width + col), mul(zbl.z[p], acc));
    st(part + ((uint64_t)p * nq + q) * width + col, acc);
}

// per (point, column): f(z) = sum_q P_q (Z^CH)^q
__global__ void k_eval_final(const Fr* part, uint64_t nq, uint32_t width, Pts zch, uint32_t np, Fr* values) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)np * width) return;
    const uint32_t col = (uint32_t)(t % width), p = (uint32_t)(t / width);
    Fr acc = Fr::zero();
    for (uint64_t q = nq; q-- > 0;) acc = add(ld(part + ((uint64_t)p * nq + q) * width + col), mul(zch.z[p], acc));
    st(values + (uint64_t)p * width + col, acc);
}

}  // namespace

extern "C" {

int eon_eval_columns_dev(eon_ctx* ctx, const eon_fr* coeffs, uint64_t rows, uint32_t width, const eon_fr* points,
                         uint32_t npoints, eon_fr* values) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = [&]() -> Status {
        if ((npoints && !points) || (width && npoints && !values)) return Status::err(EON_E_ARG, "null argument");
        if (width == 0 || npoints == 0) return Status::ok();
        if (rows == 0) {  // empty column: (empty quotient, 0) (kzg/src/util.rs:101-103)
            EON_HIP(hipMemsetAsync(values, 0, (size_t)npoints * width * sizeof(Fr), ctx->stream));
            return Status::ok();
        }
        if (!coeffs) return Status::err(EON_E_ARG, "null argument");
        const uint64_t nblk = (rows + BL - 1) / BL, nq = (nblk + CH - 1) / CH;
        EON_HIP(ctx->kzg_tmp.ensure((uint64_t)MAX_PTS * (nblk + nq) * width * sizeof(Fr)));
        Fr* totals = ctx->kzg_tmp.as<Fr>();
        Fr* part = totals + (uint64_t)MAX_PTS * nblk * width;
        const Fr* c = reinterpret_cast<const Fr*>(coeffs);
        for (uint32_t p0 = 0; p0 < npoints; p0 += MAX_PTS) {
            const uint32_t np = std::min<uint32_t>(MAX_PTS, npoints - p0);
            Pts zs{}, zbl{}, zch{};
            PtsShoup zsh{};
            for (uint32_t p = 0; p < np; p++) {
                zs.z[p] = fr_from_abi(points + p0 + p);
                if (!fr_is_canonical(zs.z[p])) return Status::err(EON_E_ARG, "point is not a canonical Fr");
                zbl.z[p] = pow_u64(zs.z[p], BL);
                zch.z[p] = pow_u64(zbl.z[p], CH);
                // z 2^261 mod p (the Montgomery form of 32 z) -> plain z and its Shoup quotient
                shoup_pair29<FrP>(unpack29(ntt_scale_form(zs.z[p])), zsh.w[p], zsh.q[p]);
            }
            ctx->prof.begin("k_eval_block", rows * width * 32ull, ctx->stream);
            hipLaunchKernelGGL(k_eval_block, dim3((unsigned)((nblk * width + 127) / 128)), dim3(128), 0, ctx->stream,
                               c, rows, width, zsh, np, totals);
            ctx->prof.end(ctx->stream);
            hipLaunchKernelGGL(k_eval_chunks, dim3((unsigned)((np * nq * width + 127) / 128)), dim3(128), 0,
                               ctx->stream, totals, nblk, width, zbl, np, part);
            hipLaunchKernelGGL(k_eval_final, dim3((unsigned)((np * width + 63) / 64)), dim3(64), 0, ctx->stream, part,
                               nq, width, zch, np, reinterpret_cast<Fr*>(values) + (uint64_t)p0 * width);
            EON_HIP(hipGetLastError());
        }
        return Status::ok();
    }();
    if (s.bad()) ctx->last_error = s.msg;
    return s.code;
}

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
