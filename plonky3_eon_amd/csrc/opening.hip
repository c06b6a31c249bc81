// KZG opening bases.  KzgPcs::open commits, per (matrix, point z, column f), the synthetic-division
// quotient of f by (X - z) (kzg/src/pcs.rs:305-316, quotient_and_eval kzg/src/util.rs:100-111):
//   W = sum_{i<n-1} q_i G_i,   q_i = sum_{j>i} c_j z^(j-1-i).
// Re-associated over the coefficients c_j of f itself:
//   W = sum_{j<n} c_j H_j(z),  H_j(z) = sum_{i<j} z^(j-1-i) G_i   (H_0 = identity),
// so the witness is an MSM of the very scalars the commitment used, against bases that depend on
// z only: the digit pairs sorted for the commitment (eon_msm_g1_columns_prepare_dev) serve every
// opening point, and the per-column quotient never exists.  The bases, for z != 0:
//   P_i = z^-i G_i  (i < n-1),   S_j = sum_{i<j} P_i  (exclusive prefix sum),   H_j = z^(j-1) S_j;
// for z = 0 the quotient is the coefficient shift q_i = c_(i+1), i.e. H_j = G_(j-1).
// Cost per point: 2 variable-base scalar multiplications (double-and-add, ~3.6k Fq products) and
// two additions of the scan, then the fixed-base window table of the SRS layout (msm.hip).
#include "context.h"
#include "ec.h"
#include "msm.h"

using namespace eon;

namespace {

constexpr uint32_t SCAN = 16;  // points summed per thread at each level of the prefix sum

// k * G for an affine G and a canonical 254-bit k (double-and-add, MSB first)
__device__ G1Xyzz smul_affine(const G1Affine& g, const Fr& k) {
    G1Xyzz acc = xyzz_inf();
    if (is_inf(g)) return acc;
    for (int w = 7; w >= 0; w--) {
        const uint32_t word = k.v[w];
        for (int bit = 31; bit >= 0; bit--) {
            acc = xyzz_dbl(acc);
            if ((word >> bit) & 1) acc = xyzz_add_affine(acc, g);
        }
    }
    return acc;
}

// out[i] = z^-i G_i for i < n - 1; out[n - 1] = identity (the scan's unused last term)
__global__ void k_open_scale(const G1Affine* g, uint64_t n, Fr zinv, G1Xyzz* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (i + 1 == n) {
        st_xyzz(out + i, xyzz_inf());
        return;
    }
    const Fr k = to_canonical(pow_u64(zinv, i));
    st_xyzz(out + i, smul_affine(ld_affine(g + i), k));
}

// tot[t] = sum of a[SCAN t .. SCAN t + SCAN)
__global__ void k_scan_totals(const G1Xyzz* a, uint64_t len, G1Xyzz* tot) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t i0 = t * SCAN;
    if (i0 >= len) return;
    const uint64_t i1 = i0 + SCAN < len ? i0 + SCAN : len;
    G1Xyzz acc = ld_xyzz(a + i0);
    for (uint64_t i = i0 + 1; i < i1; i++) acc = xyzz_add(acc, ld_xyzz(a + i));
    st_xyzz(tot + t, acc);
}

// a <- exclusive prefix sums, chunk t starting from carry[t] (the exclusive prefix of the totals)
__global__ void k_scan_apply(G1Xyzz* a, uint64_t len, const G1Xyzz* carry) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t i0 = t * SCAN;
    if (i0 >= len) return;
    const uint64_t i1 = i0 + SCAN < len ? i0 + SCAN : len;
    G1Xyzz acc = ld_xyzz(carry + t);
    for (uint64_t i = i0; i < i1; i++) {
        const G1Xyzz v = ld_xyzz(a + i);
        st_xyzz(a + i, acc);
        acc = xyzz_add(acc, v);
    }
}

// exclusive prefix sums of a short array, one thread
__global__ void k_scan_serial(G1Xyzz* a, uint64_t len) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    G1Xyzz acc = xyzz_inf();
    for (uint64_t i = 0; i < len; i++) {
        const G1Xyzz v = ld_xyzz(a + i);
        st_xyzz(a + i, acc);
        acc = xyzz_add(acc, v);
    }
}

// h[j] = z^(j-1) S_j for 0 < j < n, h[0] = identity
__global__ void k_open_finish(const G1Affine* s, uint64_t n, Fr z, G1Xyzz* h) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    if (j == 0) {
        st_xyzz(h, xyzz_inf());
        return;
    }
    const Fr k = to_canonical(pow_u64(z, j - 1));
    st_xyzz(h + j, smul_affine(ld_affine(s + j), k));
}

// z = 0: h[j] = G_(j-1), h[0] = identity
__global__ void k_open_shift(const G1Affine* g, uint64_t n, G1Affine* h) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    G1Affine r;
    if (j == 0) {
        r.x = Fq::zero();
        r.y = Fq::zero();
    } else {
        r = ld_affine(g + j - 1);
    }
    st_affine(h + j, r);
}

unsigned grid_for(uint64_t threads, uint32_t block) { return (unsigned)((threads + block - 1) / block); }

// exclusive prefix sum of a[0..len) in place; tmp holds >= len / SCAN + len / SCAN^2 + ... points
void scan_exclusive(G1Xyzz* a, uint64_t len, G1Xyzz* tmp, hipStream_t st) {
    if (len <= SCAN) {
        hipLaunchKernelGGL(k_scan_serial, dim3(1), dim3(1), 0, st, a, len);
        return;
    }
    const uint64_t nt = (len + SCAN - 1) / SCAN;
    hipLaunchKernelGGL(k_scan_totals, dim3(grid_for(nt, 64)), dim3(64), 0, st, a, len, tmp);
    scan_exclusive(tmp, nt, tmp + nt, st);
    hipLaunchKernelGGL(k_scan_apply, dim3(grid_for(nt, 64)), dim3(64), 0, st, a, len, tmp);
}

// one point's scratch, alive until its stream is synchronised
struct Scratch {
    DevBuf h_aff, pts, tmp, aff, table_tmp;
    void release() {
        for (DevBuf* b : {&h_aff, &pts, &tmp, &aff, &table_tmp}) b->release();
    }
};

// enqueue the bases of point z on st (no host sync)
Status opening_bases_async(eon_ctx* ctx, const eon_msm_bases* srs, uint64_t n, const Fr& z, hipStream_t st,
                           Scratch& sc, eon_msm_bases** out) {
    const G1Affine* g = bases_points(srs);
    EON_HIP(sc.h_aff.ensure(n * sizeof(G1Affine)));
    if (z.is_zero()) {
        hipLaunchKernelGGL(k_open_shift, dim3(grid_for(n, 256)), dim3(256), 0, st, g, n, sc.h_aff.as<G1Affine>());
        EON_HIP(hipGetLastError());
    } else {
        EON_HIP(sc.pts.ensure(n * sizeof(G1Xyzz)));
        EON_HIP(sc.tmp.ensure((n / (SCAN - 1) + 64) * sizeof(G1Xyzz)));
        EON_HIP(sc.aff.ensure(n * sizeof(G1Affine)));
        // algorithmic cost: 2 scalar multiplications per point, ~254 dbl (6M+3S) + ~127 madd (8M+2S)
        ctx->prof.begin("k_open_scale", n * (64ull + 128ull), st, n * 3556ull);
        hipLaunchKernelGGL(k_open_scale, dim3(grid_for(n, 64)), dim3(64), 0, st, g, n, inverse(z),
                           sc.pts.as<G1Xyzz>());
        ctx->prof.end(st);
        scan_exclusive(sc.pts.as<G1Xyzz>(), n, sc.tmp.as<G1Xyzz>(), st);
        EON_HIP(launch_batch_to_affine(sc.pts.as<G1Xyzz>(), n, sc.aff.as<G1Affine>(), st));
        ctx->prof.begin("k_open_finish", n * (64ull + 128ull), st, n * 3556ull);
        hipLaunchKernelGGL(k_open_finish, dim3(grid_for(n, 64)), dim3(64), 0, st, sc.aff.as<G1Affine>(), n, z,
                           sc.pts.as<G1Xyzz>());
        ctx->prof.end(st);
        EON_HIP(launch_batch_to_affine(sc.pts.as<G1Xyzz>(), n, sc.h_aff.as<G1Affine>(), st));
        EON_HIP(hipGetLastError());
    }
    // same window layout as the SRS, so scalars prepared against the SRS serve these bases
    return bases_create(ctx, reinterpret_cast<const eon_g1_affine*>(sc.h_aff.as<G1Affine>()), n,
                        bases_precomputed(srs) ? EON_MSM_PRECOMPUTE : 0u, true, out, bases_window(srs), st,
                        &sc.table_tmp);
}

// every point's bases at once: point t's whole pipeline on stream t % 3 (the latency-bound
// scalar multiplications of different points overlap)
Status opening_bases_many(eon_ctx* ctx, const eon_msm_bases* srs, uint64_t n, const eon_fr* points,
                          uint32_t npoints, eon_msm_bases** outs) {
    if (!srs || (npoints && (!points || !outs))) return Status::err(EON_E_ARG, "null argument");
    if (n == 0) return Status::err(EON_E_SHAPE, "opening bases need n >= 1");
    if (n - 1 > eon_msm_bases_len(srs)) return Status::err(EON_E_SHAPE, "more opening bases than SRS points");
    std::vector<Fr> zs(npoints);
    for (uint32_t t = 0; t < npoints; t++) {
        zs[t] = fr_from_abi(points + t);
        if (!fr_is_canonical(zs[t])) return Status::err(EON_E_ARG, "point is not a canonical Fr");
        outs[t] = nullptr;
    }
    hipStream_t streams[3] = {ctx->stream, ctx->msm_side, ctx->msm_side2};
    EON_HIP(hipEventRecord(ctx->msm_ev[0], ctx->stream));
    EON_HIP(hipStreamWaitEvent(ctx->msm_side, ctx->msm_ev[0], 0));
    EON_HIP(hipStreamWaitEvent(ctx->msm_side2, ctx->msm_ev[0], 0));
    std::vector<Scratch> sc(npoints);
    Status s = Status::ok();
    for (uint32_t t = 0; t < npoints && !s.bad(); t++)
        s = opening_bases_async(ctx, srs, n, zs[t], streams[t % 3], sc[t], outs + t);
    for (hipStream_t st : streams) (void)hipStreamSynchronize(st);
    for (auto& x : sc) x.release();
    if (s.bad())
        for (uint32_t t = 0; t < npoints; t++)
            if (outs[t]) {
                bases_free(outs[t]);
                outs[t] = nullptr;
            }
    return s;
}

}  // namespace

extern "C" {

int eon_kzg_opening_bases_create(eon_ctx* ctx, const eon_msm_bases* srs, uint64_t n, const eon_fr* point,
                                 eon_msm_bases** out) {
    if (!ctx) return EON_E_ARG;
    if (!point || !out) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = opening_bases_many(ctx, srs, n, point, 1, out);
    if (s.bad()) ctx->last_error = s.msg;
    return s.code;
}

int eon_kzg_opening_bases_create_many(eon_ctx* ctx, const eon_msm_bases* srs, uint64_t n, const eon_fr* points,
                                      uint32_t npoints, eon_msm_bases** outs) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = opening_bases_many(ctx, srs, n, points, npoints, outs);
    if (s.bad()) ctx->last_error = s.msg;
    return s.code;
}

}  // extern "C"
