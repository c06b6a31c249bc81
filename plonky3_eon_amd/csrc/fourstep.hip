// Four-step NTT middle step for a transform split over ranks (BASELINE configs[4]).
//
// A size-N forward DFT (dft/src/traits.rs:27-61 semantics: X[k] = sum_j x[j] w_N^(jk)) with
// N = N1 N2 is, for x viewed as the N1 x N2 row-major matrix M[i1][i2] = x[N2 i1 + i2]:
//   1. Y = size-N1 DFT of every column of M                   (eon_dft_batch_dev, height N1)
//   2. Z[k1][i2] = Y[k1][i2] * w_N^(i2 k1)                       (this file)
//   3. transpose (the all-to-all between ranks)                 (this file packs, RCCL moves)
//   4. X[k1 + N1 k2] = size-N2 DFT over i2 of Z[k1][.]          (eon_dft_batch_dev, height N2)
// Rank g of G owns the column block i2 in [g C, (g+1) C), C = N2 / G, of M (N1 x C row-major) and
// ends with the column block k1 in [g N1/G, (g+1) N1/G) of the N2 x N1 view of X.
//
// eon_fourstep_twiddle_pack_dev fuses steps 2 and 3's local half: it reads the rank's N1 x C
// block Y and writes send[h][i2][k1'] = Y[h N1/G + k1'][i2] * w_N^((col0 + i2) (h N1/G + k1')),
// so the block for rank h is contiguous (C x N1/G) and all_to_all's concatenation in source-rank
// order is directly the N2 x N1/G row-major input of step 4.  The twiddle is
// w_N^e = lo[e mod 2^a] * hi[e >> a] from two cached power tables (a = ceil(log N / 2)).
#include "context.h"
#include "ntt.h"

using namespace eon;

namespace eon {

constexpr uint32_t FS_TILE = 32;  // 32 x 32 elements per block, staged in LDS
constexpr uint32_t FS_ROWS = 8;   // blockDim = (32, 8)

__global__ void __launch_bounds__(256)
    k_fourstep_twiddle_pack(const Fr* y, uint32_t n1, uint32_t cols, uint64_t col0, uint32_t per,
                            uint32_t log_n, uint32_t lo_bits, const Fr* tw_lo, const Fr* tw_hi,
                            Fr* send) {
    __shared__ uint4 lo[FS_TILE * (FS_TILE + 1)];
    __shared__ uint4 hi[FS_TILE * (FS_TILE + 1)];
    const uint32_t k1_0 = blockIdx.y * FS_TILE, i2_0 = blockIdx.x * FS_TILE;
    const uint32_t tx = threadIdx.x, ty = threadIdx.y;
    const uint64_t mask = (1ull << log_n) - 1;
    const uint32_t lo_mask = (1u << lo_bits) - 1;
    // load rows k1 (coalesced along i2) and twist
    for (uint32_t r = ty; r < FS_TILE; r += FS_ROWS) {
        const uint32_t k1 = k1_0 + r, i2 = i2_0 + tx;
        Fr z = Fr::zero();
        if (k1 < n1 && i2 < cols) {
            z = ld_pinned(y + (uint64_t)k1 * cols + i2);
            const uint64_t e = ((col0 + i2) * (uint64_t)k1) & mask;
            if (e) {
                Fr w = ld_pinned(tw_lo + (e & lo_mask));
                if (e >> lo_bits) w = mul(w, ld_pinned(tw_hi + (e >> lo_bits)));
                z = mul(z, w);
            }
        }
        const uint32_t s = r * (FS_TILE + 1) + tx;
        lo[s] = make_uint4(z.v[0], z.v[1], z.v[2], z.v[3]);
        hi[s] = make_uint4(z.v[4], z.v[5], z.v[6], z.v[7]);
    }
    __syncthreads();
    // store columns i2 (coalesced along k1 within the destination rank's block)
    for (uint32_t r = ty; r < FS_TILE; r += FS_ROWS) {
        const uint32_t i2 = i2_0 + r, k1 = k1_0 + tx;
        if (k1 >= n1 || i2 >= cols) continue;
        const uint32_t s = tx * (FS_TILE + 1) + r;
        const uint4 a = lo[s], b = hi[s];
        Fr z;
        z.v[0] = a.x; z.v[1] = a.y; z.v[2] = a.z; z.v[3] = a.w;
        z.v[4] = b.x; z.v[5] = b.y; z.v[6] = b.z; z.v[7] = b.w;
        const uint32_t h = k1 / per, k1l = k1 - h * per;
        st_vec(send + ((uint64_t)h * cols + i2) * per + k1l, z);
    }
}

Status fourstep_twiddle_pack(eon_ctx* ctx, const Fr* y, uint32_t log_n, uint32_t log_n1, uint64_t col0,
                             uint32_t cols, uint32_t parts, Fr* send) {
    if (log_n > 28 || log_n1 > log_n)
        return Status::err(EON_E_SHAPE, "need log_n1 <= log_n <= Fr::TWO_ADICITY = 28");
    const uint32_t n1 = 1u << log_n1;
    const uint64_t n2 = 1ull << (log_n - log_n1);
    if (parts == 0 || n1 % parts) return Status::err(EON_E_SHAPE, "parts must divide N1");
    if (col0 + cols > n2) return Status::err(EON_E_SHAPE, "column block exceeds N2");
    if (cols == 0) return Status::ok();
    if (!y || !send) return Status::err(EON_E_ARG, "null argument");
    const uint32_t lo_bits = (log_n + 1) / 2, hi_bits = log_n - lo_bits;
    const Fr w = fr_two_adic_generator(log_n);
    Fr w_hi = w;
    for (uint32_t i = 0; i < lo_bits; i++) w_hi = sqr(w_hi);
    const Fr *t_lo = nullptr, *t_hi = nullptr;
    EON_TRY(get_power_table(ctx, lo_bits, w, Fr::one(), false, &t_lo));
    EON_TRY(get_power_table(ctx, hi_bits, w_hi, Fr::one(), false, &t_hi));
    // the bounded table cache may have been flushed while building t_hi: look t_lo up again
    EON_TRY(get_power_table(ctx, lo_bits, w, Fr::one(), false, &t_lo));
    const dim3 grid((cols + FS_TILE - 1) / FS_TILE, (n1 + FS_TILE - 1) / FS_TILE);
    ctx->prof.begin("k_fourstep_twiddle_pack", (uint64_t)n1 * cols * 64, ctx->stream,
                    (uint64_t)n1 * cols * 2);
    hipLaunchKernelGGL(k_fourstep_twiddle_pack, grid, dim3(FS_TILE, FS_ROWS), 0, ctx->stream, y, n1, cols,
                       col0, n1 / parts, log_n, lo_bits, t_lo, t_hi, send);
    ctx->prof.end(ctx->stream);
    EON_HIP(hipGetLastError());
    return Status::ok();
}

}  // namespace eon

extern "C" {

int eon_fourstep_twiddle_pack_dev(eon_ctx* ctx, const eon_fr* y, uint32_t log_n, uint32_t log_n1,
                                  uint64_t col0, uint32_t cols, uint32_t parts, eon_fr* send) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = fourstep_twiddle_pack(ctx, reinterpret_cast<const Fr*>(y), log_n, log_n1, col0, cols, parts,
                                     reinterpret_cast<Fr*>(send));
    if (s.bad()) ctx->last_error = s.msg;
    return s.code;
}

}  // extern "C"
