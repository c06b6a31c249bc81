// Multi-GPU entry points of the C ABI (BASELINE configs[4]): one process per GPU,
// the exchanges through the caller's eon_collective (RCCL over xGMI: eon_rccl_collective_init in
// libeonprove.so, or any host-staged implementation of the same contract).
//
//   eon_fourstep_dft_dev  one forward DFT of N = N1 N2 elements spread over the ranks:
//                         size-N1 column DFTs -> twiddle + pack per destination (fourstep.hip)
//                         -> all_to_all -> size-N2 DFTs [-> all_to_all -> block interleave for
//                         the natural layout].  The reference has no multi-GPU DFT; the result is
//                         dft_batch's (dft/src/traits.rs:61) on the whole column.
//   eon_msm_sharded_dev   one MSM split by contiguous term range: a full Pippenger per rank
//                         (msm.hip), an all-gather of the `world` affine partials, their sum by
//                         EC additions on the device (k_sum_partials, in rank order; RCCL has no
//                         elliptic-curve reduction op), so every rank returns the same bytes.
#include <cstring>
#include <vector>

#include "context.h"
#include "msm.h"

using namespace eon;

namespace eon {

// out[r * row_len + s * blk + j] = in[s][r][j]: the `parts` received (rows x blk) blocks laid side
// by side (block s = columns [s blk, (s+1) blk) of the rows x row_len output)
__global__ void k_interleave_blocks(const uint4* in, uint64_t rows, uint32_t blk, uint32_t parts, uint4* out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // one 16-byte half per thread
    const uint64_t row_halves = (uint64_t)blk * parts * 2;
    if (t >= rows * row_halves) return;
    const uint64_t r = t / row_halves, c = t % row_halves;  // c: half-element column in the output row
    const uint64_t s = c / (2ull * blk), j = c % (2ull * blk);
    out[t] = in[(s * rows + r) * 2ull * blk + j];
}

namespace {

const eon_collective* pick_collective(eon_ctx* ctx, const eon_collective* coll) {
    if (coll && coll->world > 1) return coll;
    if (!coll && ctx->coll.world > 1) return &ctx->coll;
    return nullptr;
}

Status fourstep_dft(eon_ctx* ctx, const Fr* in, Fr* out, uint32_t log_n, int layout, const eon_collective* coll) {
    if (log_n > 28) return Status::err(EON_E_SHAPE, "log_n exceeds Fr::TWO_ADICITY = 28");
    if (layout != EON_FOURSTEP_NATURAL && layout != EON_FOURSTEP_TRANSPOSED)
        return Status::err(EON_E_ARG, "layout must be EON_FOURSTEP_NATURAL or EON_FOURSTEP_TRANSPOSED");
    if (!in || !out) return Status::err(EON_E_ARG, "null pointer");
    const uint32_t world = coll ? coll->world : 1, rank = coll ? coll->rank : 0;
    if (coll && (!coll->all_to_all || rank >= world))
        return Status::err(EON_E_ARG, "the collective has no all_to_all (or rank >= world)");
    const uint32_t log_n1 = (log_n + 1) / 2, log_n2 = log_n - log_n1;
    const uint64_t n1 = 1ull << log_n1, n2 = 1ull << log_n2;
    if (n1 % world || n2 % world) return Status::err(EON_E_SHAPE, "world must divide N1 and N2");
    const uint64_t cols = n2 / world, per = n1 / world, local = n1 * cols;  // local = N / world
    hipStream_t st = ctx->stream;
    EON_HIP(ctx->fs_a.ensure(local * sizeof(Fr)));
    EON_HIP(ctx->fs_b.ensure(local * sizeof(Fr)));
    Fr* a = ctx->fs_a.as<Fr>();
    Fr* b = ctx->fs_b.as<Fr>();
    // 1. size-N1 DFTs of the rank's columns; 2. twiddle + pack per destination rank
    EON_TRY(dft_natural_dev(ctx, in, a, n1, (uint32_t)cols));
    EON_TRY(fourstep_twiddle_pack(ctx, a, log_n, log_n1, (uint64_t)rank * cols, (uint32_t)cols, world, b));
    // 3. the transpose across ranks: block h (cols x per) to rank h
    const Fr* z = b;
    if (coll) {
        if (coll->all_to_all(coll->user, b, a, cols * per * sizeof(Fr), st) != 0)
            return Status::err(EON_E_DEVICE, "collective all_to_all failed (four-step transpose)");
        z = a;
    }
    // 4. size-N2 DFTs over i2: the N2 x per block of the N2 x N1 view of X
    // (one rank: the N2 x N1 view of X row-major is X in natural order -- both layouts are `out`)
    Fr* t = (layout == EON_FOURSTEP_TRANSPOSED || !coll) ? out : (z == a ? b : a);
    EON_TRY(dft_natural_dev(ctx, z, t, n2, (uint32_t)per));
    if (t == out) return Status::ok();
    // 5. natural slice X[rank N/G, (rank+1) N/G) = rows k2 in [rank C2, (rank+1) C2) of the N2 x N1
    //    view: rank h's rows are contiguous in t, so a second all_to_all brings every rank's
    //    (C2 x per) block of this rank's rows, laid side by side by the interleave
    const uint64_t c2 = n2 / world;
    Fr* recv = t == a ? b : a;
    if (coll->all_to_all(coll->user, t, recv, c2 * per * sizeof(Fr), st) != 0)
        return Status::err(EON_E_DEVICE, "collective all_to_all failed (natural-order exchange)");
    const uint64_t halves = local * 2;
    hipLaunchKernelGGL(k_interleave_blocks, dim3((unsigned)((halves + 255) / 256)), dim3(256), 0, st,
                       reinterpret_cast<const uint4*>(recv), c2, (uint32_t)per, world, reinterpret_cast<uint4*>(out));
    EON_HIP(hipGetLastError());
    return Status::ok();
}

eon_g1_affine to_abi(const G1Affine& a) {
    eon_g1_affine r;
    for (int i = 0; i < 4; i++) {
        r.x[i] = (uint64_t)a.x.v[2 * i] | (uint64_t)a.x.v[2 * i + 1] << 32;
        r.y[i] = (uint64_t)a.y.v[2 * i] | (uint64_t)a.y.v[2 * i + 1] << 32;
    }
    return r;
}

// out = sum of the n affine partials (ABI layout = G1Affine), in index order
__global__ void k_sum_partials(const G1Affine* parts, uint32_t n, G1Affine* out) {
    if (threadIdx.x != 0) return;
    G1Xyzz acc = xyzz_inf();
    for (uint32_t g = 0; g < n; g++) acc = xyzz_add_affine(acc, ld_affine(parts + g));
    st_affine(out, xyzz_to_affine(acc));
}

Status msm_sharded(eon_ctx* ctx, const eon_msm_bases* bases, const Fr* scalars, uint64_t n_local,
                   const eon_collective* coll, eon_g1_affine* out) {
    G1Affine part;
    EON_TRY(msm_run(ctx, bases, scalars, n_local, &part));
    if (!coll) {
        *out = to_abi(part);
        return Status::ok();
    }
    const uint32_t world = coll->world;
    // context-owned (reused across calls); every exit drains the stream first, so neither the
    // host-side `pa` nor a later reuse of the buffers can race work still queued on it
    DevBuf& send = ctx->shard_send;
    DevBuf& recv = ctx->shard_recv;
    struct Drain {
        hipStream_t s;
        ~Drain() { (void)hipStreamSynchronize(s); }
    } drain{ctx->stream};
    EON_HIP(send.ensure(sizeof(eon_g1_affine)));
    EON_HIP(recv.ensure(world * sizeof(eon_g1_affine)));
    const eon_g1_affine pa = to_abi(part);
    EON_HIP(hipMemcpyAsync(send.p, &pa, sizeof pa, hipMemcpyHostToDevice, ctx->stream));
    if (coll->all_gather(coll->user, send.p, recv.p, sizeof(eon_g1_affine), ctx->stream) != 0)
        return Status::err(EON_E_DEVICE, "collective all_gather failed (MSM partials)");
    // the partials summed on device in rank order (EC additions: not an RCCL reduction op), the
    // same on every rank, so every rank ends with identical bytes
    hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(64), 0, ctx->stream, recv.as<G1Affine>(), world,
                       send.as<G1Affine>());
    EON_HIP(hipGetLastError());
    G1Affine r;
    EON_HIP(hipMemcpyAsync(&r, send.p, sizeof r, hipMemcpyDeviceToHost, ctx->stream));
    EON_HIP(hipStreamSynchronize(ctx->stream));
    *out = to_abi(r);
    return Status::ok();
}

}  // namespace
}  // namespace eon

extern "C" {

int eon_fourstep_dft_dev(eon_ctx* ctx, const eon_fr* in, eon_fr* out, uint32_t log_n, int layout,
                         const eon_collective* coll) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = fourstep_dft(ctx, reinterpret_cast<const Fr*>(in), reinterpret_cast<Fr*>(out), log_n, layout,
                            pick_collective(ctx, coll));
    if (s.bad()) ctx->last_error = s.msg;
    return s.code;
}

int eon_msm_sharded_dev(eon_ctx* ctx, const eon_msm_bases* bases, const eon_fr* scalars, uint64_t n_local,
                        const eon_collective* coll, eon_g1_affine* out) {
    if (!ctx) return EON_E_ARG;
    if (!bases || !out || (n_local && !scalars)) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = msm_sharded(ctx, bases, reinterpret_cast<const Fr*>(scalars), n_local, pick_collective(ctx, coll),
                           out);
    if (s.bad()) ctx->last_error = s.msg;
    return s.code;
}

}  // extern "C"
