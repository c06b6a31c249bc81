// Quotient-domain selectors and the quotient evaluation of the (vectorized) Poseidon2-AIR.
//
//   selectors_on_coset  commit/src/domain.rs:252-292 (trace domain H, shift 1; coset s*K)
//   quotient_values     eon-uni-stark/src/prover.rs:539-709 with ProverConstraintFolder
//                       (folder.rs:81-85): out[i] = (sum_k alpha^(K-1-k) C_k(row_i)) / Z_H(x_i)
//   Poseidon2-AIR       poseidon2-air/src/air.rs:108-288 (WIDTH 3, x^5 with one committed x^3
//                       register, BN254 layers: external mds_light, internal [2,1,1;1,2,1;1,1,3])
//   trace generation    poseidon2-air/src/generation.rs:130-288
//
// The folder's accumulator sum_k alpha^(K-1-k) C_k is evaluated as a Horner chain
// acc = acc * alpha + C_k in constraint order, so no alpha-power table is read.  One thread owns
// one (row, vector lane) pair; the VECTOR_LEN lanes of a row are adjacent threads and are
// combined as sum_v P_v * alpha^(160 * (VL - 1 - v)) through LDS.
#include <cstring>

#include "field29.h"
#include "quotient.h"
#include <vector>

using namespace eon;

struct eon_p2air {
    eon_ctx* ctx = nullptr;
    uint32_t hf = 0, pr = 0, vl = 0;
    DevBuf consts;    // begin (hf*3), partial (pr), end (hf*3)
    DevBuf consts29;  // the same as x 2^261 in 29-bit limbs, < 2p (the quotient fold's operands)
};

namespace eon {

struct P2Args {
    const Fr* begin;
    const Fr* partial;
    const Fr* end;
    const F29* begin29;  // the round constants as the quotient fold uses them (eon_p2air::consts29)
    const F29* partial29;
    const F29* end29;
    uint32_t hf, pr, vl, ncols;  // ncols = columns of one permutation
};

__device__ __forceinline__ Fr ldg(const Fr* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    const uint4 a = q[0], b = q[1];
    Fr x;
    x.v[0] = a.x; x.v[1] = a.y; x.v[2] = a.z; x.v[3] = a.w;
    x.v[4] = b.x; x.v[5] = b.y; x.v[6] = b.z; x.v[7] = b.w;
    return x;
}

__device__ __forceinline__ void stg(Fr* p, const Fr& x) {
    uint4* q = reinterpret_cast<uint4*>(p);
    q[0] = make_uint4(x.v[0], x.v[1], x.v[2], x.v[3]);
    q[1] = make_uint4(x.v[4], x.v[5], x.v[6], x.v[7]);
}

__device__ __forceinline__ void p2_ext(Fr* s) {
    const Fr t = add(add(s[0], s[1]), s[2]);
    s[0] = add(s[0], t);
    s[1] = add(s[1], t);
    s[2] = add(s[2], t);
}

__device__ __forceinline__ void p2_int(Fr* s) {
    const Fr t = add(s[0], add(s[1], s[2]));
    s[0] = add(s[0], t);
    s[1] = add(s[1], t);
    s[2] = add(dbl(s[2]), t);
}

// one permutation per thread: generate_trace_rows_for_perm
__global__ void k_p2_trace(const Fr* inputs, uint64_t n, P2Args a, Fr* trace) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    Fr* c = trace + (j / a.vl) * (uint64_t)a.ncols * a.vl + (j % a.vl) * (uint64_t)a.ncols;
    Fr s[3] = {ldg(inputs + 3 * j), ldg(inputs + 3 * j + 1), ldg(inputs + 3 * j + 2)};
    uint32_t k = 0;
    stg(c + k++, Fr::one());
    for (int i = 0; i < 3; i++) stg(c + k++, s[i]);
    p2_ext(s);
    for (uint32_t half = 0; half < 2; half++) {
        if (half == 1) {
            for (uint32_t r = 0; r < a.pr; r++) {
                s[0] = add(s[0], ldg(a.partial + r));
                const Fr x2 = sqr(s[0]);
                const Fr x3 = mul(x2, s[0]);
                stg(c + k++, x3);
                s[0] = mul(x3, x2);
                stg(c + k++, s[0]);
                p2_int(s);
            }
        }
        const Fr* rc = half == 0 ? a.begin : a.end;
        for (uint32_t r = 0; r < a.hf; r++) {
#pragma unroll
            for (int i = 0; i < 3; i++) {
                s[i] = add(s[i], ldg(rc + 3 * r + i));
                const Fr x2 = sqr(s[i]);
                const Fr x3 = mul(x2, s[i]);
                stg(c + k++, x3);
                s[i] = mul(x3, x2);
            }
            p2_ext(s);
            for (int i = 0; i < 3; i++) stg(c + k++, s[i]);
        }
    }
}

// Horner fold of one permutation's 160 constraints, in air.rs assert order, in radix-2^29
// arithmetic (field29.h: 162-multiply-add carry-free products instead of the radix-2^32 product's
// multiply-adds with carry captures).  Values are held as x 2^261 ("29-Montgomery"): trace cells
// are converted on load (shl5_to261, < 2p), alpha and the round constants arrive converted.  Bounds
// (multiples of p; mul29 takes any a b < 167 p^2 and returns < 2p): loaded values and products
// < 2p; an external layer takes inputs < 2p to outputs < 8p; S-box input s + rc < 9p (or < 11p at
// the partial round after an internal layer); a constraint value x3 - x^3 + 2p, y - post + 2p < 4p
// and s - post + 2p < 10p.  The committed x^3 cells skip the reduction (shl5_raw, < 32p): they only
// enter x3 - x^3 + 2p (< 34p) and x3 x^2 (< 64 p^2).  So acc = acc alpha + C < 36p and acc alpha
// is a < 72 p^2 product.  The internal layer's s1, s2 are reduced (reduce_top29) every round: they
// are never reloaded.  Round constants come pre-converted (P2Args::*29).
__device__ __forceinline__ F29 ld29(const Fr* p) { return shl5_to261<FrP>(ldg(p)); }
__device__ __forceinline__ F29 ld29_raw(const Fr* p) { return shl5_raw<FrP>(ldg(p)); }

// the inner sums carry-free: add29_norm takes one addend with limbs < 2^30
__device__ __forceinline__ void p2_ext29(F29* s) {
    const F29 t = add29_norm(add29_lazy(s[0], s[1]), s[2]);
    s[0] = add29_norm(s[0], t);
    s[1] = add29_norm(s[1], t);
    s[2] = add29_norm(s[2], t);
}

__device__ __forceinline__ void p2_int29(F29* s) {
    const F29 t = add29_norm(s[0], add29_lazy(s[1], s[2]));
    s[0] = add29_norm(s[0], t);
    s[1] = reduce_top29<FrP>(add29_norm(s[1], t));
    s[2] = reduce_top29<FrP>(add29_norm(add29_lazy(s[2], s[2]), t));
}

// two Horner steps at once, acc alpha^2 + c0 alpha + c1, with ONE Montgomery reduction.  c1 is
// added without carry propagation (both normalised: limbs < 2^30), since acc only ever feeds a
// product (the next step, the lane power, inv_vanishing)
// (mul29_sum2: alpha^2, alpha and c0 normalised, acc's limbs < 2^30; acc alpha^2 + c0 alpha
// < 36p 2p + 34p 2p = 140 p^2, inside its 0.99 p 2^261 = 167 p^2)
__device__ __forceinline__ void horner2_29(F29& acc, const F29& alpha, const F29& alpha2,
                                           const F29& c0, const F29& c1) {
    acc = add29_lazy(mul29_sum2_u<FrP>(alpha2, acc, alpha, c0), c1);
}

// The constraints are folded in pairs (every round asserts an even number of them): the same
// acc as one Horner step per constraint, 80 instead of 160 reductions per permutation.
__device__ F29 p2_fold29(const Fr* c, const P2Args& a, const F29& alpha) {
    const F29 alpha2 = uniform29(sqr29<FrP>(alpha));  // alpha, alpha^2 in SGPRs
    F29 acc;
#pragma unroll
    for (int i = 0; i < 9; i++) acc.l[i] = 0;
    F29 s[3] = {ld29(c + 1), ld29(c + 2), ld29(c + 3)};
    uint32_t k = 4;
    p2_ext29(s);
    for (uint32_t half = 0; half < 2; half++) {
        if (half == 1) {
            for (uint32_t r = 0; r < a.pr; r++) {
                const F29 x = add29_lazy(s[0], a.partial29[r]);  // normalised + normalised: a product input
                const F29 x3 = ld29_raw(c + k), post = ld29(c + k + 1);
                k += 2;
                const F29 x2 = sqr29<FrP>(x);
                horner2_29(acc, alpha, alpha2,
                           sub29<FrP, 2>(x3, mul29<FrP>(x2, x)),            // assert_eq(x3, x2 * x)
                           sub29<FrP, 2>(mul29<FrP>(x3, x2), post));        // assert_eq(state[0], post_sbox)
                s[0] = post;
                p2_int29(s);
            }
        }
        const F29* rc = half == 0 ? a.begin29 : a.end29;
        for (uint32_t r = 0; r < a.hf; r++) {
            F29 cs[3];  // the S-box constraints assert_eq(x3, x2 * x)
#pragma unroll
            for (int i = 0; i < 3; i++) {
                const F29 x = add29_lazy(s[i], rc[3 * r + i]);
                const F29 x3 = ld29_raw(c + k + i);
                const F29 x2 = sqr29<FrP>(x);
                cs[i] = sub29<FrP, 2>(x3, mul29<FrP>(x2, x));
                s[i] = mul29<FrP>(x3, x2);
            }
            horner2_29(acc, alpha, alpha2, cs[0], cs[1]);
            p2_ext29(s);
            F29 cp[3];  // assert_eq(state_i, post_i)
#pragma unroll
            for (int i = 0; i < 3; i++) {
                const F29 post = ld29(c + k + 3 + i);
                cp[i] = sub29<FrP, 2>(s[i], post);
                s[i] = post;
            }
            horner2_29(acc, alpha, alpha2, cs[2], cp[0]);
            horner2_29(acc, alpha, alpha2, cp[1], cp[2]);
            k += 6;
        }
    }
    return acc;
}

constexpr uint32_t MAX_VL = 32;
struct LanePow {
    Fr v[MAX_VL];  // alpha^(K_lane * (vl - 1 - v))
};

// blockDim.x = 256 = (256 / vl) rows x vl lanes
__global__ void __launch_bounds__(256) k_p2_quotient(const Fr* lde, uint64_t q, P2Args a, Fr alpha,
                                                     LanePow lane_pow, const Fr* inv_van,
                                                     uint32_t nr_mask, Fr* out) {
    __shared__ Fr part[256];
    const uint32_t v = threadIdx.x % a.vl;
    const uint64_t row = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / a.vl;
    Fr p = Fr::zero();
    if (row < q) {
        const Fr* c = lde + row * (uint64_t)a.ncols * a.vl + (uint64_t)v * a.ncols;
        F29 acc = p2_fold29(c, a, uniform29(shl5_to261<FrP>(alpha)));
        // the lane's share times its alpha power (29-Montgomery), then times inv_vanishing in the
        // ABI form: mul29 of x 2^261 and y 2^256 is x y 2^256 (prover.rs:699)
        if (a.vl > 1) acc = mul29<FrP>(acc, shl5_to261<FrP>(lane_pow.v[v]));
        const F29 iv = unpack29(ldg(inv_van + (row & nr_mask)));
        p = pack29<FrP>(canon29<FrP>(mul29<FrP>(acc, iv)));
    }
    part[threadIdx.x] = p;
    __syncthreads();
    if (v == 0 && row < q) {
        Fr acc = part[threadIdx.x];
        for (uint32_t u = 1; u < a.vl; u++) acc = add(acc, part[threadIdx.x + u]);
        stg(out + row, acc);
    }
}

constexpr uint32_t MAX_LINCOMB = 64;
struct LincombCoeffs {
    Fr c[MAX_LINCOMB];
};

// out[i] = sum_j c_j * in[j * rows + i]: combines per-shard partial quotients (mod-p sums are not
// an RCCL reduction, so shards all-gather their partials and every rank combines them here).
__global__ void k_fr_lincomb(const Fr* in, uint32_t k, uint64_t rows, LincombCoeffs c, Fr* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows) return;
    Fr acc = mul(ldg(in + i), c.c[0]);
    for (uint32_t j = 1; j < k; j++) acc = add(acc, mul(ldg(in + (uint64_t)j * rows + i), c.c[j]));
    stg(out + i, acc);
}

// Z_H(x_i) = s^n * w_rate^j - 1 and its inverse for j < 2^rate (one thread each)
__global__ void k_vanishing_table(Fr s_pow_n, Fr g_rate, uint32_t nr, Fr* zh, Fr* zh_inv) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nr) return;
    const Fr z = sub(mul(s_pow_n, pow_u64(g_rate, j)), Fr::one());
    zh[j] = z;
    zh_inv[j] = inverse(z);
}

constexpr uint32_t SEL_CHUNK = 32;

// selectors_on_coset: x_i = shift * w_Q^i; two batch inversions per chunk (Montgomery's trick)
__global__ void k_selectors(uint64_t q, Fr shift, Fr g_q, Fr h_inv, const Fr* zh, const Fr* zh_inv,
                            uint32_t nr_mask, Fr* first, Fr* last, Fr* trans, Fr* inv_van) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t i0 = t * SEL_CHUNK;
    if (i0 >= q) return;
    const uint64_t i1 = i0 + SEL_CHUNK < q ? i0 + SEL_CHUNK : q;
    Fr x0 = mul(shift, pow_u64(g_q, i0));
    // pass 1: prefix products of (x - 1) and (x - h^-1)
    Fr pa = Fr::one(), pb = Fr::one(), x = x0;
    for (uint64_t i = i0; i < i1; i++) {
        stg(first + i, pa);  // stash prefixes in the outputs
        stg(last + i, pb);
        pa = mul(pa, sub(x, Fr::one()));
        pb = mul(pb, sub(x, h_inv));
        x = mul(x, g_q);
    }
    Fr ia = inverse(pa), ib = inverse(pb);
    // pass 2 (backwards): x_i = x0 * g^(i - i0), recomputed from the end
    Fr xe = mul(x0, pow_u64(g_q, i1 - 1 - i0));
    const Fr g_inv = inverse(g_q);
    for (uint64_t i = i1; i-- > i0;) {
        const Fr da = sub(xe, Fr::one()), db = sub(xe, h_inv);
        const Fr inv_da = mul(ia, ldg(first + i)), inv_db = mul(ib, ldg(last + i));
        ia = mul(ia, da);
        ib = mul(ib, db);
        const Fr z = ldg(zh + (i & nr_mask));
        stg(first + i, mul(z, inv_da));
        stg(last + i, mul(z, inv_db));
        stg(trans + i, db);
        stg(inv_van + i, ldg(zh_inv + (i & nr_mask)));
        xe = mul(xe, g_inv);
    }
}

Status vanishing_table(eon_ctx* ctx, uint32_t log_n, uint32_t log_q, const Fr& shift, Fr** zh,
                       Fr** zh_inv) {
    const uint32_t rate = log_q - log_n;
    const uint32_t nr = 1u << rate;
    EON_HIP(ctx->sel_tab.ensure(2ull * nr * sizeof(Fr)));
    *zh = ctx->sel_tab.as<Fr>();
    *zh_inv = *zh + nr;
    // the same domains every proof: the table is kept (a single-thread inversion per entry is a
    // ~0.5 ms latency-bound launch otherwise)
    if (ctx->van_valid && ctx->van_log_n == log_n && ctx->van_log_q == log_q &&
        std::memcmp(&ctx->van_shift, &shift, sizeof(Fr)) == 0)
        return Status::ok();
    ctx->van_valid = false;
    Fr s_pow_n = shift;
    for (uint32_t i = 0; i < log_n; i++) s_pow_n = sqr(s_pow_n);
    hipLaunchKernelGGL(k_vanishing_table, dim3((nr + 63) / 64), dim3(64), 0, ctx->stream, s_pow_n,
                       fr_two_adic_generator(rate), nr, *zh, *zh_inv);
    EON_HIP(hipGetLastError());
    ctx->van_valid = true;
    ctx->van_log_n = log_n;
    ctx->van_log_q = log_q;
    ctx->van_shift = shift;
    return Status::ok();
}

Status check_domains(uint32_t log_n, uint32_t log_q) {
    if (log_q < log_n || log_q > 28 || log_q - log_n > 16)
        return Status::err(EON_E_SHAPE, "coset must be at least the trace domain size, <= 2^28");
    return Status::ok();
}

Status selectors_launch(eon_ctx* ctx, uint32_t log_n, uint32_t log_q, const Fr& sh, Fr* o) {
    Fr *zh, *zh_inv;
    EON_TRY(vanishing_table(ctx, log_n, log_q, sh, &zh, &zh_inv));
    const uint64_t q = 1ull << log_q;
    const uint64_t threads = (q + SEL_CHUNK - 1) / SEL_CHUNK;
    hipLaunchKernelGGL(k_selectors, dim3((unsigned)((threads + 63) / 64)), dim3(64), 0, ctx->stream, q, sh,
                       fr_two_adic_generator(log_q), inverse(fr_two_adic_generator(log_n)), zh, zh_inv,
                       (1u << (log_q - log_n)) - 1, o, o + q, o + 2 * q, o + 3 * q);
    EON_HIP(hipGetLastError());
    return Status::ok();
}

}  // namespace eon

namespace {

int finish(eon_ctx* ctx, const Status& s) {
    if (s.bad()) ctx->last_error = s.msg;
    return s.code;
}

P2Args p2_args(const eon_p2air* air) {
    P2Args a;
    const Fr* base = air->consts.as<Fr>();
    a.begin = base;
    a.partial = base + 3 * air->hf;
    a.end = base + 3 * air->hf + air->pr;
    const F29* b29 = air->consts29.as<F29>();
    a.begin29 = b29;
    a.partial29 = b29 + 3 * air->hf;
    a.end29 = b29 + 3 * air->hf + air->pr;
    a.hf = air->hf;
    a.pr = air->pr;
    a.vl = air->vl;
    a.ncols = 1 + 3 + 12 * air->hf + 2 * air->pr;
    return a;
}

}  // namespace

extern "C" {

int eon_selectors_on_coset_dev(eon_ctx* ctx, uint32_t log_n, uint32_t log_q, const eon_fr* shift,
                               eon_fr* out) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = [&]() -> Status {
        if (!shift || !out) return Status::err(EON_E_ARG, "null argument");
        EON_TRY(check_domains(log_n, log_q));
        const Fr sh = fr_from_abi(shift);
        if (!fr_is_canonical(sh)) return Status::err(EON_E_ARG, "shift is not a canonical Fr");
        // selectors_on_coset asserts coset.shift != 1 (domain.rs:254)
        if (sh == Fr::one()) return Status::err(EON_E_ARG, "coset shift must not be ONE");
        return selectors_launch(ctx, log_n, log_q, sh, reinterpret_cast<Fr*>(out));
    }();
    return finish(ctx, s);
}

int eon_p2air_create(eon_ctx* ctx, const eon_poseidon2_constants* k, uint32_t vector_len,
                     eon_p2air** out) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = [&]() -> Status {
        if (!k || !out || !k->beginning || !k->partial || !k->ending)
            return Status::err(EON_E_ARG, "null argument");
        if (vector_len == 0 || vector_len > MAX_VL || (256 % vector_len) != 0)
            return Status::err(EON_E_ARG, "vector_len must be a power of two <= 32");
        const uint32_t hf = k->half_full_rounds, pr = k->partial_rounds;
        const uint64_t n = 6ull * hf + pr;
        std::vector<Fr> host(n);
        for (uint32_t i = 0; i < 3 * hf; i++) host[i] = fr_from_abi(&k->beginning[i]);
        for (uint32_t i = 0; i < pr; i++) host[3 * hf + i] = fr_from_abi(&k->partial[i]);
        for (uint32_t i = 0; i < 3 * hf; i++) host[3 * hf + pr + i] = fr_from_abi(&k->ending[i]);
        for (auto& x : host)
            if (!fr_is_canonical(x)) return Status::err(EON_E_ARG, "round constant not canonical");
        eon_p2air* air = new eon_p2air();
        air->ctx = ctx;
        air->hf = hf;
        air->pr = pr;
        air->vl = vector_len;
        std::vector<F29> host29(n);
        for (uint64_t i = 0; i < n; i++) host29[i] = shl5_to261<FrP>(host[i]);
        hipError_t e = air->consts.ensure((n ? n : 1) * sizeof(Fr));
        if (e == hipSuccess && n) e = hipMemcpy(air->consts.p, host.data(), n * sizeof(Fr), hipMemcpyHostToDevice);
        if (e == hipSuccess) e = air->consts29.ensure((n ? n : 1) * sizeof(F29));
        if (e == hipSuccess && n) e = hipMemcpy(air->consts29.p, host29.data(), n * sizeof(F29), hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            air->consts.release();
            air->consts29.release();
            delete air;
            EON_HIP(e);
        }
        *out = air;
        return Status::ok();
    }();
    return finish(ctx, s);
}

void eon_p2air_destroy(eon_p2air* air) {
    if (!air) return;
    std::lock_guard<std::mutex> lk(air->ctx->mu);
    (void)hipSetDevice(air->ctx->device);
    (void)hipStreamSynchronize(air->ctx->stream);
    air->consts.release();
    air->consts29.release();
    delete air;
}

uint32_t eon_p2air_width(const eon_p2air* air) {
    return air ? (1 + 3 + 12 * air->hf + 2 * air->pr) * air->vl : 0;
}

uint32_t eon_p2air_vector_len(const eon_p2air* air) { return air ? air->vl : 0; }

uint32_t eon_p2air_constraints_per_perm(const eon_p2air* air) {
    return air ? 12 * air->hf + 2 * air->pr : 0;
}

int eon_p2air_generate_trace_dev(eon_ctx* ctx, const eon_p2air* air, const eon_fr* inputs,
                                 uint64_t n_perms, eon_fr* trace) {
    if (!ctx || !air) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = [&]() -> Status {
        if (n_perms == 0) return Status::ok();
        if (!inputs || !trace) return Status::err(EON_E_ARG, "null argument");
        // generate_vectorized_trace_rows asserts n = VECTOR_LEN * 2^k (generation.rs:30-34)
        const uint64_t rows = n_perms / air->vl;
        if (n_perms % air->vl || (rows & (rows - 1)))
            return Status::err(EON_E_SHAPE, "n_perms must be VECTOR_LEN times a power of two");
        hipLaunchKernelGGL(k_p2_trace, dim3((unsigned)((n_perms + 127) / 128)), dim3(128), 0,
                           ctx->stream, reinterpret_cast<const Fr*>(inputs), n_perms, p2_args(air),
                           reinterpret_cast<Fr*>(trace));
        EON_HIP(hipGetLastError());
        return Status::ok();
    }();
    return finish(ctx, s);
}

int eon_p2air_quotient_values_dev(eon_ctx* ctx, const eon_p2air* air, const eon_fr* lde,
                                  uint32_t log_n, uint32_t log_qd, const eon_fr* alpha,
                                  eon_fr* out) {
    if (!ctx || !air) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = [&]() -> Status {
        if (!lde || !alpha || !out) return Status::err(EON_E_ARG, "null argument");
        const uint32_t log_q = log_n + log_qd;
        EON_TRY(check_domains(log_n, log_q));
        const Fr al = fr_from_abi(alpha);
        if (!fr_is_canonical(al)) return Status::err(EON_E_ARG, "alpha is not a canonical Fr");
        // quotient domain = trace domain (shift 1) .create_disjoint_domain: shift GENERATOR
        // (commit/src/domain.rs:155-168)
        Fr *zh, *zh_inv;
        EON_TRY(vanishing_table(ctx, log_n, log_q, from_u64<FrP>(5), &zh, &zh_inv));
        const P2Args a = p2_args(air);
        const uint32_t k_lane = 6 * a.hf * 2 + 2 * a.pr;  // constraints per permutation
        LanePow lp;
        const Fr step = pow_u64(al, k_lane);
        Fr cur = Fr::one();
        for (int v = (int)a.vl - 1; v >= 0; v--) {
            lp.v[v] = cur;
            cur = mul(cur, step);
        }
        const uint64_t q = 1ull << log_q;
        const uint64_t threads = q * a.vl;
        // algorithmic 256-bit products per (row, lane): per partial round x^2, x^2 x, x3 x^2 and two
        // Horner steps; per full-round S-box x^2, x^2 x, x3 x^2 and one Horner step, plus one per
        // post-state constraint; the lane power and inv_vanishing.  (Algorithmic: p2_fold29 folds
        // the Horner steps in pairs, two products sharing one reduction.)
        const uint64_t lane_products = 5ull * a.pr + 2ull * a.hf * 3 * 4 + 2ull * a.hf * 3 + 2;
        ctx->prof.begin("k_p2_quotient", q * (uint64_t)a.ncols * a.vl * 32 + q * 32, ctx->stream,
                        q * a.vl * lane_products);
        hipLaunchKernelGGL(k_p2_quotient, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                           ctx->stream, reinterpret_cast<const Fr*>(lde), q, a, al, lp, zh_inv,
                           (1u << log_qd) - 1,
                           reinterpret_cast<Fr*>(out));
        ctx->prof.end(ctx->stream);
        EON_HIP(hipGetLastError());
        return Status::ok();
    }();
    return finish(ctx, s);
}

int eon_fr_lincomb_dev(eon_ctx* ctx, const eon_fr* in, uint32_t k, uint64_t rows,
                       const eon_fr* coeffs, eon_fr* out) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = [&]() -> Status {
        if (rows == 0) return Status::ok();
        if (!in || !coeffs || !out) return Status::err(EON_E_ARG, "null argument");
        if (k == 0 || k > MAX_LINCOMB) return Status::err(EON_E_SHAPE, "1 <= k <= 64 vectors");
        LincombCoeffs c;
        for (uint32_t j = 0; j < k; j++) {
            c.c[j] = fr_from_abi(&coeffs[j]);
            if (!fr_is_canonical(c.c[j])) return Status::err(EON_E_ARG, "coefficient is not a canonical Fr");
        }
        ctx->prof.begin("k_fr_lincomb", (k + 1) * rows * 32, ctx->stream, (uint64_t)k * rows);
        hipLaunchKernelGGL(k_fr_lincomb, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, ctx->stream,
                           reinterpret_cast<const Fr*>(in), k, rows, c, reinterpret_cast<Fr*>(out));
        ctx->prof.end(ctx->stream);
        EON_HIP(hipGetLastError());
        return Status::ok();
    }();
    return finish(ctx, s);
}

}  // extern "C"
