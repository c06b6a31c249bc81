/*
 * eon_oracle.c -- CPU restatement of the reference's hot-path algorithms, in C (OpenMP).
 *
 * TEST INFRASTRUCTURE ONLY: the checker for parity tests and the `cpu_baseline` leg of bench.py
 * (cpu_baseline.kind = "port").  Nothing in plonky3_eon_amd/ links or calls this.
 *
 * Restated (reference = Lolazyx/plonky3-eon; read as text, not compiled -- it is Rust with
 * crates.io dependencies absent here):
 *   - Fr arithmetic: bn254/src/helpers.rs:60-205 (wrapping add/sub, mul_small,
 *     mul_small_and_acc, interleaved_monty_reduction with mu = p^-1 mod 2^64, monty_mul) and
 *     bn254/src/field.rs:464-526 (add/sub/mul), :553-574 (two_adic_generator).
 *   - Radix2Dit::dft_batch (dft/src/radix_2_dit.rs:61-122) and the trait defaults
 *     idft/coset_dft/coset_idft/coset_lde (dft/src/traits.rs:83-249, dft/src/util.rs:15-36).
 *   - Radix2DitParallel::dft_batch / coset_lde_batch with its two-half schedule
 *     (dft/src/radix_2_dit_parallel.rs:53-553), OpenMP standing in for rayon's
 *     par_row_chunks_exact_mut; reverse_matrix_index_bits (matrix/src/util.rs:36-57).
 */
#include "eon_oracle.h"

#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

static const uint64_t P[4] = {0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull,
                              0x30644e72e131a029ull};
static const uint64_t MU = 0x3d1e0a6c10000001ull; /* P^-1 mod 2^64 (bn254/src/field.rs:40) */
static const uint64_t R2[4] = {0x1bb8e645ae216da7ull, 0x53fe3ab1e35c59e3ull, 0x8c49833d53bb8085ull,
                               0x0216d0b17f4e44a5ull};
static const uint64_t ONE[4] = {0xac96341c4ffffffbull, 0x36fc76959f60cd29ull, 0x666ea36f7879462eull,
                                0x0e0a77c19a07df2full};
static const uint64_t TWO_ADIC_GEN[4] = {0x636e735580d13d9cull, 0xa22bf3742445ffd6ull,
                                         0x56452ac01eb203d8ull, 0x1860ef942963f9e7ull};

/* ---- Fr (bn254/src/helpers.rs, bn254/src/field.rs) ----------------------------------------- */
static inline int wrapping_add4(const uint64_t* a, const uint64_t* b, uint64_t* o) {
    u128 c = 0;
    for (int i = 0; i < 4; i++) {
        c += (u128)a[i] + b[i];
        o[i] = (uint64_t)c;
        c >>= 64;
    }
    return (int)c;
}

static inline int wrapping_sub4(const uint64_t* a, const uint64_t* b, uint64_t* o) {
    int borrow = 0;
    for (int i = 0; i < 4; i++) {
        uint64_t d = a[i] - b[i];
        int b1 = a[i] < b[i];
        uint64_t e = d - (uint64_t)borrow;
        int b2 = d < (uint64_t)borrow;
        o[i] = e;
        borrow = b1 | b2;
    }
    return borrow;
}

static inline uint64_t mul_small_and_acc(const uint64_t* lhs, uint64_t rhs, const uint64_t* add,
                                         uint64_t* out) {
    u128 acc = (u128)lhs[0] * rhs + (add ? add[0] : 0);
    uint64_t out0 = (uint64_t)acc;
    acc >>= 64;
    for (int i = 1; i < 4; i++) {
        acc += (u128)lhs[i] * rhs + (add ? add[i] : 0);
        out[i - 1] = (uint64_t)acc;
        acc >>= 64;
    }
    out[3] = (uint64_t)acc;
    return out0;
}

static inline void interleaved_monty_reduction(uint64_t acc0, const uint64_t* acc, uint64_t* res) {
    uint64_t t = acc0 * MU, u[4], sub[4];
    (void)mul_small_and_acc(P, t, NULL, u);
    if (wrapping_sub4(acc, u, sub)) {
        wrapping_add4(sub, P, res);
    } else {
        memcpy(res, sub, 32);
    }
}

void or_fr_mul(const fr_t* a, const fr_t* b, fr_t* r) {
    /* monty_mul (bn254/src/helpers.rs:188-205) */
    uint64_t acc[4], res[4];
    uint64_t acc0 = mul_small_and_acc(a->v, b->v[0], NULL, acc);
    interleaved_monty_reduction(acc0, acc, res);
    for (int i = 1; i < 4; i++) {
        acc0 = mul_small_and_acc(a->v, b->v[i], res, acc);
        interleaved_monty_reduction(acc0, acc, res);
    }
    memcpy(r->v, res, 32);
}

void or_fr_add(const fr_t* a, const fr_t* b, fr_t* r) {
    /* Fr::add (bn254/src/field.rs:464-489) */
    uint64_t sum[4], corr[4];
    wrapping_add4(a->v, b->v, sum);
    if (wrapping_sub4(sum, P, corr))
        memcpy(r->v, sum, 32);
    else
        memcpy(r->v, corr, 32);
}

void or_fr_sub(const fr_t* a, const fr_t* b, fr_t* r) {
    /* Fr::sub (bn254/src/field.rs:491-508) */
    uint64_t d[4];
    if (wrapping_sub4(a->v, b->v, d)) wrapping_add4(d, P, d);
    memcpy(r->v, d, 32);
}

static inline fr_t fmul(fr_t a, fr_t b) {
    fr_t r;
    or_fr_mul(&a, &b, &r);
    return r;
}
static inline fr_t fadd(fr_t a, fr_t b) {
    fr_t r;
    or_fr_add(&a, &b, &r);
    return r;
}
static inline fr_t fsub(fr_t a, fr_t b) {
    fr_t r;
    or_fr_sub(&a, &b, &r);
    return r;
}
static inline fr_t fone(void) {
    fr_t r;
    memcpy(r.v, ONE, 32);
    return r;
}

fr_t or_fr_from_u64(uint64_t x) {
    /* Fr::new (bn254/src/field.rs:111-117): monty_mul(R^2, [x,0,0,0]) */
    fr_t a = {{x, 0, 0, 0}}, r2;
    memcpy(r2.v, R2, 32);
    return fmul(r2, a);
}

fr_t or_fr_pow(fr_t b, uint64_t e) {
    fr_t r = fone();
    while (e) {
        if (e & 1) r = fmul(r, b);
        b = fmul(b, b);
        e >>= 1;
    }
    return r;
}

fr_t or_fr_inverse(fr_t a) {
    /* a^(p-2); the reference uses a gcd inversion (bn254/src/helpers.rs:417), same value */
    uint64_t e[4];
    const uint64_t two[4] = {2, 0, 0, 0};
    wrapping_sub4(P, two, e);
    fr_t r = fone();
    for (int w = 3; w >= 0; w--)
        for (int bit = 63; bit >= 0; bit--) {
            r = fmul(r, r);
            if ((e[w] >> bit) & 1) r = fmul(r, a);
        }
    return r;
}

fr_t or_two_adic_generator(uint32_t bits) {
    fr_t w;
    memcpy(w.v, TWO_ADIC_GEN, 32);
    for (uint32_t i = bits; i < 28; i++) w = fmul(w, w);
    return w;
}

static inline uint64_t rev_bits(uint64_t x, uint32_t bits) {
    /* p3_util::reverse_bits_len (util/src/lib.rs:70-78) */
    uint64_t r = 0;
    for (uint32_t i = 0; i < bits; i++) {
        r = (r << 1) | (x & 1);
        x >>= 1;
    }
    return r;
}

static uint32_t log2_strict(uint64_t n) { return 63 - __builtin_clzll(n); }

/* ---- matrix helpers ------------------------------------------------------------------------ */
static void swap_rows(fr_t* m, uint64_t w, uint64_t i, uint64_t j) {
    for (uint64_t c = 0; c < w; c++) {
        fr_t t = m[i * w + c];
        m[i * w + c] = m[j * w + c];
        m[j * w + c] = t;
    }
}

void or_reverse_matrix_index_bits(fr_t* m, uint64_t h, uint64_t w) {
    /* matrix/src/util.rs:36-57 */
    uint32_t lg = log2_strict(h);
#pragma omp parallel for schedule(static)
    for (uint64_t i = 0; i < h; i++) {
        uint64_t j = rev_bits(i, lg);
        if (i < j) swap_rows(m, w, i, j);
    }
}

static void butterfly_rows(fr_t* lo, fr_t* hi, uint64_t w, fr_t t) {
    /* DitButterfly (dft/src/butterflies.rs:177-185) */
    for (uint64_t c = 0; c < w; c++) {
        fr_t x2t = fmul(hi[c], t);
        fr_t x1 = lo[c];
        lo[c] = fadd(x1, x2t);
        hi[c] = fsub(x1, x2t);
    }
}

static void powers(fr_t base, fr_t start, uint64_t n, fr_t* out) {
    fr_t cur = start;
    for (uint64_t i = 0; i < n; i++) {
        out[i] = cur;
        cur = fmul(cur, base);
    }
}

static void reverse_slice(fr_t* v, uint64_t n) {
    if (n <= 1) return;
    uint32_t lg = log2_strict(n);
    for (uint64_t i = 0; i < n; i++) {
        uint64_t j = rev_bits(i, lg);
        if (i < j) {
            fr_t t = v[i];
            v[i] = v[j];
            v[j] = t;
        }
    }
}

/* ---- Radix2Dit (dft/src/radix_2_dit.rs:61-122) --------------------------------------------- */
void or_radix2dit_dft_batch(fr_t* m, uint64_t h, uint64_t w) {
    uint32_t log_h = log2_strict(h);
    fr_t* tw = (fr_t*)malloc(sizeof(fr_t) * (h ? h : 1));
    powers(or_two_adic_generator(log_h), fone(), h, tw);
    or_reverse_matrix_index_bits(m, h, w);
    for (uint32_t layer = 0; layer < log_h; layer++) {
        uint32_t layer_rev = log_h - 1 - layer;
        uint64_t half = 1ull << layer, block = half * 2;
#pragma omp parallel for schedule(static)
        for (uint64_t b = 0; b < h / block; b++) {
            for (uint64_t ind = 0; ind < half; ind++) {
                fr_t* lo = m + (b * block + ind) * w;
                fr_t* hi = m + (b * block + half + ind) * w;
                if (ind == 0) {
                    for (uint64_t c = 0; c < w; c++) { /* TwiddleFreeButterfly */
                        fr_t x1 = lo[c], x2 = hi[c];
                        lo[c] = fadd(x1, x2);
                        hi[c] = fsub(x1, x2);
                    }
                } else {
                    butterfly_rows(lo, hi, w, tw[ind << layer_rev]);
                }
            }
        }
    }
    free(tw);
}

static void scale_all(fr_t* m, uint64_t n, fr_t s) {
#pragma omp parallel for schedule(static)
    for (uint64_t i = 0; i < n; i++) m[i] = fmul(m[i], s);
}

static void coset_shift_cols(fr_t* m, uint64_t h, uint64_t w, fr_t shift) {
    /* dft/src/util.rs:28-36 */
    fr_t* p = (fr_t*)malloc(sizeof(fr_t) * h);
    powers(shift, fone(), h, p);
#pragma omp parallel for schedule(static)
    for (uint64_t r = 0; r < h; r++)
        for (uint64_t c = 0; c < w; c++) m[r * w + c] = fmul(m[r * w + c], p[r]);
    free(p);
}

void or_idft_batch(fr_t* m, uint64_t h, uint64_t w) {
    /* dft/src/traits.rs:111-122 over Radix2Dit: dft, divide_by_height, swap rows r <-> h-r */
    or_radix2dit_dft_batch(m, h, w);
    scale_all(m, h * w, or_fr_inverse(or_fr_from_u64(h)));
    for (uint64_t r = 1; r < h / 2; r++) swap_rows(m, w, r, h - r);
}

void or_coset_dft_batch(fr_t* m, uint64_t h, uint64_t w, fr_t shift) {
    coset_shift_cols(m, h, w, shift); /* dft/src/traits.rs:83-91 */
    or_radix2dit_dft_batch(m, h, w);
}

void or_coset_idft_batch(fr_t* m, uint64_t h, uint64_t w, fr_t shift) {
    or_idft_batch(m, h, w); /* dft/src/traits.rs:144-153 */
    coset_shift_cols(m, h, w, or_fr_inverse(shift));
}

void or_coset_lde_batch(const fr_t* in, fr_t* out, uint64_t h, uint64_t w, uint32_t added_bits,
                        fr_t shift) {
    /* dft/src/traits.rs:226-249 (default path, natural order) */
    memcpy(out, in, sizeof(fr_t) * h * w);
    or_idft_batch(out, h, w);
    memset(out + h * w, 0, sizeof(fr_t) * ((h << added_bits) - h) * w);
    or_coset_dft_batch(out, h << added_bits, w, shift);
}

/* ---- Radix2DitParallel (dft/src/radix_2_dit_parallel.rs) ----------------------------------- */
/* dit_layer (:452-484): blocks of 2^(layer+1) rows, twiddle i = tw[i * tw_stride] */
static void dit_layer(fr_t* sub, uint64_t rows, uint64_t w, uint32_t layer, const fr_t* tw,
                      uint64_t tw_stride) {
    uint64_t half = 1ull << layer, block = half * 2;
    for (uint64_t b = 0; b < rows / block; b++)
        for (uint64_t i = 0; i < half; i++)
            butterfly_rows(sub + (b * block + i) * w, sub + (b * block + half + i) * w, w,
                           tw[i * tw_stride]);
}

/* dit_layer_rev (:524-553): blocks of 2^(layer_rev+1) rows, block b uses twiddles_rev[b] */
static void dit_layer_rev(fr_t* sub, uint64_t rows, uint64_t w, uint32_t log_h, uint32_t layer,
                          const fr_t* tw_rev) {
    uint32_t layer_rev = log_h - 1 - layer;
    uint64_t half = 1ull << layer_rev, block = half * 2;
    /* the whole half-block is one (lo, hi) pair of slices, one twiddle per block */
    for (uint64_t b = 0; b < rows / block; b++)
        butterfly_rows(sub + b * block * w, sub + (b * block + half) * w, half * w, tw_rev[b]);
}

/* first_half (:296-315) with uniform twiddles; per-layer twiddles when coset != NULL
 * (first_half_general, :320-335) */
static void first_half(fr_t* m, uint64_t h, uint64_t w, uint32_t mid, const fr_t* tw,
                       fr_t* const* coset) {
    uint32_t log_h = log2_strict(h);
    uint64_t chunk = 1ull << mid;
#pragma omp parallel for schedule(static)
    for (uint64_t t = 0; t < h / chunk; t++) {
        fr_t* sub = m + t * chunk * w;
        for (uint32_t layer = 0; layer < mid; layer++) {
            uint32_t layer_rev = log_h - 1 - layer;
            if (coset)
                dit_layer(sub, chunk, w, layer, coset[layer_rev], 1);
            else
                dit_layer(sub, chunk, w, layer, tw, 1ull << layer_rev);
        }
    }
}

/* second_half (:393-421, optional scale) / second_half_general (:426-449) */
static void second_half(fr_t* m, uint64_t h, uint64_t w, uint32_t mid, const fr_t* tw_rev,
                        fr_t* const* coset, const fr_t* scale) {
    uint32_t log_h = log2_strict(h);
    uint64_t chunk = 1ull << (log_h - mid);
#pragma omp parallel for schedule(static)
    for (uint64_t t = 0; t < h / chunk; t++) {
        fr_t* sub = m + t * chunk * w;
        if (scale)
            for (uint64_t i = 0; i < chunk * w; i++) sub[i] = fmul(sub[i], *scale);
        for (uint32_t layer = mid; layer < log_h; layer++) {
            uint64_t first_block = t << (layer - mid);
            uint32_t layer_rev = log_h - 1 - layer;
            const fr_t* twr = coset ? coset[layer_rev] : tw_rev;
            dit_layer_rev(sub, chunk, w, log_h, layer, twr + first_block);
        }
    }
}

/* get_or_compute_coset_twiddles (:80-115): layer l holds shift^(2^l) * (root^(2^l))^j for
 * j < h >> (l+1), bit-reversed when log_h - 1 - l >= mid */
static fr_t** coset_twiddles(uint32_t log_h, fr_t shift) {
    uint32_t mid = (log_h + 1) / 2;
    uint64_t h = 1ull << log_h;
    fr_t root = or_two_adic_generator(log_h);
    fr_t** tw = (fr_t**)calloc(log_h ? log_h : 1, sizeof(fr_t*));
    fr_t shift_pow = shift, root_pow = root;
    for (uint32_t layer = 0; layer < log_h; layer++) {
        uint64_t n = h >> (layer + 1);
        tw[layer] = (fr_t*)malloc(sizeof(fr_t) * n);
        powers(root_pow, shift_pow, n, tw[layer]);
        if (log_h - 1 - layer >= mid) reverse_slice(tw[layer], n);
        shift_pow = fmul(shift_pow, shift_pow);
        root_pow = fmul(root_pow, root_pow);
    }
    return tw;
}

static void free_twiddles(fr_t** tw, uint32_t log_h) {
    for (uint32_t i = 0; i < log_h; i++) free(tw[i]);
    free(tw);
}

/* coset_dft (:232-250), in place on a height-h block that holds bit-reversed coefficients */
static void coset_dft_block(fr_t* m, uint64_t h, uint64_t w, fr_t shift) {
    uint32_t log_h = log2_strict(h);
    if (log_h == 0) return;
    uint32_t mid = (log_h + 1) / 2;
    fr_t** tw = coset_twiddles(log_h, shift);
    first_half(m, h, w, mid, NULL, tw);
    or_reverse_matrix_index_bits(m, h, w);
    second_half(m, h, w, mid, NULL, tw, NULL);
    free_twiddles(tw, log_h);
}

void or_r2dp_dft_batch(fr_t* m, uint64_t h, uint64_t w) {
    /* dft_batch (:148-166): result storage is bit-reversed */
    uint32_t log_h = log2_strict(h);
    uint32_t mid = (log_h + 1) / 2;
    uint64_t half_h = h >> 1;
    fr_t* tw = (fr_t*)malloc(sizeof(fr_t) * (half_h ? half_h : 1));
    powers(or_two_adic_generator(log_h), fone(), half_h, tw);
    fr_t* twr = (fr_t*)malloc(sizeof(fr_t) * (half_h ? half_h : 1));
    memcpy(twr, tw, sizeof(fr_t) * half_h);
    reverse_slice(twr, half_h);
    or_reverse_matrix_index_bits(m, h, w);
    first_half(m, h, w, mid, tw, NULL);
    or_reverse_matrix_index_bits(m, h, w);
    second_half(m, h, w, mid, twr, NULL, NULL);
    free(tw);
    free(twr);
}

void or_r2dp_coset_lde_batch(const fr_t* in, fr_t* out, uint64_t h, uint64_t w, uint32_t added_bits,
                             fr_t shift) {
    /* coset_lde_batch (:169-228): `out` has (h << added_bits) rows; result storage bit-reversed */
    uint32_t log_h = log2_strict(h);
    uint32_t mid = (log_h + 1) / 2;
    uint64_t half_h = h >> 1;
    memcpy(out, in, sizeof(fr_t) * h * w);
    fr_t* tw = (fr_t*)malloc(sizeof(fr_t) * (half_h ? half_h : 1));
    powers(or_fr_inverse(or_two_adic_generator(log_h)), fone(), half_h, tw);
    fr_t* twr = (fr_t*)malloc(sizeof(fr_t) * (half_h ? half_h : 1));
    memcpy(twr, tw, sizeof(fr_t) * half_h);
    reverse_slice(twr, half_h);
    or_reverse_matrix_index_bits(out, h, w);
    first_half(out, h, w, mid, tw, NULL);
    or_reverse_matrix_index_bits(out, h, w);
    fr_t scale = or_fr_inverse(or_fr_from_u64(h));
    second_half(out, h, w, mid, twr, NULL, &scale);
    free(tw);
    free(twr);
    /* coefficients are now bit-reversed in block 0 */
    fr_t g_big = or_two_adic_generator(log_h + added_bits);
    for (uint64_t coset_idx = 1; coset_idx < (1ull << added_bits); coset_idx++) {
        fr_t total_shift = fmul(or_fr_pow(g_big, coset_idx), shift);
        uint64_t dest = rev_bits(coset_idx, added_bits);
        fr_t* dst = out + dest * h * w;
        /* coset_dft_oop (:254-292) == copy + in-place coset_dft (same arithmetic) */
        memcpy(dst, out, sizeof(fr_t) * h * w);
        coset_dft_block(dst, h, w, total_shift);
    }
    coset_dft_block(out, h, w, shift);
}

/* ---- conversions for the Python side ------------------------------------------------------- */
void or_fr_mul_batch(const fr_t* a, const fr_t* b, fr_t* r, uint64_t n) {
#pragma omp parallel for schedule(static)
    for (uint64_t i = 0; i < n; i++) or_fr_mul(&a[i], &b[i], &r[i]);
}

int or_num_threads(void) {
#ifdef _OPENMP
    extern int omp_get_max_threads(void);
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* threads of every later parallel region (the cpu_baseline's T = 1 beside T = nproc) */
void or_set_num_threads(int n) {
#ifdef _OPENMP
    extern void omp_set_num_threads(int);
    omp_set_num_threads(n > 0 ? n : 1);
#else
    (void)n;
#endif
}

/* ---- KzgPcs::get_evaluations_on_domain (kzg/src/pcs.rs:267-287) ----------------------------- */
fr_t or_eval_poly_col(const fr_t* coeffs, uint64_t h, uint64_t w, uint64_t col, fr_t point) {
    /* eval_poly (kzg/src/util.rs:63-68): Horner from the top coefficient */
    fr_t acc = {{0, 0, 0, 0}};
    for (uint64_t i = h; i-- > 0;) acc = fadd(fmul(acc, point), coeffs[i * w + col]);
    return acc;
}

void or_kzg_evaluations_on_domain(const fr_t* coeffs, uint64_t h, uint64_t w, uint32_t log_q,
                                  fr_t shift, fr_t* out) {
    /* every column polynomial at every point shift * w_Q^i of the domain, row-major Q x w */
    uint64_t q = 1ull << log_q;
    fr_t g = or_two_adic_generator(log_q);
#pragma omp parallel for schedule(dynamic, 16)
    for (uint64_t i = 0; i < q; i++) {
        fr_t pt = fmul(shift, or_fr_pow(g, i));
        for (uint64_t c = 0; c < w; c++) out[i * w + c] = or_eval_poly_col(coeffs, h, w, c, pt);
    }
}

/* ---- BN254 G1 over Fq (halo2curves 0.9 is not in the reference tree; the group law and the MSM
 * value are restated directly: y^2 = x^3 + 3, generator (1, 2)) ----------------------------- */
static const uint64_t FQ_P[4] = {0x3c208c16d87cfd47ull, 0x97816a916871ca8dull, 0xb85045b68181585dull,
                                 0x30644e72e131a029ull};
static const uint64_t FQ_MU = 0x782df87d1b799c77ull; /* q^-1 mod 2^64 */
static const uint64_t FQ_R2[4] = {0xf32cfc5b538afa89ull, 0xb5e71911d44501fbull, 0x47ab1eff0a417ff6ull,
                                  0x06d89f71cab8351full};
static const uint64_t FQ_ONE[4] = {0xd35d438dc58f0d9dull, 0x0a78eb28f5c70b3dull, 0x666ea36f7879462cull,
                                   0x0e0a77c19a07df2full};

typedef struct {
    uint64_t v[4];
} fq_t;

static inline void fq_reduce_step(uint64_t acc0, const uint64_t* acc, uint64_t* res) {
    uint64_t t = acc0 * FQ_MU, u[4], sub[4];
    (void)mul_small_and_acc(FQ_P, t, NULL, u);
    if (wrapping_sub4(acc, u, sub))
        wrapping_add4(sub, FQ_P, res);
    else
        memcpy(res, sub, 32);
}

static inline fq_t qmul(fq_t a, fq_t b) {
    /* the same interleaved Montgomery product as Fr (bn254/src/helpers.rs:188-205), modulus q */
    uint64_t acc[4], res[4];
    uint64_t acc0 = mul_small_and_acc(a.v, b.v[0], NULL, acc);
    fq_reduce_step(acc0, acc, res);
    for (int i = 1; i < 4; i++) {
        acc0 = mul_small_and_acc(a.v, b.v[i], res, acc);
        fq_reduce_step(acc0, acc, res);
    }
    fq_t r;
    memcpy(r.v, res, 32);
    return r;
}
static inline fq_t qadd(fq_t a, fq_t b) {
    fq_t r;
    uint64_t s[4], c[4];
    wrapping_add4(a.v, b.v, s);
    if (wrapping_sub4(s, FQ_P, c))
        memcpy(r.v, s, 32);
    else
        memcpy(r.v, c, 32);
    return r;
}
static inline fq_t qsub(fq_t a, fq_t b) {
    fq_t r;
    if (wrapping_sub4(a.v, b.v, r.v)) wrapping_add4(r.v, FQ_P, r.v);
    return r;
}
static inline int qzero(fq_t a) { return (a.v[0] | a.v[1] | a.v[2] | a.v[3]) == 0; }
static inline int qeq(fq_t a, fq_t b) { return !memcmp(a.v, b.v, 32); }
static inline fq_t qone(void) {
    fq_t r;
    memcpy(r.v, FQ_ONE, 32);
    return r;
}
static inline fq_t qfrom_u64(uint64_t x) {
    fq_t a = {{x, 0, 0, 0}}, r2;
    memcpy(r2.v, FQ_R2, 32);
    return qmul(r2, a);
}
static fq_t qinv(fq_t a) {
    uint64_t e[4];
    const uint64_t two[4] = {2, 0, 0, 0};
    wrapping_sub4(FQ_P, two, e);
    fq_t r = qone();
    for (int w = 3; w >= 0; w--)
        for (int bit = 63; bit >= 0; bit--) {
            r = qmul(r, r);
            if ((e[w] >> bit) & 1) r = qmul(r, a);
        }
    return r;
}

typedef struct {
    fq_t X, Y, Z; /* Jacobian; Z = 0 is the point at infinity */
} g1j_t;

static g1j_t jinf(void) {
    g1j_t r;
    r.X = qone();
    r.Y = qone();
    memset(r.Z.v, 0, 32);
    return r;
}

static g1j_t jfrom_affine(const g1_affine_t* a) {
    g1j_t r;
    if (qzero(*(const fq_t*)a->x) && qzero(*(const fq_t*)a->y)) return jinf();
    memcpy(r.X.v, a->x, 32);
    memcpy(r.Y.v, a->y, 32);
    r.Z = qone();
    return r;
}

static g1j_t jdbl(g1j_t p) {
    /* dbl-2009-l */
    if (qzero(p.Z)) return p;
    fq_t A = qmul(p.X, p.X), B = qmul(p.Y, p.Y), C = qmul(B, B);
    fq_t t = qadd(p.X, B);
    fq_t D = qsub(qsub(qmul(t, t), A), C);
    D = qadd(D, D);
    fq_t E = qadd(qadd(A, A), A), F = qmul(E, E);
    g1j_t r;
    r.X = qsub(F, qadd(D, D));
    fq_t C8 = qadd(C, C);
    C8 = qadd(C8, C8);
    C8 = qadd(C8, C8);
    r.Y = qsub(qmul(E, qsub(D, r.X)), C8);
    fq_t yz = qmul(p.Y, p.Z);
    r.Z = qadd(yz, yz);
    return r;
}

static g1j_t jadd(g1j_t p, g1j_t q) {
    /* add-2007-bl with the doubling / inverse cases */
    if (qzero(p.Z)) return q;
    if (qzero(q.Z)) return p;
    fq_t Z1Z1 = qmul(p.Z, p.Z), Z2Z2 = qmul(q.Z, q.Z);
    fq_t U1 = qmul(p.X, Z2Z2), U2 = qmul(q.X, Z1Z1);
    fq_t S1 = qmul(qmul(p.Y, q.Z), Z2Z2), S2 = qmul(qmul(q.Y, p.Z), Z1Z1);
    fq_t H = qsub(U2, U1), rr = qsub(S2, S1);
    if (qzero(H)) {
        if (qzero(rr)) return jdbl(p);
        return jinf();
    }
    fq_t H2 = qadd(H, H), I = qmul(H2, H2), J = qmul(H, I);
    rr = qadd(rr, rr);
    fq_t V = qmul(U1, I);
    g1j_t r;
    r.X = qsub(qsub(qmul(rr, rr), J), qadd(V, V));
    fq_t s1j = qmul(S1, J);
    r.Y = qsub(qmul(rr, qsub(V, r.X)), qadd(s1j, s1j));
    fq_t zs = qadd(p.Z, q.Z);
    r.Z = qmul(qsub(qsub(qmul(zs, zs), Z1Z1), Z2Z2), H);
    return r;
}

static void jto_affine(g1j_t p, g1_affine_t* out) {
    if (qzero(p.Z)) {
        memset(out, 0, sizeof *out);
        return;
    }
    fq_t zi = qinv(p.Z), zi2 = qmul(zi, zi), zi3 = qmul(zi2, zi);
    fq_t x = qmul(p.X, zi2), y = qmul(p.Y, zi3);
    memcpy(out->x, x.v, 32);
    memcpy(out->y, y.v, 32);
}

static void fr_canonical(const fr_t* s, uint64_t* out) {
    fr_t one_int = {{1, 0, 0, 0}}, r;
    or_fr_mul(s, &one_int, &r); /* as_canonical_biguint (bn254/src/field.rs:456-461) */
    memcpy(out, r.v, 32);
}

static g1j_t jmul(g1j_t p, const uint64_t* k) {
    g1j_t acc = jinf();
    for (int w = 3; w >= 0; w--)
        for (int b = 63; b >= 0; b--) {
            acc = jdbl(acc);
            if ((k[w] >> b) & 1) acc = jadd(acc, p);
        }
    return acc;
}

void or_g1_generator(g1_affine_t* out) {
    fq_t x = qfrom_u64(1), y = qfrom_u64(2);
    memcpy(out->x, x.v, 32);
    memcpy(out->y, y.v, 32);
}

void or_g1_mul(const g1_affine_t* p, const fr_t* scalar, g1_affine_t* out) {
    uint64_t k[4];
    fr_canonical(scalar, k);
    jto_affine(jmul(jfrom_affine(p), k), out);
}

void or_g1_add(const g1_affine_t* a, const g1_affine_t* b, g1_affine_t* out) {
    jto_affine(jadd(jfrom_affine(a), jfrom_affine(b)), out);
}

int or_g1_on_curve(const g1_affine_t* a) {
    fq_t x, y;
    memcpy(x.v, a->x, 32);
    memcpy(y.v, a->y, 32);
    if (qzero(x) && qzero(y)) return 1;
    fq_t rhs = qadd(qmul(qmul(x, x), x), qfrom_u64(3));
    return qeq(qmul(y, y), rhs);
}

void or_g1_srs(uint64_t n, const fr_t* alpha, g1_affine_t* out) {
    /* init_srs_unsafe g1_powers (kzg/src/params.rs:123-139): g1_powers[i] = alpha^i * G */
    g1_affine_t g;
    or_g1_generator(&g);
    g1j_t gj = jfrom_affine(&g);
#pragma omp parallel for schedule(dynamic, 64)
    for (uint64_t i = 0; i < n; i++) {
        fr_t s = or_fr_pow(*alpha, i);
        uint64_t k[4];
        fr_canonical(&s, k);
        jto_affine(jmul(gj, k), &out[i]);
    }
}

/* XYZZ coordinates (x = X / ZZ, y = Y / ZZZ; ZZ = 0 is the identity) for the Pippenger buckets */
typedef struct {
    fq_t X, Y, ZZ, ZZZ;
} g1x_t;

static g1x_t xinf(void) {
    g1x_t r;
    memset(&r, 0, sizeof r);
    r.X = qone();
    r.Y = qone();
    return r;
}

static g1x_t xdbl(g1x_t p) { /* dbl-2008-s-1, a = 0 */
    if (qzero(p.ZZ)) return p;
    fq_t U = qadd(p.Y, p.Y), V = qmul(U, U), W = qmul(U, V), S = qmul(p.X, V);
    fq_t X2 = qmul(p.X, p.X), M = qadd(qadd(X2, X2), X2);
    g1x_t r;
    r.X = qsub(qmul(M, M), qadd(S, S));
    r.Y = qsub(qmul(M, qsub(S, r.X)), qmul(W, p.Y));
    r.ZZ = qmul(V, p.ZZ);
    r.ZZZ = qmul(W, p.ZZZ);
    return r;
}

static g1x_t xdbl_affine(fq_t x, fq_t y) { /* mdbl-2008-s-1 */
    fq_t U = qadd(y, y), V = qmul(U, U), W = qmul(U, V), S = qmul(x, V);
    fq_t X2 = qmul(x, x), M = qadd(qadd(X2, X2), X2);
    g1x_t r;
    r.X = qsub(qmul(M, M), qadd(S, S));
    r.Y = qsub(qmul(M, qsub(S, r.X)), qmul(W, y));
    r.ZZ = V;
    r.ZZZ = W;
    return r;
}

static void xmadd(g1x_t* p, fq_t x, fq_t y) { /* madd-2008-s: p += (x, y) affine, 8M + 2S */
    if (qzero(p->ZZ)) {
        p->X = x;
        p->Y = y;
        p->ZZ = qone();
        p->ZZZ = qone();
        return;
    }
    fq_t U2 = qmul(x, p->ZZ), S2 = qmul(y, p->ZZZ);
    fq_t P = qsub(U2, p->X), R = qsub(S2, p->Y);
    if (qzero(P)) {
        if (qzero(R))
            *p = xdbl_affine(x, y);
        else
            *p = xinf();
        return;
    }
    fq_t PP = qmul(P, P), PPP = qmul(P, PP), Q = qmul(p->X, PP);
    fq_t X3 = qsub(qsub(qmul(R, R), PPP), qadd(Q, Q));
    p->Y = qsub(qmul(R, qsub(Q, X3)), qmul(p->Y, PPP));
    p->X = X3;
    p->ZZ = qmul(p->ZZ, PP);
    p->ZZZ = qmul(p->ZZZ, PPP);
}

static void xadd(g1x_t* p, const g1x_t* q) { /* add-2008-s: p += q */
    if (qzero(q->ZZ)) return;
    if (qzero(p->ZZ)) {
        *p = *q;
        return;
    }
    fq_t U1 = qmul(p->X, q->ZZ), U2 = qmul(q->X, p->ZZ), S1 = qmul(p->Y, q->ZZZ), S2 = qmul(q->Y, p->ZZZ);
    fq_t P = qsub(U2, U1), R = qsub(S2, S1);
    if (qzero(P)) {
        if (qzero(R))
            *p = xdbl(*p);
        else
            *p = xinf();
        return;
    }
    fq_t PP = qmul(P, P), PPP = qmul(P, PP), Q = qmul(U1, PP);
    fq_t X3 = qsub(qsub(qmul(R, R), PPP), qadd(Q, Q));
    p->Y = qsub(qmul(R, qsub(Q, X3)), qmul(S1, PPP));
    p->X = X3;
    p->ZZ = qmul(qmul(p->ZZ, q->ZZ), PP);
    p->ZZZ = qmul(qmul(p->ZZZ, q->ZZZ), PPP);
}

static void xto_affine(g1x_t p, g1_affine_t* out) {
    if (qzero(p.ZZ)) {
        memset(out, 0, sizeof *out);
        return;
    }
    fq_t x = qmul(p.X, qinv(p.ZZ)), y = qmul(p.Y, qinv(p.ZZZ));
    memcpy(out->x, x.v, 32);
    memcpy(out->y, y.v, 32);
}

/* Pippenger core: scalars[i * stride]; `par` = OpenMP inside (one large MSM) or serial (the
 * caller parallelises over many MSMs: or_g1_msm_columns / or_open_columns) */
static void msm_core(const g1_affine_t* pts, const fr_t* scalars, uint64_t stride, uint64_t n, g1_affine_t* out,
                     int par) {
    /* The value of G1::multi_exp (bn254/src/curve.rs:158-179; halo2curves' msm_best is not in the
     * tree).  Pippenger with SIGNED c-bit windows (digits in [-2^(c-1), 2^(c-1)], 2^(c-1) buckets
     * per window), XYZZ buckets with mixed additions of the affine bases (madd-2008-s), and OpenMP
     * over (window, point chunk) tasks so that every thread has work at any window count; the
     * chunks' buckets of a window are merged, then each window's running sum, then the windows by
     * doublings.  Empty input -> identity. */
    if (n == 0) {
        memset(out, 0, sizeof *out);
        return;
    }
    uint32_t lg = 0;
    while ((1ull << (lg + 1)) <= n) lg++;
    uint32_t c = lg > 5 ? lg - 3 : 2; /* ~n / 8 buckets per window */
    if (c > 16) c = 16;
    const uint32_t nw = (254 + c) / c; /* signed digits need the carry bit of the top window */
    const uint64_t nb = 1ull << (c - 1);
    /* signed digits, window-major: dg[w * n + i] in [-2^(c-1), 2^(c-1)] */
    int32_t* dg = (int32_t*)malloc(sizeof(int32_t) * nw * n);
#pragma omp parallel for schedule(static) if (par)
    for (uint64_t i = 0; i < n; i++) {
        uint64_t k[4];
        fr_canonical(&scalars[i * stride], k);
        int32_t carry = 0;
        for (uint32_t w = 0; w < nw; w++) {
            const uint32_t pos = w * c, li = pos / 64, off = pos % 64;
            uint64_t v = li < 4 ? k[li] >> off : 0;
            if (off && li + 1 < 4) v |= k[li + 1] << (64 - off);
            int32_t d = (int32_t)(v & ((1ull << c) - 1)) + carry;
            carry = 0;
            if (d > (int32_t)nb) {
                d -= (int32_t)(1u << c);
                carry = 1;
            }
            dg[(uint64_t)w * n + i] = d;
        }
    }
    extern int omp_get_max_threads(void);
    const int T = par ? omp_get_max_threads() : 1;
    uint32_t chunks = (uint32_t)((2 * T + nw - 1) / nw);
    if ((uint64_t)chunks > n / 64 + 1) chunks = (uint32_t)(n / 64 + 1);
    const uint64_t per = (n + chunks - 1) / chunks;
    g1x_t* bk = (g1x_t*)malloc(sizeof(g1x_t) * nb * nw * chunks);
#pragma omp parallel for schedule(dynamic, 1) if (par)
    for (uint64_t task = 0; task < (uint64_t)nw * chunks; task++) {
        const uint32_t w = (uint32_t)(task / chunks), ch = (uint32_t)(task % chunks);
        g1x_t* b = bk + task * nb;
        for (uint64_t j = 0; j < nb; j++) b[j] = xinf();
        const uint64_t i0 = ch * per, i1 = i0 + per < n ? i0 + per : n;
        for (uint64_t i = i0; i < i1; i++) {
            const int32_t d = dg[(uint64_t)w * n + i];
            if (!d) continue;
            fq_t x, y;
            memcpy(x.v, pts[i].x, 32);
            memcpy(y.v, pts[i].y, 32);
            if (qzero(x) && qzero(y)) continue; /* identity base */
            if (d < 0) y = qsub((fq_t){{0, 0, 0, 0}}, y);
            xmadd(&b[(d < 0 ? -d : d) - 1], x, y);
        }
    }
    g1x_t* wsum = (g1x_t*)malloc(sizeof(g1x_t) * nw);
#pragma omp parallel for schedule(dynamic, 1) if (par)
    for (uint32_t w = 0; w < nw; w++) {
        g1x_t* b0 = bk + (uint64_t)w * chunks * nb;
        for (uint32_t ch = 1; ch < chunks; ch++)
            for (uint64_t j = 0; j < nb; j++) xadd(&b0[j], &b0[ch * nb + j]);
        g1x_t run = xinf(), acc = xinf();
        for (uint64_t j = nb; j-- > 0;) {
            xadd(&run, &b0[j]);
            xadd(&acc, &run);
        }
        wsum[w] = acc;
    }
    g1x_t acc = wsum[nw - 1];
    for (int w = (int)nw - 2; w >= 0; w--) {
        for (uint32_t k = 0; k < c; k++) acc = xdbl(acc);
        xadd(&acc, &wsum[w]);
    }
    xto_affine(acc, out);
    free(wsum);
    free(bk);
    free(dg);
}

void or_g1_msm(const g1_affine_t* pts, const fr_t* scalars, uint64_t n, g1_affine_t* out) {
    msm_core(pts, scalars, 1, n, out, 1);
}

/* KzgPcs::commit's per-column loop (kzg/src/pcs.rs:244-251): out[j] = commit_column(column j of the
 * n x w row-major matrix) = sum_i mat[i][j] pts[i]; OpenMP over columns, each MSM serial -- the
 * schedule a CPU prover with many columns uses (the reference runs the columns one after another,
 * each multi_exp parallel inside). */
void or_g1_msm_columns(const g1_affine_t* pts, const fr_t* mat, uint64_t n, uint64_t w, g1_affine_t* out) {
#pragma omp parallel for schedule(dynamic, 1)
    for (uint64_t j = 0; j < w; j++) msm_core(pts, mat + j, w, n, &out[j], 0);
}

/* KzgPcs::open for one matrix and one point (kzg/src/pcs.rs:289-335): per column,
 * quotient_and_eval (kzg/src/util.rs:100-111) and the witness commit_column(quotient) over the
 * first n - 1 bases; OpenMP over columns.  values[j], witnesses[j]. */
void or_open_columns(const g1_affine_t* pts, const fr_t* coeffs, uint64_t n, uint64_t w, fr_t point,
                     fr_t* values, g1_affine_t* witnesses) {
#pragma omp parallel for schedule(dynamic, 1)
    for (uint64_t j = 0; j < w; j++) {
        fr_t* q = (fr_t*)malloc(sizeof(fr_t) * (n > 1 ? n - 1 : 1));
        or_quotient_and_eval(coeffs + j, n, w, point, q, &values[j]);
        if (n > 1)
            msm_core(pts, q, 1, n - 1, &witnesses[j], 0);
        else
            memset(&witnesses[j], 0, sizeof witnesses[j]);
        free(q);
    }
}

/* ---- Poseidon2-AIR over BN254 Fr: WIDTH 3, SBOX_DEGREE 5, SBOX_REGISTERS 1 ----
 * poseidon2-air/src/{air.rs:108-288, columns.rs:12-71, generation.rs:76-288, vectorized.rs};
 * linear layers: external = mds_light width 3 (poseidon2/src/external.rs:128-133),
 * internal = [2,1,1;1,2,1;1,1,3] (bn254/src/poseidon2.rs:55-63).
 * Columns per permutation: export, inputs[3], HF x (sbox x3[3], post[3]), PR x (x3, post_sbox),
 * HF x (x3[3], post[3]).  Permutation j of a VECTOR_LEN-wide trace sits at row j / VL,
 * columns [(j % VL) * cols, ...). */
static void p2_ext(fr_t* s) {
    fr_t sum = fadd(fadd(s[0], s[1]), s[2]);
    s[0] = fadd(s[0], sum);
    s[1] = fadd(s[1], sum);
    s[2] = fadd(s[2], sum);
}
static void p2_int(fr_t* s) {
    fr_t sum = fadd(s[0], fadd(s[1], s[2]));
    s[0] = fadd(s[0], sum);
    s[1] = fadd(s[1], sum);
    s[2] = fadd(fadd(s[2], s[2]), sum);
}

uint32_t or_p2_num_cols(uint32_t hf, uint32_t pr) { return 1 + 3 + 2 * hf * 6 + pr * 2; }

void or_p2_generate_trace(const fr_t* inputs, uint64_t n_perms, uint32_t vl, uint32_t hf, uint32_t pr,
                          const fr_t* rc_begin, const fr_t* rc_partial, const fr_t* rc_end,
                          fr_t* trace) {
    /* generate_trace_rows_for_perm (poseidon2-air/src/generation.rs:130-288) */
    uint32_t nc = or_p2_num_cols(hf, pr);
#pragma omp parallel for schedule(static)
    for (uint64_t j = 0; j < n_perms; j++) {
        fr_t* c = trace + (j / vl) * (uint64_t)nc * vl + (j % vl) * nc;
        fr_t s[3] = {inputs[3 * j], inputs[3 * j + 1], inputs[3 * j + 2]};
        uint32_t k = 0;
        c[k++] = fone(); /* export */
        for (int i = 0; i < 3; i++) c[k++] = s[i];
        p2_ext(s);
        for (uint32_t half = 0; half < 2; half++) {
            if (half == 1) {
                for (uint32_t r = 0; r < pr; r++) {
                    s[0] = fadd(s[0], rc_partial[r]);
                    fr_t x2 = fmul(s[0], s[0]), x3 = fmul(x2, s[0]);
                    c[k++] = x3;
                    s[0] = fmul(x3, x2);
                    c[k++] = s[0];
                    p2_int(s);
                }
            }
            const fr_t* rc = half == 0 ? rc_begin : rc_end;
            for (uint32_t r = 0; r < hf; r++) {
                for (int i = 0; i < 3; i++) {
                    s[i] = fadd(s[i], rc[3 * r + i]);
                    fr_t x2 = fmul(s[i], s[i]), x3 = fmul(x2, s[i]);
                    c[k++] = x3;
                    s[i] = fmul(x3, x2);
                }
                p2_ext(s);
                for (int i = 0; i < 3; i++) c[k++] = s[i];
            }
        }
    }
}

/* Constraint folding of one permutation row (air.rs:108-288 in assert order), accumulated as the
 * ProverConstraintFolder does: acc += alpha^(K-1-k) * C_k (folder.rs:81-85), i.e. Horner
 * acc = acc * alpha + C_k over the global constraint index k. */
static fr_t p2_fold(const fr_t* c, fr_t acc, fr_t alpha, uint32_t hf, uint32_t pr, const fr_t* rc_begin,
                    const fr_t* rc_partial, const fr_t* rc_end) {
    fr_t s[3] = {c[1], c[2], c[3]};
    uint32_t k = 4;
    p2_ext(s);
    for (uint32_t half = 0; half < 2; half++) {
        if (half == 1) {
            for (uint32_t r = 0; r < pr; r++) {
                s[0] = fadd(s[0], rc_partial[r]);
                fr_t x3 = c[k], post = c[k + 1];
                k += 2;
                fr_t x2 = fmul(s[0], s[0]);
                acc = fadd(fmul(acc, alpha), fsub(x3, fmul(x2, s[0]))); /* assert_eq(x3, x2 * x) */
                s[0] = fmul(x3, x2);
                acc = fadd(fmul(acc, alpha), fsub(s[0], post)); /* assert_eq(state0, post_sbox) */
                s[0] = post;
                p2_int(s);
            }
        }
        const fr_t* rc = half == 0 ? rc_begin : rc_end;
        for (uint32_t r = 0; r < hf; r++) {
            for (int i = 0; i < 3; i++) {
                s[i] = fadd(s[i], rc[3 * r + i]);
                fr_t x3 = c[k + i];
                fr_t x2 = fmul(s[i], s[i]);
                acc = fadd(fmul(acc, alpha), fsub(x3, fmul(x2, s[i])));
                s[i] = fmul(x3, x2);
            }
            p2_ext(s);
            for (int i = 0; i < 3; i++) {
                acc = fadd(fmul(acc, alpha), fsub(s[i], c[k + 3 + i])); /* assert_eq(state_i, post_i) */
                s[i] = c[k + 3 + i];
            }
            k += 6;
        }
    }
    return acc;
}

/* selectors_on_coset (commit/src/domain.rs:252-292) for trace domain H (shift 1, size 2^log_n) on
 * the coset shift * K (size 2^log_q); four Q-long vectors */
void or_selectors_on_coset(uint32_t log_n, uint32_t log_q, fr_t shift, fr_t* is_first, fr_t* is_last,
                           fr_t* is_transition, fr_t* inv_vanishing) {
    uint64_t q = 1ull << log_q, n = 1ull << log_n;
    uint32_t rate = log_q - log_n;
    fr_t s_pow_n = shift;
    for (uint32_t i = 0; i < log_n; i++) s_pow_n = fmul(s_pow_n, s_pow_n);
    fr_t g_rate = or_two_adic_generator(rate), g_q = or_two_adic_generator(log_q);
    fr_t h_inv = or_fr_inverse(or_two_adic_generator(log_n));
    uint64_t nr = 1ull << rate;
    fr_t* zh = (fr_t*)malloc(sizeof(fr_t) * nr);
    fr_t* zh_inv = (fr_t*)malloc(sizeof(fr_t) * nr);
    fr_t one = fone(), pw = one;
    for (uint64_t j = 0; j < nr; j++) {
        zh[j] = fsub(fmul(s_pow_n, pw), one);
        zh_inv[j] = or_fr_inverse(zh[j]);
        pw = fmul(pw, g_rate);
    }
    (void)n;
#pragma omp parallel for schedule(static)
    for (uint64_t i = 0; i < q; i++) {
        fr_t x = fmul(shift, or_fr_pow(g_q, i));
        fr_t z = zh[i % nr];
        is_first[i] = fmul(z, or_fr_inverse(fsub(x, one)));
        is_last[i] = fmul(z, or_fr_inverse(fsub(x, h_inv)));
        is_transition[i] = fsub(x, h_inv);
        inv_vanishing[i] = zh_inv[i % nr];
    }
    free(zh);
    free(zh_inv);
}

void or_p2_quotient_values(const fr_t* lde, uint32_t log_n, uint32_t log_qd, uint32_t vl, uint32_t hf,
                           uint32_t pr, const fr_t* rc_begin, const fr_t* rc_partial, const fr_t* rc_end,
                           fr_t alpha, fr_t* out) {
    /* quotient_values (eon-uni-stark/src/prover.rs:539-709) for the (vectorized) Poseidon2-AIR on
     * the quotient domain 5 * K, |K| = 2^(log_n + log_qd): out[i] = acc(row i) * inv_vanishing[i]
     * (the AIR reads no selectors and no next row) */
    uint32_t log_q = log_n + log_qd;
    uint64_t q = 1ull << log_q;
    uint32_t nc = or_p2_num_cols(hf, pr);
    fr_t* f = (fr_t*)malloc(sizeof(fr_t) * q * 4);
    or_selectors_on_coset(log_n, log_q, or_fr_from_u64(5), f, f + q, f + 2 * q, f + 3 * q);
#pragma omp parallel for schedule(static)
    for (uint64_t i = 0; i < q; i++) {
        fr_t acc = {{0, 0, 0, 0}};
        for (uint32_t v = 0; v < vl; v++)
            acc = p2_fold(lde + i * (uint64_t)nc * vl + (uint64_t)v * nc, acc, alpha, hf, pr, rc_begin,
                          rc_partial, rc_end);
        out[i] = fmul(acc, f[3 * q + i]);
    }
    free(f);
}

/* quotient_and_eval (kzg/src/util.rs:100-111) */
void or_quotient_and_eval(const fr_t* coeffs, uint64_t n, uint64_t stride, fr_t point, fr_t* quotient,
                          fr_t* value) {
    if (n == 0) {
        memset(value, 0, sizeof *value);
        return;
    }
    fr_t carry = coeffs[(n - 1) * stride];
    for (uint64_t i = n - 1; i-- > 0;) {
        quotient[i] = carry;
        carry = fadd(coeffs[i * stride], fmul(carry, point));
    }
    *value = carry;
}

/* Values at arbitrary points of the polynomials that interpolate each column of `evals` (n x w,
 * natural order) over the subgroup H = <omega_n>: the f(z) quotient_and_eval returns
 * (kzg/src/util.rs:100-111) computed straight from the evaluations by the barycentric formula
 * f(x) = (x^n - 1)/n * sum_i e_i * omega^i / (x - omega^i) -- O(n w) per point, so the verifier
 * restatement can check a full-size proof's opened values against the trace itself.  Points in H
 * are returned as the evaluation there.  out[p * w + c]. */
void or_bary_eval_cols(const fr_t* evals, uint64_t n, uint64_t w, const fr_t* points, uint32_t npts,
                       fr_t* out) {
    uint32_t lg = log2_strict(n);
    fr_t g = or_two_adic_generator(lg), one = fone();
    fr_t inv_n = or_fr_inverse(or_fr_from_u64(n));
    fr_t* wt = (fr_t*)malloc(sizeof(fr_t) * n);
    for (uint32_t p = 0; p < npts; p++) {
        fr_t x = points[p];
        /* x in H: f(x) is the evaluation at that row */
        fr_t xn = x;
        for (uint32_t i = 0; i < lg; i++) xn = fmul(xn, xn);
        if (memcmp(xn.v, one.v, 32) == 0) {
            fr_t pw = one;
            for (uint64_t i = 0; i < n; i++) {
                if (memcmp(pw.v, x.v, 32) == 0) {
                    memcpy(out + (uint64_t)p * w, evals + i * w, sizeof(fr_t) * w);
                    break;
                }
                pw = fmul(pw, g);
            }
            continue;
        }
        /* weights omega^i / (x - omega^i): batch inversion (Montgomery's trick) per thread block */
        int nt = or_num_threads();
        uint64_t blk = (n + nt - 1) / nt;
#pragma omp parallel for schedule(static)
        for (int t = 0; t < nt; t++) {
            uint64_t lo = t * blk, hi = lo + blk < n ? lo + blk : n;
            if (lo >= hi) continue;
            fr_t pw = or_fr_pow(g, lo), acc = one;
            for (uint64_t i = lo; i < hi; i++) {
                wt[i] = acc; /* prefix product of the denominators before i */
                acc = fmul(acc, fsub(x, pw));
                pw = fmul(pw, g);
            }
            fr_t inv = or_fr_inverse(acc);
            pw = or_fr_pow(g, hi - 1);
            fr_t g_inv = or_fr_inverse(g);
            for (uint64_t i = hi; i-- > lo;) {
                fr_t d = fsub(x, pw);
                fr_t di = fmul(inv, wt[i]); /* 1 / (x - omega^i) */
                inv = fmul(inv, d);
                wt[i] = fmul(di, pw);
                pw = fmul(pw, g_inv);
            }
        }
        fr_t scale = fmul(fsub(xn, one), inv_n);
        fr_t* part = (fr_t*)calloc((size_t)nt * w, sizeof(fr_t));
#pragma omp parallel for schedule(static)
        for (int t = 0; t < nt; t++) {
            uint64_t lo = t * blk, hi = lo + blk < n ? lo + blk : n;
            fr_t* acc = part + (uint64_t)t * w;
            for (uint64_t i = lo; i < hi; i++)
                for (uint64_t c = 0; c < w; c++) acc[c] = fadd(acc[c], fmul(evals[i * w + c], wt[i]));
        }
        for (uint64_t c = 0; c < w; c++) {
            fr_t s = {{0, 0, 0, 0}};
            for (int t = 0; t < nt; t++) s = fadd(s, part[(uint64_t)t * w + c]);
            out[(uint64_t)p * w + c] = fmul(s, scale);
        }
        free(part);
    }
    free(wt);
}
