/* eon_oracle.h -- CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY; see
 * eon_oracle.c).  fr_t is p3_bn254::Fr's layout: [u64;4] LE Montgomery, canonical. */
#ifndef EON_ORACLE_H
#define EON_ORACLE_H
#include <stdint.h>

typedef struct {
    uint64_t v[4];
} fr_t;

void or_fr_mul(const fr_t* a, const fr_t* b, fr_t* r);
void or_fr_add(const fr_t* a, const fr_t* b, fr_t* r);
void or_fr_sub(const fr_t* a, const fr_t* b, fr_t* r);
fr_t or_fr_from_u64(uint64_t x);
fr_t or_fr_pow(fr_t b, uint64_t e);
fr_t or_fr_inverse(fr_t a);
fr_t or_two_adic_generator(uint32_t bits);
void or_fr_mul_batch(const fr_t* a, const fr_t* b, fr_t* r, uint64_t n);
void or_reverse_matrix_index_bits(fr_t* m, uint64_t h, uint64_t w);

/* Radix2Dit + trait defaults: natural order, in place on m (h x w) */
void or_radix2dit_dft_batch(fr_t* m, uint64_t h, uint64_t w);
void or_idft_batch(fr_t* m, uint64_t h, uint64_t w);
void or_coset_dft_batch(fr_t* m, uint64_t h, uint64_t w, fr_t shift);
void or_coset_idft_batch(fr_t* m, uint64_t h, uint64_t w, fr_t shift);
void or_coset_lde_batch(const fr_t* in, fr_t* out, uint64_t h, uint64_t w, uint32_t added_bits,
                        fr_t shift);

/* Radix2DitParallel: bit-reversed storage */
void or_r2dp_dft_batch(fr_t* m, uint64_t h, uint64_t w);
void or_r2dp_coset_lde_batch(const fr_t* in, fr_t* out, uint64_t h, uint64_t w, uint32_t added_bits,
                             fr_t shift);

int or_num_threads(void);
void or_set_num_threads(int n);

/* BN254 G1: affine x, y as Fq Montgomery [u64;4] LE; identity = (0, 0) (the C-ABI layout) */
typedef struct {
    uint64_t x[4];
    uint64_t y[4];
} g1_affine_t;
void or_g1_generator(g1_affine_t* out);
void or_g1_mul(const g1_affine_t* p, const fr_t* scalar, g1_affine_t* out);
void or_g1_add(const g1_affine_t* a, const g1_affine_t* b, g1_affine_t* out);
int or_g1_on_curve(const g1_affine_t* a);
void or_g1_srs(uint64_t n, const fr_t* alpha, g1_affine_t* out);
void or_g1_msm(const g1_affine_t* pts, const fr_t* scalars, uint64_t n, g1_affine_t* out);
void or_g1_msm_columns(const g1_affine_t* pts, const fr_t* mat, uint64_t n, uint64_t w, g1_affine_t* out);
void or_open_columns(const g1_affine_t* pts, const fr_t* coeffs, uint64_t n, uint64_t w, fr_t point,
                     fr_t* values, g1_affine_t* witnesses);

/* KzgPcs::get_evaluations_on_domain's Horner evaluation (kzg/src/pcs.rs:267-287) */
fr_t or_eval_poly_col(const fr_t* coeffs, uint64_t h, uint64_t w, uint64_t col, fr_t point);
void or_kzg_evaluations_on_domain(const fr_t* coeffs, uint64_t h, uint64_t w, uint32_t log_q,
                                  fr_t shift, fr_t* out);

/* Poseidon2-AIR over BN254 (width 3, x^5 with one register) and the eon quotient */
uint32_t or_p2_num_cols(uint32_t hf, uint32_t pr);
void or_p2_generate_trace(const fr_t* inputs, uint64_t n_perms, uint32_t vl, uint32_t hf, uint32_t pr,
                          const fr_t* rc_begin, const fr_t* rc_partial, const fr_t* rc_end, fr_t* trace);
void or_selectors_on_coset(uint32_t log_n, uint32_t log_q, fr_t shift, fr_t* is_first, fr_t* is_last,
                           fr_t* is_transition, fr_t* inv_vanishing);
void or_p2_quotient_values(const fr_t* lde, uint32_t log_n, uint32_t log_qd, uint32_t vl, uint32_t hf,
                           uint32_t pr, const fr_t* rc_begin, const fr_t* rc_partial, const fr_t* rc_end,
                           fr_t alpha, fr_t* out);
void or_quotient_and_eval(const fr_t* coeffs, uint64_t n, uint64_t stride, fr_t point, fr_t* quotient,
                          fr_t* value);
/* the column polynomials (evaluations over H) at arbitrary points, barycentric: out[p * w + c] */
void or_bary_eval_cols(const fr_t* evals, uint64_t n, uint64_t w, const fr_t* points, uint32_t npts,
                       fr_t* out);
#endif

