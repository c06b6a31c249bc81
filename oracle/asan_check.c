/* asan_check.c -- TEST INFRASTRUCTURE: drives the C restatement (eon_oracle.c) under
 * AddressSanitizer + UndefinedBehaviorSanitizer (an ASan host build of the CPU
 * restatement).  Built and run by tests/test_oracle_asan.py (`make -C oracle asan_check`); every
 * entry point the tests and the bench's CPU baseline use is exercised on small, ragged and edge
 * shapes, with self-consistency checks (round trips, orders, identities), so that an out-of-bounds
 * access or undefined behaviour in the oracle fails the CPU suite.  Exit 0 = clean. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "eon_oracle.h"

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint64_t next64(void) { /* splitmix64 */
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static fr_t rand_fr(void) { return or_fr_from_u64(next64()); } /* canonical Montgomery residue */

static int fails = 0;
#define CHECK(c, msg)                                   \
    do {                                                \
        if (!(c)) {                                     \
            fprintf(stderr, "asan_check: %s\n", (msg)); \
            fails++;                                    \
        }                                               \
    } while (0)

static fr_t* rand_mat(uint64_t n) {
    fr_t* m = (fr_t*)malloc(sizeof(fr_t) * (n ? n : 1));
    for (uint64_t i = 0; i < n; i++) m[i] = rand_fr();
    return m;
}

static void dft_checks(void) {
    const uint64_t ws[] = {1, 3, 5};
    for (uint32_t lg = 0; lg <= 7; lg++)
        for (int k = 0; k < 3; k++) {
            const uint64_t h = 1ull << lg, w = ws[k], n = h * w;
            fr_t* x = rand_mat(n);
            fr_t* y = (fr_t*)malloc(sizeof(fr_t) * n);
            memcpy(y, x, sizeof(fr_t) * n);
            or_radix2dit_dft_batch(y, h, w);
            or_idft_batch(y, h, w);
            CHECK(memcmp(x, y, sizeof(fr_t) * n) == 0, "idft(dft(x)) != x");
            const fr_t s = or_fr_from_u64(5);
            memcpy(y, x, sizeof(fr_t) * n);
            or_coset_dft_batch(y, h, w, s);
            or_coset_idft_batch(y, h, w, s);
            CHECK(memcmp(x, y, sizeof(fr_t) * n) == 0, "coset_idft(coset_dft(x)) != x");
            /* Radix2DitParallel storage is the bit reversal of Radix2Dit's natural output */
            memcpy(y, x, sizeof(fr_t) * n);
            or_radix2dit_dft_batch(y, h, w);
            fr_t* z = (fr_t*)malloc(sizeof(fr_t) * n);
            memcpy(z, x, sizeof(fr_t) * n);
            or_r2dp_dft_batch(z, h, w);
            or_reverse_matrix_index_bits(z, h, w);
            CHECK(memcmp(y, z, sizeof(fr_t) * n) == 0, "Radix2DitParallel order");
            for (uint32_t b = 0; b <= 2 && lg + b <= 9; b++) {
                fr_t* o1 = (fr_t*)malloc(sizeof(fr_t) * (n << b));
                fr_t* o2 = (fr_t*)malloc(sizeof(fr_t) * (n << b));
                or_coset_lde_batch(x, o1, h, w, b, s);
                or_r2dp_coset_lde_batch(x, o2, h, w, b, s);
                or_reverse_matrix_index_bits(o2, h << b, w);
                CHECK(memcmp(o1, o2, sizeof(fr_t) * (n << b)) == 0, "coset_lde orders differ");
                /* get_evaluations_on_domain by Horner from the coefficients equals the LDE */
                if (lg <= 5) {
                    fr_t* c = (fr_t*)malloc(sizeof(fr_t) * n);
                    memcpy(c, x, sizeof(fr_t) * n);
                    or_idft_batch(c, h, w);
                    fr_t* o3 = (fr_t*)malloc(sizeof(fr_t) * (n << b));
                    or_kzg_evaluations_on_domain(c, h, w, lg + b, s, o3);
                    CHECK(memcmp(o1, o3, sizeof(fr_t) * (n << b)) == 0, "Horner LDE != coset LDE");
                    free(c);
                    free(o3);
                }
                free(o1);
                free(o2);
            }
            free(x);
            free(y);
            free(z);
        }
}

static void msm_checks(void) {
    g1_affine_t g;
    or_g1_generator(&g);
    CHECK(or_g1_on_curve(&g), "generator off the curve");
    const uint64_t ns[] = {0, 1, 2, 7, 64, 300};
    for (int k = 0; k < 6; k++) {
        const uint64_t n = ns[k];
        g1_affine_t* pts = (g1_affine_t*)malloc(sizeof(g1_affine_t) * (n ? n : 1));
        const fr_t alpha = or_fr_from_u64(12345);
        or_g1_srs(n, &alpha, pts);
        fr_t* s = rand_mat(n);
        g1_affine_t got, want;
        or_g1_msm(pts, s, n, &got);
        /* sum_i s_i alpha^i G = [f(alpha)] G */
        fr_t f = or_eval_poly_col(s, n, 1, 0, alpha);
        or_g1_mul(&g, &f, &want);
        CHECK(n == 0 ? (got.x[0] | got.y[0]) == 0 : memcmp(&got, &want, sizeof got) == 0, "MSM != [f(alpha)]G");
        free(pts);
        free(s);
    }
}

static void quotient_checks(void) {
    /* quotient_and_eval: f(X) = q(X)(X - z) + f(z), checked at a random point */
    for (uint64_t n = 1; n <= 33; n += 8) {
        fr_t* c = rand_mat(n);
        fr_t* q = (fr_t*)malloc(sizeof(fr_t) * n);
        fr_t z = rand_fr(), v, x = rand_fr();
        or_quotient_and_eval(c, n, 1, z, n > 1 ? q : NULL, &v);
        fr_t fz = or_eval_poly_col(c, n, 1, 0, z);
        CHECK(memcmp(&fz, &v, sizeof v) == 0, "quotient_and_eval value");
        if (n > 1) {
            fr_t fx = or_eval_poly_col(c, n, 1, 0, x), qx = or_eval_poly_col(q, n - 1, 1, 0, x), d, r;
            or_fr_sub(&x, &z, &d);
            or_fr_mul(&qx, &d, &r);
            or_fr_add(&r, &v, &r);
            CHECK(memcmp(&fx, &r, sizeof r) == 0, "f != q (X - z) + f(z)");
        }
        free(c);
        free(q);
    }
    /* barycentric evaluation of evaluations over H == Horner of the coefficients */
    for (uint32_t lg = 0; lg <= 5; lg++) {
        const uint64_t h = 1ull << lg, w = 3;
        fr_t* e = rand_mat(h * w);
        fr_t* c = (fr_t*)malloc(sizeof(fr_t) * h * w);
        memcpy(c, e, sizeof(fr_t) * h * w);
        or_idft_batch(c, h, w);
        fr_t pts[2] = {rand_fr(), rand_fr()}, out[6];
        or_bary_eval_cols(e, h, w, pts, 2, out);
        for (int p = 0; p < 2; p++)
            for (uint64_t col = 0; col < w; col++) {
                fr_t want = or_eval_poly_col(c, h, w, col, pts[p]);
                CHECK(memcmp(&out[p * w + col], &want, sizeof want) == 0, "barycentric != Horner");
            }
        free(e);
        free(c);
    }
    /* Poseidon2-AIR: trace, selectors and quotient on small shapes (VECTOR_LEN 1 and 2) */
    const uint32_t hf = 4, pr = 56;
    fr_t* rb = rand_mat(hf * 3);
    fr_t* rp = rand_mat(pr);
    fr_t* re = rand_mat(hf * 3);
    for (uint32_t vl = 1; vl <= 2; vl++)
        for (uint32_t lg = 1; lg <= 3; lg++) {
            const uint64_t h = 1ull << lg, cols = (uint64_t)or_p2_num_cols(hf, pr) * vl;
            fr_t* in = rand_mat(h * vl * 3);
            fr_t* tr = (fr_t*)malloc(sizeof(fr_t) * h * cols);
            or_p2_generate_trace(in, h * vl, vl, hf, pr, rb, rp, re, tr);
            const uint64_t q = h << 1;
            fr_t* lde = (fr_t*)malloc(sizeof(fr_t) * q * cols);
            or_coset_lde_batch(tr, lde, h, cols, 1, or_fr_from_u64(5));
            fr_t* sel = (fr_t*)malloc(sizeof(fr_t) * q * 4);
            or_selectors_on_coset(lg, lg + 1, or_fr_from_u64(5), sel, sel + q, sel + 2 * q, sel + 3 * q);
            fr_t* qv = (fr_t*)malloc(sizeof(fr_t) * q);
            or_p2_quotient_values(lde, lg, 1, vl, hf, pr, rb, rp, re, rand_fr(), qv);
            free(in);
            free(tr);
            free(lde);
            free(sel);
            free(qv);
        }
    free(rb);
    free(rp);
    free(re);
}

int main(void) {
    dft_checks();
    msm_checks();
    quotient_checks();
    if (fails) {
        fprintf(stderr, "asan_check: %d failed checks\n", fails);
        return 1;
    }
    printf("asan_check: ok\n");
    return 0;
}
