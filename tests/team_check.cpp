// Host check of csrc/pairing_team.h (tests/test_pairing_team_host.py): the six lanes' COMPUTE halves,
// run one after another on published slots, against the tower's sequential Fq12 functions
// (pairing.h) on random elements.  Prints "ok <cases>" or the first mismatch and exits 1.
#include <cstdio>
#include <cstdlib>
#include <random>

#include "pairing_team.h"

using namespace eon;

static std::mt19937_64 rng(12345);

static Fq rand_fq() {
    Fq a = from_u64<FqP>(rng() | 1), b = from_u64<FqP>(rng() | 1), c = from_u64<FqP>(rng() | 1);
    return mul(mul(mul(a, b), mul(c, a)), from_u64<FqP>(rng()));
}

static Fq2 rand_fq2() { return {rand_fq(), rand_fq()}; }

static Fq12 rand_fq12() {
    Fq12 r;
    for (int k = 0; k < 6; k++) set_w_coef(r, k, rand_fq2());
    return r;
}

static bool eq12(const Fq12& a, const Fq12& b) {
    for (int k = 0; k < 6; k++)
        if (!f2_eq(w_coef(a, k), w_coef(b, k))) return false;
    return true;
}

struct Slots {
    Fq2 v[6], vx[6];
};

static Slots publish(const Fq12& a) {
    Slots s;
    for (int k = 0; k < 6; k++) {
        s.v[k] = w_coef(a, k);
        s.vx[k] = f2_mul_xi(s.v[k]);
    }
    return s;
}

static int fail(const char* what, int i) {
    std::printf("FAIL %s case %d\n", what, i);
    return 1;
}

int main(int argc, char** argv) {
    const int cases = argc > 1 ? std::atoi(argv[1]) : 50;
    for (int i = 0; i < cases; i++) {
        const Fq12 a = rand_fq12(), b = rand_fq12();
        const Slots sa = publish(a), sb = publish(b);
        Fq12 r;
        // products and squares
        for (int k = 0; k < 6; k++) set_w_coef(r, k, tm_mul(sa.v, sb.v, sb.vx, k));
        if (!eq12(r, f12_mul(a, b))) return fail("mul", i);
        for (int k = 0; k < 6; k++) set_w_coef(r, k, tm_mul(sa.v, sa.v, sa.vx, k));
        if (!eq12(r, f12_sqr(a))) return fail("sqr", i);
        // the Granger-Scott formula (an identity of formulas: any input)
        for (int k = 0; k < 6; k++) set_w_coef(r, k, tm_cyc_sqr(sa.v, k));
        if (!eq12(r, f12_cyc_sqr(a))) return fail("cyc_sqr", i);
        // a line l0 + l1 w + l3 w^3 and a vertical line l0 + l2 w^2
        const Fq2 l0 = rand_fq2(), l1 = rand_fq2(), l3 = rand_fq2();
        const int j3[3] = {0, 1, 3};
        const Fq2 v3[3] = {l0, l1, l3};
        for (int k = 0; k < 6; k++) set_w_coef(r, k, tm_sparse(sa.v, sa.vx, j3, v3, k));
        if (!eq12(r, f12_mul_line(a, l0, l1, l3))) return fail("line", i);
        const int j2[2] = {0, 2};
        const Fq2 v2[2] = {l0, l1};
        Fq12 vert = {f6_zero(), f6_zero()};
        vert.c0.c0 = l0;
        vert.c0.c1 = l1;
        for (int k = 0; k < 6; k++) set_w_coef(r, k, tm_sparse(sa.v, sa.vx, j2, v2, k));
        if (!eq12(r, f12_mul(a, vert))) return fail("vertical", i);
        // Frobenius maps and the conjugate
        for (int k = 0; k < 6; k++) set_w_coef(r, k, tm_frob<1>(w_coef(a, k), k));
        if (!eq12(r, f12_frob<1>(a))) return fail("frob1", i);
        for (int k = 0; k < 6; k++) set_w_coef(r, k, tm_frob<2>(w_coef(a, k), k));
        if (!eq12(r, f12_frob<2>(a))) return fail("frob2", i);
        for (int k = 0; k < 6; k++) set_w_coef(r, k, tm_frob<3>(w_coef(a, k), k));
        if (!eq12(r, f12_frob<3>(a))) return fail("frob3", i);
        for (int k = 0; k < 6; k++) set_w_coef(r, k, tm_conj(w_coef(a, k), k));
        if (!eq12(r, f12_conj(a))) return fail("conj", i);
    }
    std::printf("ok %d\n", cases);
    return 0;
}
