// Host-side driver for tests/test_field29_host.py: runs the radix-2^29 products of
// plonky3_eon_amd/csrc/field29.h (their host instantiation: the same C++ with the plain
// multiply-add in place of the inline asm) on operands at the edges of their documented
// contracts -- limbs up to the largest allowed width, values up to the largest allowed product --
// and prints operands and results as 29-bit limbs for the Python side to check against big
// integers: r = a b 2^-261 (mod p), r < 2p, r normalised.  A column sum that overflowed 64 bits
// would show up as a wrong residue.
#include <cstdio>
#include <cstdlib>

#include "field29.h"

using namespace eon;

static uint64_t rng_state = 0x243F6A8885A308D3ull;
static uint64_t next64() {  // splitmix64
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// a random value below K p in normalised limbs (value drawn limb by limb below the top limb of
// K p, so it stays below K p up to the top-limb granularity handled by `below`)
template <class M>
static F29 random_below(uint32_t K) {
    constexpr KP29<M, 1> p1{};
    uint64_t kp[9];
    uint64_t c = 0;
    for (int i = 0; i < 9; i++) {
        c += (uint64_t)p1.l[i] * K;
        kp[i] = c & M29;
        c >>= 29;
    }
    F29 r;
    const bool edge = (next64() & 3) == 0;  // all low limbs at their maximum
    for (int i = 0; i < 8; i++) r.l[i] = edge ? M29 : (uint32_t)(next64() & M29);
    r.l[8] = (uint32_t)(next64() % kp[8]);  // top limb below K p's: value < K p
    return r;
}

// the same value with its low limbs widened: limb i gains k 2^29 and limb i + 1 loses k, while
// the widened limb stays below 2^(29 + extra_bits)
static F29 widen(F29 a, int extra_bits) {
    for (int i = 0; i < 8; i++) {
        if ((next64() & 3) == 0) continue;
        uint32_t k = 1 + (uint32_t)(next64() % ((1u << extra_bits) - 1));
        while (k && (a.l[i + 1] < k || (((uint64_t)a.l[i] + ((uint64_t)k << 29)) >> (29 + extra_bits)))) k--;
        a.l[i] += k << 29;
        a.l[i + 1] -= k;
    }
    return a;
}

static void put(const F29& a) {
    for (int i = 0; i < 9; i++) printf("%s%x", i ? "," : "", a.l[i]);
    printf(" ");
}

// the uniform-operand forms (SGPR operands on the device) compute the same columns
static void same(const F29& x, const F29& y, const char* what) {
    for (int i = 0; i < 9; i++)
        if (x.l[i] != y.l[i]) {
            fprintf(stderr, "%s differs from its VGPR form\n", what);
            exit(1);
        }
}

template <class M>
static void run(const char* name, int trials) {
    for (int t = 0; t < trials; t++) {
        // mul29 / sqr29: limbs < 2^30, values < 12p (a b < 144 p^2 < 0.99 p 2^261)
        const F29 a = widen(random_below<M>(12), 1), b = widen(random_below<M>(12), 1);
        printf("%s mul ", name);
        put(a);
        put(b);
        put(mul29<M>(a, b));
        printf("\n%s sqr ", name);
        put(a);
        put(sqr29<M>(a));
        // mul29_sum2: a, c, d normalised, b limbs < 2^31; the curve formulas' widest case
        // a < 6p, b < 11p, c < 4p, d < 2p
        const F29 s_a = random_below<M>(6), s_b = widen(random_below<M>(11), 2);
        const F29 s_c = random_below<M>(4), s_d = random_below<M>(2);
        printf("\n%s sum2 ", name);
        put(s_a);
        put(s_b);
        put(s_c);
        put(s_d);
        put(mul29_sum2<M>(s_a, s_b, s_c, s_d));
        printf("\n");
        same(mul29_sum2_u<M>(s_a, s_b, s_c, s_d), mul29_sum2<M>(s_a, s_b, s_c, s_d), "mul29_sum2_u");
    }
}

// mul29_shoup (the NTT's twiddle product) and shoup_pair29 (its table entries): T < p canonical,
// y any normalised value < 2^261 (all limbs at 2^29 - 1 on the edge draws)
static void run_shoup(int trials) {
    for (int t = 0; t < trials; t++) {
        const F29 T = random_below<FrP>(1);
        F29 y;
        const bool edge = (next64() & 3) == 0;
        for (int i = 0; i < 9; i++) y.l[i] = edge ? M29 : (uint32_t)(next64() & M29);
        F29 w, wq;
        shoup_pair29<FrP>(T, w, wq);
        printf("fr shoup ");
        put(T);
        put(y);
        put(w);
        put(wq);
        put(mul29_shoup<FrP>(y, w, wq));
        printf("\n");
        same(mul29_shoup_u<FrP>(y, w, wq), mul29_shoup<FrP>(y, w, wq), "mul29_shoup_u");
    }
}

int main(int argc, char** argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 2000;
    run<FqP>("fq", trials);
    run<FrP>("fr", trials);
    run_shoup(trials);
    return 0;
}
