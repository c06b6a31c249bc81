// CPU check of the prove driver's host Fr arithmetic (plonky3_eon_amd/host/fr_host.h): the
// portable u128 CIOS product, the MULX/ADCX/ADOX product, the lazy addition and the halving, on
// random operands and on operands at the edges of their contracts (< 2r).  Prints one line per
// case, "op a b out" in hex (4 little-endian u64 words each, comma-separated); the Python side
// (tests/test_fr_host.py) checks every line with big integers.
#include <stdio.h>
#include <stdlib.h>

#include <random>

#include "fr_host.h"

using namespace eon_host;

static void put(const char* op, const uint64_t* a, const uint64_t* b, const uint64_t* r) {
    printf("%s", op);
    for (const uint64_t* v : {a, b, r}) {
        printf(" %016llx,%016llx,%016llx,%016llx", (unsigned long long)v[0], (unsigned long long)v[1],
               (unsigned long long)v[2], (unsigned long long)v[3]);
    }
    printf("\n");
}

static bool below_2r(const uint64_t* v) {
    for (int i = 3; i >= 0; i--)
        if (v[i] != Fr::P2[i]) return v[i] < Fr::P2[i];
    return false;
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 1000;
    const bool adx = detail::kCpuAdx;
    std::mt19937_64 g(12345);
    // edge operands: 0, 1, r - 1, r, r + 1, 2r - 1, 2r - 2, all-ones below 2r
    uint64_t edges[8][4] = {{0, 0, 0, 0}, {1, 0, 0, 0}};
    for (int i = 0; i < 4; i++) {
        edges[2][i] = Fr::P[i];
        edges[3][i] = Fr::P[i];
        edges[4][i] = Fr::P[i];
        edges[5][i] = Fr::P2[i];
        edges[6][i] = Fr::P2[i];
    }
    edges[2][0] -= 1, edges[4][0] += 1, edges[5][0] -= 1, edges[6][0] -= 2;
    edges[7][0] = edges[7][1] = edges[7][2] = ~0ull;
    edges[7][3] = Fr::P2[3] - 1;
    for (int it = 0; it < n + 64; it++) {
        uint64_t a[4], b[4];
        if (it < 64) {
            for (int i = 0; i < 4; i++) a[i] = edges[it & 7][i], b[i] = edges[it >> 3][i];
        } else {
            do {
                for (int i = 0; i < 4; i++) a[i] = g(), b[i] = g();
                a[3] &= (it & 1) ? 0x3fffffffffffffffull : 0x7fffffffffffffffull;
                b[3] &= (it & 2) ? 0x3fffffffffffffffull : 0x7fffffffffffffffull;
            } while (!below_2r(a) || !below_2r(b));
        }
        uint64_t r[4];
        detail::mont_mul_lazy(a, b, r);
        put("mul", a, b, r);
        if (adx) {
            detail::mont_mul_adx(a, b, r);
            put("mul", a, b, r);
            detail::mont_sqr_adx(a, r);
            put("mul", a, a, r);
        }
        detail::add_lazy(a, b, r);
        put("add", a, b, r);
        const FrLazy h = lz_half(FrLazy{{a[0], a[1], a[2], a[3]}});
        put("half", a, b, h.l);
        if (!(a[3] >> 62)) {  // the canonical product (fr_mul) for inputs < 2r as well
            const Fr c = fr_mul(Fr{{a[0], a[1], a[2], a[3]}}, Fr{{b[0], b[1], b[2], b[3]}});
            put("fr_mul", a, b, c.l);
        }
    }
    fprintf(stderr, "adx=%d\n", (int)adx);
    return 0;
}
