// Host transcript microbenchmark (VERDICT r03 "next" 1): the headline prove's Fiat-Shamir work --
// observe 1312 trace-column commitments (kzg/src/pcs.rs:417-436) and sample alpha -- through
// libeonprove.so's eon_challenger, plus the bare Poseidon2 permutation rate.
//
//   hipcc -O2 -std=c++17 -Iinclude tools/ubench_transcript.cpp -Lplonky3_eon_amd -leonprove \
//         -Wl,-rpath,$PWD/plonky3_eon_amd -o build/ubench_transcript && build/ubench_transcript
#include <stdint.h>
#include <stdio.h>

#include <chrono>
#include <vector>

#include "eon_prove.h"

static uint64_t rng_state = 0x243f6a8885a308d3ull;
static uint64_t rnd() {  // splitmix64
    uint64_t z = (rng_state += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
static eon_fr rnd_fr() {  // < 2^253 < r
    eon_fr f;
    for (int i = 0; i < 4; i++) f.l[i] = rnd();
    f.l[3] &= 0x0fffffffffffffffull;
    return f;
}

int main(int argc, char** argv) {
    const int n_commit = argc > 1 ? atoi(argv[1]) : 1312;
    std::vector<eon_fr> beg(4 * 3), part(56), end(4 * 3);
    for (auto& x : beg) x = rnd_fr();
    for (auto& x : part) x = rnd_fr();
    for (auto& x : end) x = rnd_fr();
    eon_poseidon2_constants c{4, 56, beg.data(), part.data(), end.data()};
    std::vector<eon_g1_affine> pts(n_commit);
    for (auto& p : pts) {
        eon_fr a = rnd_fr(), b = rnd_fr();
        for (int i = 0; i < 4; i++) p.x[i] = a.l[i], p.y[i] = b.l[i];
    }
    using clk = std::chrono::steady_clock;
    double best_abs = 1e30, best_perm = 1e30;
    for (int rep = 0; rep < 7; rep++) {
        eon_challenger* ch = nullptr;
        if (eon_challenger_create(&c, &ch)) return 1;
        eon_fr out;
        const auto t0 = clk::now();
        if (eon_challenger_observe_g1(ch, pts.data(), pts.size()) || eon_challenger_sample(ch, &out)) return 2;
        const double ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
        best_abs = ms < best_abs ? ms : best_abs;
        eon_challenger_destroy(ch);

        eon_fr s[3] = {rnd_fr(), rnd_fr(), rnd_fr()};
        const int np = 2000;
        const auto t1 = clk::now();
        for (int i = 0; i < np; i++) eon_poseidon2_bn254_permute(&c, s);
        const double us = std::chrono::duration<double, std::micro>(clk::now() - t1).count() / np;
        best_perm = us < best_perm ? us : best_perm;
    }
    printf("{\"commitments\": %d, \"absorb_and_sample_ms\": %.3f, \"permute_us\": %.3f}\n", n_commit, best_abs,
           best_perm);
    return 0;
}
