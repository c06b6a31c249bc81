// See transcript.h.
#include "transcript.h"

#include <cstring>

#include "pcs.h"

namespace eon_host {

namespace {

// BN254 base field q: the G1 coordinates of eon_g1_affine are Montgomery
// residues x * 2^256 mod q
constexpr uint64_t Q[4] = {0x3c208c16d87cfd47ull, 0x97816a916871ca8dull, 0xb85045b68181585dull,
                           0x30644e72e131a029ull};
constexpr uint64_t Q_INV = 0x87d20782e4866389ull;  // -q^-1 mod 2^64

bool geq(const uint64_t a[4], const uint64_t b[4]) {
    for (int i = 3; i >= 0; i--)
        if (a[i] != b[i]) return a[i] > b[i];
    return true;
}

void sub_in_place(uint64_t a[4], const uint64_t b[4]) {
    unsigned __int128 br = 0;
    uint64_t borrow = 0;
    for (int i = 0; i < 4; i++) {
        br = (unsigned __int128)a[i] - b[i] - borrow;
        a[i] = (uint64_t)br;
        borrow = (uint64_t)(br >> 64) & 1;
    }
}

// a * 2^-256 mod q (Montgomery form -> canonical integer): REDC of a 4-word value
void fq_from_mont(const uint64_t a[4], uint64_t out[4]) {
    uint64_t t[5] = {a[0], a[1], a[2], a[3], 0};
    for (int i = 0; i < 4; i++) {
        const uint64_t m = t[0] * Q_INV;
        unsigned __int128 c = (unsigned __int128)m * Q[0] + t[0];
        c >>= 64;
        for (int j = 1; j < 4; j++) {
            c += (unsigned __int128)m * Q[j] + t[j];
            t[j - 1] = (uint64_t)c;
            c >>= 64;
        }
        c += t[4];
        t[3] = (uint64_t)c;
        t[4] = (uint64_t)(c >> 64);
    }
    std::memcpy(out, t, 32);
    if (t[4] || geq(out, Q)) sub_in_place(out, Q);
}

template <bool ADX>
FrLazy sbox(const FrLazy& x) {  // x^5
    const FrLazy x2 = lz_sqr<ADX>(x);
    return lz_mul<ADX>(lz_sqr<ADX>(x2), x);
}

void mds_light(FrLazy s[3]) {  // external.rs:128-133
    const FrLazy t = lz_add(lz_add(s[0], s[1]), s[2]);
    for (int i = 0; i < 3; i++) s[i] = lz_add(s[i], t);
}

void matmul_internal(FrLazy s[3]) {  // bn254/src/poseidon2.rs:55-63
    const FrLazy t = lz_add(s[0], lz_add(s[1], s[2]));
    s[0] = lz_add(s[0], t);
    s[1] = lz_add(s[1], t);
    s[2] = lz_add(lz_add(s[2], s[2]), t);
}

}  // namespace

Fr fr_add(const Fr& a, const Fr& b) {
    // canonical inputs < r < 2^254: the sum fits in 256 bits
    Fr s;
    unsigned __int128 c = 0;
    for (int i = 0; i < 4; i++) {
        c += (unsigned __int128)a.l[i] + b.l[i];
        s.l[i] = (uint64_t)c;
        c >>= 64;
    }
    detail::cond_sub(s.l, Fr::P);
    return s;
}

Poseidon2Bn254::Poseidon2Bn254(const eon_poseidon2_constants& c) : hf_(c.half_full_rounds) {
    if ((hf_ && (!c.beginning || !c.ending)) || (c.partial_rounds && !c.partial))
        throw Error(EON_E_ARG, "null Poseidon2 round constants");
    for (uint32_t i = 0; i < 3 * hf_; i++) {
        begin_.push_back(FrLazy::of(Fr::from_abi(c.beginning[i])));
        end_.push_back(FrLazy::of(Fr::from_abi(c.ending[i])));
    }
    for (uint32_t i = 0; i < c.partial_rounds; i++) partial_.push_back(FrLazy::of(Fr::from_abi(c.partial[i])));
    for (const auto* v : {&begin_, &end_, &partial_})
        for (const FrLazy& x : *v)
            if (geq(x.l, Fr::P)) throw Error(EON_E_ARG, "Poseidon2 round constant is not a canonical Fr");
}

template <bool ADX>
void Poseidon2Bn254::permute_impl(Fr st[3]) const {
    // every intermediate stays below 2r (fr_host.h: FrLazy); the state is canonical again at the end
    FrLazy s[3] = {FrLazy::of(st[0]), FrLazy::of(st[1]), FrLazy::of(st[2])};
    mds_light(s);  // external_initial_permute_state (external.rs:321-336)
    for (uint32_t r = 0; r < hf_; r++) {
        for (int i = 0; i < 3; i++) s[i] = sbox<ADX>(lz_add(s[i], begin_[3 * r + i]));
        mds_light(s);
    }
    // internal_permute_state (internal.rs:70-84): s0 <- (s0 + rc)^5, then [2,1,1;1,2,1;1,1,3] s.
    // Only s0 is a dependent chain, so the round is re-associated to keep one addition on it:
    // with v = x^5 and p = s1 + s2, s0' = 2v + p = x^4 (2x) + p and the next round's input is
    // s0' + rc' = x^4 (2x) + (p + rc'); v itself (for s1' = s1 + v + p, s2' = 2 s2 + v + p) is
    // 2v halved beside the chain.  Same field values, so bit-identical after canonicalisation.
    if (!partial_.empty()) {
        FrLazy x = lz_add(s[0], partial_[0]);
        for (size_t r = 0; r < partial_.size(); r++) {
            const FrLazy p = lz_add(s[1], s[2]);
            const FrLazy x2 = lz_sqr<ADX>(x), xd = lz_add(x, x);
            const FrLazy x4 = lz_sqr<ADX>(x2);
            const FrLazy v2 = lz_mul<ADX>(x4, xd), v = lz_half(v2);
            const FrLazy t = lz_add(v, p);
            s[1] = lz_add(s[1], t);
            s[2] = lz_add(lz_add(s[2], s[2]), t);
            if (r + 1 < partial_.size())
                x = lz_add(v2, lz_add(p, partial_[r + 1]));
            else
                s[0] = lz_add(v2, p);
        }
    }
    for (uint32_t r = 0; r < hf_; r++) {  // external_terminal_permute_state (external.rs:288-306)
        for (int i = 0; i < 3; i++) s[i] = sbox<ADX>(lz_add(s[i], end_[3 * r + i]));
        mds_light(s);
    }
    for (int i = 0; i < 3; i++) st[i] = s[i].canonical();
}

void Poseidon2Bn254::permute(Fr st[3]) const {
    if (detail::kCpuAdx)
        permute_impl<true>(st);
    else
        permute_impl<false>(st);
}

void DuplexChallenger::duplexing() {
    // duplex_challenger.rs:79-92: the buffered inputs overwrite the first elements of the state
    for (size_t i = 0; i < in_.size(); i++) state_[i] = in_[i];
    in_.clear();
    perm_.permute(state_);
    out_.assign(state_, state_ + RATE);
}

void DuplexChallenger::observe(const Fr& v) {
    out_.clear();  // duplex_challenger.rs:111-121
    in_.push_back(v);
    if (in_.size() == (size_t)RATE) duplexing();
}

Fr DuplexChallenger::sample() {
    if (!in_.empty() || out_.empty()) duplexing();  // duplex_challenger.rs:191-200
    const Fr v = out_.back();
    out_.pop_back();
    return v;
}

void DuplexChallenger::observe_g1(const eon_g1_affine* points, uint64_t n) {
    uint8_t b[32];
    for (uint64_t i = 0; i < n; i++) {
        g1_to_bytes(points[i], b);
        for (int c = 0; c < 4; c++) {
            uint64_t v = 0;
            for (int k = 0; k < 8; k++) v |= (uint64_t)b[8 * c + k] << (8 * k);
            observe(fr_from_u64(v));
        }
    }
}

void g1_to_bytes(const eon_g1_affine& p, uint8_t out[32]) {
    bool inf = true;
    for (int i = 0; i < 4; i++) inf = inf && p.x[i] == 0 && p.y[i] == 0;
    std::memset(out, 0, 32);
    if (inf) {
        out[31] = 0x40;
        return;
    }
    uint64_t x[4], y[4];
    fq_from_mont(p.x, x);
    fq_from_mont(p.y, y);
    for (int i = 0; i < 4; i++)
        for (int k = 0; k < 8; k++) out[8 * i + k] = (uint8_t)(x[i] >> (8 * k));
    if (y[0] & 1) out[31] |= 0x80;
}

}  // namespace eon_host
