"""rand 0.9's `SmallRng` and the reference's `Distribution<Fr>`, restated (TEST INFRASTRUCTURE).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline / input generation may import
this; the product path never does.

The reference seeds every random parameter of the path with `SmallRng::seed_from_u64(s)`
(workspace `Cargo.toml:72`: rand 0.9.0 with `small_rng`):
  * Poseidon2-AIR round constants: `RoundConstants::from_rng` (poseidon2-air/src/constants.rs:37-46)
  * Poseidon2-AIR trace inputs: `generate_trace_rows` draws `[F; WIDTH]` from SmallRng(1)
    (poseidon2-air/src/air.rs:60-80)
  * the challenger's permutation: `Poseidon2::new_from_rng` (poseidon2/src/lib.rs:66-75,
    poseidon2/src/external.rs:199-214), e.g. `new_from_rng(4, 22, SmallRng(1))` in
    eon-uni-stark/tests/fib_air.rs:113-115.

rand 0.9 is a crates.io dependency absent from /root/reference, so its published algorithm is
restated here:
  * `SmallRng` on 64-bit targets is Xoshiro256++ (rand/src/rngs/small.rs); `seed_from_u64` fills
    the four state words with SplitMix64 outputs (rand/src/rngs/xoshiro256plusplus.rs).
  * `next_u32` is the HIGH half of `next_u64` (the low bits of xoshiro have linear dependencies).
  * `u8: StandardUniform` is `next_u32() as u8` (rand/src/distr/integer.rs), and `[T; N]` is
    sampled element by element (rand/src/distr/other.rs), so `rng.random::<[u8; 32]>()` consumes
    32 `next_u64` calls and keeps bits 32..39 of each.
  * `Distribution<Fr> for StandardUniform` (bn254/src/field.rs:534-551): 32 such bytes, top two bits
    of byte 31 cleared, accepted when the little-endian value is < P by `from_bytes_monty`
    (bn254/src/field.rs:168-185), which takes it as the MONTGOMERY form.

Pinned by the published Xoshiro256++ vector (rand_xoshiro's test of state (1, 2, 3, 4), first
output 5·2^23 + 1 by hand) in tests/test_smallrng.py; the Fr/constant streams built on it carry no
reference-held output vector (no Rust toolchain here), so the bytes-to-Fr step rests on reading
field.rs.
"""

from __future__ import annotations

M64 = (1 << 64) - 1


def _rotl(x: int, k: int) -> int:
    return ((x << k) | (x >> (64 - k))) & M64


def splitmix64_fill(seed: int, n: int = 4) -> list[int]:
    """`seed_from_u64`'s state fill: n SplitMix64 outputs from `seed` (PHI = 0x9e3779b97f4a7c15)."""
    s = seed & M64
    out = []
    for _ in range(n):
        s = (s + 0x9E3779B97F4A7C15) & M64
        z = s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        out.append(z ^ (z >> 31))
    return out


class SmallRng:
    """Xoshiro256++ (rand 0.9 `SmallRng` on 64-bit platforms)."""

    def __init__(self, state: list[int]):
        assert len(state) == 4 and any(state), "xoshiro256++ state must be four words, not all zero"
        self.s = [w & M64 for w in state]

    @classmethod
    def seed_from_u64(cls, seed: int) -> "SmallRng":
        return cls(splitmix64_fill(seed))

    def next_u64(self) -> int:
        s = self.s
        result = (_rotl((s[0] + s[3]) & M64, 23) + s[0]) & M64
        t = (s[1] << 17) & M64
        s[2] ^= s[0]
        s[3] ^= s[1]
        s[1] ^= s[2]
        s[0] ^= s[3]
        s[2] ^= t
        s[3] = _rotl(s[3], 45)
        return result

    def next_u32(self) -> int:
        return self.next_u64() >> 32

    def random_u8(self) -> int:
        return self.next_u32() & 0xFF

    def random_bytes32(self) -> bytes:
        """`rng.random::<[u8; 32]>()`: one `next_u32` per byte."""
        return bytes(self.random_u8() for _ in range(32))

    def fr_mont(self) -> int:
        """One `StandardUniform` Fr sample, returned as its Montgomery residue (field.rs:534-551)."""
        from .pyoracle import P

        while True:
            b = bytearray(self.random_bytes32())
            b[31] &= (1 << 6) - 1
            v = int.from_bytes(b, "little")
            if v < P:
                return v

    def fr(self) -> int:
        """One `StandardUniform` Fr sample, canonical value."""
        from .pyoracle import from_mont

        return from_mont(self.fr_mont())


def round_constants_from_rng(rng: SmallRng, hf: int = 4, pr: int = 56, width: int = 3):
    """`RoundConstants::from_rng` (poseidon2-air/src/constants.rs:37-46): beginning full rounds
    ([F; WIDTH] each), partial rounds, ending full rounds -- as (begin, partial, end) canonical."""
    begin = [[rng.fr() for _ in range(width)] for _ in range(hf)]
    partial = [rng.fr() for _ in range(pr)]
    end = [[rng.fr() for _ in range(width)] for _ in range(hf)]
    return begin, partial, end


def poseidon2_new_from_rng(rng: SmallRng, rounds_f: int, rounds_p: int, width: int = 3):
    """`Poseidon2::new_from_rng(rounds_f, rounds_p, rng)` (poseidon2/src/lib.rs:66-75): the external
    layer's initial then terminal constants (`ExternalLayerConstants::new_from_rng`,
    poseidon2/src/external.rs:199-214, rounds_f / 2 arrays each), then rounds_p internal constants.
    Returned in the (begin, partial, end) layout the permutation restatements take."""
    assert rounds_f % 2 == 0, "The total number of external rounds should be even"
    half = rounds_f // 2
    initial = [[rng.fr() for _ in range(width)] for _ in range(half)]
    terminal = [[rng.fr() for _ in range(width)] for _ in range(half)]
    internal = [rng.fr() for _ in range(rounds_p)]
    return initial, internal, terminal


def trace_inputs(num_hashes: int, seed: int = 1, width: int = 3):
    """`generate_trace_rows`'s inputs (poseidon2-air/src/air.rs:70-71): `num_hashes` draws of
    `[F; WIDTH]` from SmallRng(seed), canonical values."""
    rng = SmallRng.seed_from_u64(seed)
    return [[rng.fr() for _ in range(width)] for _ in range(num_hashes)]
