"""Pins both oracles (oracle/pyoracle.py and the C restatement oracle/eon_oracle.c) against the
known-answer tests the reference holds for the hot path (CPU only)."""

import numpy as np
import pytest

from oracle import coracle as C
from oracle import pyoracle as O


def to_np(mat):
    return np.array([[O.int_to_limbs(O.to_mont(x)) for x in row] for row in mat], dtype=np.uint64)


def from_np(arr):
    return [[O.from_mont(O.limbs_to_int(e)) for e in row] for row in arr]


# ---- Fr (bn254/src/field.rs) -----------------------------------------------------------------
def test_fr_constants():
    # ONE, TWO, NEG_ONE, GENERATOR in Montgomery form (bn254/src/field.rs:256-281, 372-377)
    assert O.int_to_limbs(O.to_mont(1)) == (0xAC96341C4FFFFFFB, 0x36FC76959F60CD29, 0x666EA36F7879462E, 0x0E0A77C19A07DF2F)
    assert O.int_to_limbs(O.to_mont(2)) == (0x592C68389FFFFFF6, 0x6DF8ED2B3EC19A53, 0xCCDD46DEF0F28C5C, 0x1C14EF83340FBE5E)
    assert O.int_to_limbs(O.to_mont(O.P - 1)) == (0x974BC177A0000006, 0xF13771B2DA58A367, 0x51E1A2470908122E, 0x2259D6B14729C0FA)
    assert O.int_to_limbs(O.to_mont(5)) == (0x1B0D0EF99FFFFFE6, 0xEABA68A3A32A913F, 0x47D8EB76D8DD0689, 0x15D0085520F5BBC3)
    # R^2 and mu (bn254/src/field.rs:40-53)
    assert O.R * O.R % O.P == O.limbs_to_int((0x1BB8E645AE216DA7, 0x53FE3AB1E35C59E3, 0x8C49833D53BB8085, 0x0216D0B17F4E44A5))
    assert (0x3D1E0A6C10000001 * O.P) % 2**64 == 1
    # TWO_ADIC_GENERATOR = 5^((P-1)/2^28) (bn254/src/field.rs:553-561), order 2^28
    assert O.TWO_ADIC_GENERATOR == pow(5, (O.P - 1) >> 28, O.P)
    assert pow(O.TWO_ADIC_GENERATOR, 1 << 27, O.P) == O.P - 1
    # C oracle agrees (monty_mul restatement of bn254/src/helpers.rs)
    assert tuple(int(x) for x in C.fr_from_u64(5)) == O.int_to_limbs(O.to_mont(5))
    g = C.lib().or_two_adic_generator(28)
    assert tuple(g.v) == O.TWO_ADIC_GENERATOR_MONT


def test_bn254fr_kat():
    # test_bn254fr (bn254/src/field.rs:585-628): from_biguint reduces mod p, 2^256-1 = NEG_ONE + R
    assert (100 + O.P) * 3 % O.P == 300 % O.P
    assert (2**256 - 1) % O.P == (O.P - 1 + O.R_MOD_P) % O.P


def test_fr_mul_c_vs_python():
    a = C.random_fr(1, 2000)
    b = C.random_fr(2, 2000)
    r = np.empty_like(a)
    C.lib().or_fr_mul_batch(C._ptr(a), C._ptr(b), C._ptr(r), a.shape[0])
    for i in range(0, 2000, 7):
        x, y = O.limbs_to_int(a[i]), O.limbs_to_int(b[i])
        assert O.limbs_to_int(r[i]) == x * y * pow(O.R, -1, O.P) % O.P


# ---- DFT KATs (dft/src/naive.rs:34-105, dft/src/util.rs:38-154) -----------------------------
def test_naive_dft_kat():
    # columns 5+4x, 2+3x, 0 evaluate on {1,-1} to (9,5,0), (1,-1,0)
    mat = [[5, 2, 0], [4, 3, 0]]
    want = [[9, 5, 0], [1, O.P - 1, 0]]
    assert O.dft(mat) == want
    assert from_np(C.dft_batch(to_np(mat))) == want


def test_dft_roundtrips():
    m = O.random_matrix(1, 8, 3)
    assert O.idft(O.dft(m)) == m
    assert O.coset_idft(O.coset_dft(m, O.GENERATOR), O.GENERATOR) == m


def test_divide_by_height_and_coset_shift_kats():
    assert O.divide_by_height([[2, 4], [6, 8]]) == [[1, 2], [3, 4]]
    assert O.divide_by_height([[10, 20, 30, 40]]) == [[10, 20, 30, 40]]
    with pytest.raises(AssertionError):
        O.divide_by_height([[1], [2], [3]])
    assert O.coset_shift_cols([[1, 2], [3, 4], [5, 6]], 2) == [[1, 2], [6, 8], [20, 24]]
    assert O.coset_shift_cols([[7, 8], [9, 10]], 1) == [[7, 8], [9, 10]]


def test_bitrev_table_kat():
    # matrix/src/bitrev.rs:109-149
    assert [O.reverse_bits_len(i, 3) for i in range(8)] == [0, 4, 2, 6, 1, 5, 3, 7]
    assert O.bit_reverse_rows([[i] for i in range(8)]) == [[0], [4], [2], [6], [1], [5], [3], [7]]


@pytest.mark.parametrize("log_h,w", [(0, 1), (1, 2), (3, 3), (5, 2), (6, 1)])
def test_c_oracle_matches_python_oracle(log_h, w):
    m = O.random_matrix(11 + log_h, 1 << log_h, w)
    x = to_np(m)
    s = O.GENERATOR
    sl = O.int_to_limbs(O.to_mont(s))
    assert from_np(C.dft_batch(x)) == O.dft(m)
    assert from_np(C.idft_batch(x)) == O.idft(m)
    assert from_np(C.coset_dft_batch(x, sl)) == O.coset_dft(m, s)
    assert from_np(C.coset_idft_batch(x, sl)) == O.coset_idft(m, s)
    for b in (0, 1, 2):
        assert from_np(C.coset_lde_batch(x, b, sl)) == O.coset_lde(m, b, s)
    # Radix2DitParallel's own schedule lands in bit-reversed storage
    assert from_np(C.r2dp_dft_batch(x)) == O.bit_reverse_rows(O.dft(m))
    for b in (0, 1, 2):
        assert from_np(C.r2dp_coset_lde_batch(x, b, sl)) == O.bit_reverse_rows(O.coset_lde(m, b, s))
