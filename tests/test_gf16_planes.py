"""The arithmetic behind the GF(2^16) bit-plane kernels (celestia-app_amd/csrc/rs_decode_gf16.hip),
checked on the CPU against the field itself (tests/lagrange_rs.py: Leopard's GF(2^16) in Cantor
representation, klauspost/reedsolomon v1.12.1 leopard.go):

- a product by c as masked xors of bit planes with the basis products P_i = c * b_i;
- the tower basis b_i = prod of gamma_k = beta_{2^k} over the set bits k of i, in which a
  product by an element of the Cantor subfield GF(2^(2^J)) (representation < 2^(2^J)) maps each
  block of 2^J coordinates onto itself (the kernels skip the other masks).
"""
import random

import pytest

from lagrange_rs import CANTOR16, POLY16, Field


@pytest.fixture(scope="module")
def f16():
    return Field(16, POLY16, CANTOR16)


def mul_rep(f, a, b):
    """Product of two elements given by their Cantor representations."""
    return f.from_poly[f.mul(f.to_poly[a], f.to_poly[b])]


@pytest.fixture(scope="module")
def tower(f16):
    v = []
    for i in range(16):
        x = 1
        for k in range(4):
            if i >> k & 1:
                x = mul_rep(f16, x, 1 << (1 << k))
        v.append(x)
    tinv = [0] * 65536
    seen = [False] * 65536
    for c in range(65536):
        r = 0
        for i in range(16):
            if c >> i & 1:
                r ^= v[i]
        assert not seen[r], "the tower elements are not a basis"
        seen[r] = True
        tinv[r] = c
    return v, tinv


def planes_of(symbols):
    """16 bit planes of 32 symbols: plane i bit s = bit i of symbol s."""
    return [sum(((y >> i) & 1) << s for s, y in enumerate(symbols)) for i in range(16)]


def symbols_of(planes):
    return [sum(((planes[i] >> s) & 1) << i for i in range(16)) for s in range(32)]


def masked_xor_product(planes, pk):
    """Plane j of c*y = xor of the planes i of y whose basis product P_i has bit j set."""
    out = [0] * 16
    for i in range(16):
        for j in range(16):
            if pk[i] >> j & 1:
                out[j] ^= planes[i]
    return out


def test_bitplane_product_is_the_field_product(f16):
    rng = random.Random(5)
    for _ in range(20):
        c = rng.randrange(65536)
        ys = [rng.randrange(65536) for _ in range(32)]
        pk = [mul_rep(f16, c, 1 << i) for i in range(16)]
        got = symbols_of(masked_xor_product(planes_of(ys), pk))
        assert got == [mul_rep(f16, c, y) for y in ys]


@pytest.mark.parametrize("J", [0, 1, 2, 3, 4])
def test_tower_blocks(f16, tower, J):
    v, tinv = tower
    rng = random.Random(J)
    size = 1 << J
    for _ in range(30):
        c = rng.randrange(1 << size) if J < 4 else rng.randrange(65536)
        for i in range(16):
            p = tinv[mul_rep(f16, c, v[i])]
            block = ((1 << size) - 1) << ((i >> J) << J)
            assert p & ~block == 0, (J, c, i)


def test_tower_product_through_planes(f16, tower):
    """Scale into tower planes (P_i = T(c * e_i)), multiply by a subfield twiddle there
    (block-diagonal masks only), unscale back to Cantor planes (P_i = c' * b_i): the
    kernels' sequence gives the field product."""
    v, tinv = tower
    rng = random.Random(11)
    for J in (2, 3, 4):
        for _ in range(5):
            c1, c2 = rng.randrange(1, 65536), rng.randrange(1, 65536)
            w = rng.randrange(1 << (1 << J)) if J < 4 else rng.randrange(65536)
            ys = [rng.randrange(65536) for _ in range(32)]
            pl = masked_xor_product(planes_of(ys), [tinv[mul_rep(f16, c1, 1 << i)] for i in range(16)])
            tw = [tinv[mul_rep(f16, w, v[i])] for i in range(16)]
            out = [0] * 16
            for i in range(16):
                for j in range(16):
                    if (i >> J) == (j >> J) and tw[i] >> j & 1:
                        out[j] ^= pl[i]
            back = masked_xor_product(out, [mul_rep(f16, c2, v[i]) for i in range(16)])
            want = [mul_rep(f16, c2, mul_rep(f16, w, mul_rep(f16, c1, y))) for y in ys]
            assert symbols_of(back) == want
