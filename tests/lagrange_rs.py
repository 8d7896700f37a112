"""Reed-Solomon by Lagrange interpolation over Leopard's evaluation points: an independent
statement of the code klauspost/reedsolomon's Leopard encoder (v1.12.1, leopard8.go /
leopard.go) computes, with no FFT, no skew table and no
log/exp table of Leopard's own.

Leopard works in "Cantor representation": the element with representation r is
sum_b r_b * beta_b for the Cantor basis beta_0..beta_{n-1} (beta_0 = 1, beta_i^2 + beta_i =
beta_{i-1}) in the polynomial basis mod POLY. Its systematic encoder of m data symbols is
the polynomial P of degree < m through (w_{m+i}, data_i), evaluated at w_i for the m
parity symbols, where w_j is the element with representation j. tests/test_oracle.py
checks this statement against block 408's pinned GF(2^8) code and against the oracle's
GF(2^16) path (the field in which the reference holds no vector).
"""

CANTOR8 = (1, 214, 152, 146, 86, 200, 88, 230)
POLY8 = 0x11D
CANTOR16 = (0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
            0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E)
POLY16 = 0x1002D


class Field:
    """GF(2^bits) in the polynomial basis mod poly, with Cantor-representation maps."""

    def __init__(self, bits, poly, cantor):
        n = 1 << bits
        self.to_poly = [0] * n
        for r in range(n):
            p = 0
            for b in range(bits):
                if r >> b & 1:
                    p ^= cantor[b]
            self.to_poly[r] = p
        self.from_poly = [0] * n
        for r, p in enumerate(self.to_poly):
            self.from_poly[p] = r
        self.n = n
        self.exp = [0] * (2 * n)
        self.log = [0] * n
        x = 1
        for i in range(n - 1):
            self.exp[i] = x
            self.log[x] = i
            x <<= 1
            if x & n:
                x ^= poly
        for i in range(n - 1, 2 * n):
            self.exp[i] = self.exp[i - (n - 1)]

    def mul(self, a, b):
        return 0 if a == 0 or b == 0 else self.exp[self.log[a] + self.log[b]]

    def inv(self, a):
        return self.exp[(self.n - 1) - self.log[a]]


def encode(field, data):
    """Parity of the m data symbols `data` (Cantor representations, a list), m a power of
    two: P through (w_{m+i}, data_i), evaluated at w_0..w_{m-1}. O(m^2)."""
    m = len(data)
    xs = [field.to_poly[m + i] for i in range(m)]
    ys = [field.to_poly[v] for v in data]
    # barycentric weights 1 / prod_{j != i} (x_i - x_j) (subtraction is xor)
    cw = []
    for i in range(m):
        d = 1
        for j in range(m):
            if j != i:
                d = field.mul(d, xs[i] ^ xs[j])
        cw.append(field.mul(ys[i], field.inv(d)))
    out = []
    for t in range(m):
        x = field.to_poly[t]
        L = 1
        for xj in xs:
            L = field.mul(L, x ^ xj)
        s = 0
        for i in range(m):
            s ^= field.mul(cw[i], field.mul(L, field.inv(x ^ xs[i])))
        out.append(field.from_poly[s])
    return out
