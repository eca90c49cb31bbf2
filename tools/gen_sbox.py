"""Derives a bitsliced AES S-box (GF(2^8) inversion in the tower field
GF(((2^2)^2)^2) plus the affine map) as a straight-line program of
AND / XOR / NOT gates, verifies it on all 256 inputs against the S-box
computed from its definition, and emits aby3_amd/csrc/aes_bs_sbox.h.

Tower: GF(4) = GF(2)[w]/(w^2+w+1); GF(16) = GF(4)[z]/(z^2+z+N);
GF(256) = GF(16)[y]/(y^2+y+M). For y^2 = y + M, the inverse of
a = ah*y + al is (ah*y + (ah+al)) * (ah^2*M + ah*al + al^2)^-1, and the same
formula one level down. The change of basis between the AES polynomial
basis and the tower basis is found by searching the AES field for roots of
the tower's defining polynomials.
"""
import itertools
import os
import sys

AES_POLY = 0x11B


def gmul(a, b):
    p = 0
    for _ in range(8):
        if b & 1:
            p ^= a
        hi = a & 0x80
        a = (a << 1) & 0xFF
        if hi:
            a ^= 0x1B
        b >>= 1
    return p


def ginv(a):
    if a == 0:
        return 0
    for b in range(1, 256):
        if gmul(a, b) == 1:
            return b


def sbox(x):
    inv = ginv(x)
    r = 0x63
    for i in range(8):
        bit = ((inv >> i) ^ (inv >> ((i + 4) % 8)) ^ (inv >> ((i + 5) % 8)) ^ (inv >> ((i + 6) % 8)) ^
               (inv >> ((i + 7) % 8))) & 1
        r ^= bit << i
    return r


# ---- tower arithmetic on integers (for the search / reference) -----------
def gf4_mul(a, b):  # a = a1 w + a0
    a1, a0, b1, b0 = a >> 1, a & 1, b >> 1, b & 1
    hi = (a1 & b1) ^ (a1 & b0) ^ (a0 & b1)
    lo = (a1 & b1) ^ (a0 & b0)
    return (hi << 1) | lo


def gf16_mul(a, b, N):  # a = ah z + al, z^2 = z + N
    ah, al, bh, bl = a >> 2, a & 3, b >> 2, b & 3
    hh = gf4_mul(ah, bh)
    hi = hh ^ gf4_mul(ah, bl) ^ gf4_mul(al, bh)
    lo = gf4_mul(hh, N) ^ gf4_mul(al, bl)
    return (hi << 2) | lo


def gf256t_mul(a, b, N, M):  # a = ah y + al, y^2 = y + M
    ah, al, bh, bl = a >> 4, a & 15, b >> 4, b & 15
    hh = gf16_mul(ah, bh, N)
    hi = hh ^ gf16_mul(ah, bl, N) ^ gf16_mul(al, bh, N)
    lo = gf16_mul(hh, M, N) ^ gf16_mul(al, bl, N)
    return (hi << 4) | lo


def find_tower():
    # N in GF(4) with z^2+z+N irreducible; M in GF(16) with y^2+y+M irreducible
    for N in range(1, 4):
        if all(gf4_mul(z, z) ^ z ^ N for z in range(4)):
            break
    for M in range(1, 16):
        if all(gf16_mul(y, y, N) ^ y ^ M for y in range(16)):
            break
    return N, M


def find_iso(N, M):
    """Field isomorphism phi: tower -> AES, as images of the 8 tower basis bits."""
    tow_gen_candidates = []
    # try every AES element g as the image of a tower generator: map tower element t -> AES
    # via the tower's multiplicative structure; simplest: find AES elements w_, z_, y_ with
    # w_^2+w_+1 = 0, z_^2+z_+N(w_) = 0, y_^2+y_+M(z_,w_) = 0, then basis images.
    def aes_of_gf4(c, w_):
        return (w_ if c & 2 else 0) ^ (1 if c & 1 else 0)

    def aes_of_gf16(c, w_, z_):
        return gmul(aes_of_gf4(c >> 2, w_), z_) ^ aes_of_gf4(c & 3, w_)

    for w_ in range(2, 256):
        if gmul(w_, w_) ^ w_ ^ 1:
            continue
        for z_ in range(2, 256):
            if gmul(z_, z_) ^ z_ ^ aes_of_gf4(N, w_):
                continue
            for y_ in range(2, 256):
                if gmul(y_, y_) ^ y_ ^ aes_of_gf16(M, w_, z_):
                    continue
                # tower bit b (0..7): bit layout [ah(4) | al(4)], each [h(2)|l(2)], each [1|0]
                imgs = []
                for b in range(8):
                    t = 1 << b
                    ah, al = t >> 4, t & 15
                    v = gmul(aes_of_gf16(ah, w_, z_), y_) ^ aes_of_gf16(al, w_, z_)
                    imgs.append(v)
                # check it is a bijection and a homomorphism on a few products
                def phi(t):
                    r = 0
                    for b in range(8):
                        if t >> b & 1:
                            r ^= imgs[b]
                    return r
                if len({phi(t) for t in range(256)}) != 256:
                    continue
                ok = all(phi(gf256t_mul(a, b, N, M)) == gmul(phi(a), phi(b))
                         for a, b in itertools.product(range(0, 256, 7), range(0, 256, 11)))
                if ok:
                    return imgs
    raise SystemExit("no isomorphism found")


def mat_from_images(imgs):
    """8x8 GF(2) matrix (rows = output bits) of the linear map with given images of unit vectors."""
    return [[(imgs[c] >> r) & 1 for c in range(8)] for r in range(8)]


def mat_inv(m):
    n = 8
    a = [row[:] + [1 if i == j else 0 for j in range(n)] for i, row in enumerate(m)]
    for c in range(n):
        p = next(r for r in range(c, n) if a[r][c])
        a[c], a[p] = a[p], a[c]
        for r in range(n):
            if r != c and a[r][c]:
                a[r] = [x ^ y for x, y in zip(a[r], a[c])]
    return [row[n:] for row in a]


def mat_mul(a, b):
    return [[sum(a[i][k] & b[k][j] for k in range(8)) & 1 for j in range(8)] for i in range(8)]


# ---- straight-line program builder -----------------------------------------
class Prog:
    def __init__(self):
        self.lines = []
        self.n = 0

    def tmp(self):
        self.n += 1
        return f"t{self.n}"

    def xor(self, a, b):
        if a == "0":
            return b
        if b == "0":
            return a
        t = self.tmp()
        self.lines.append(("^", t, a, b))
        return t

    def xorn(self, xs):
        xs = [x for x in xs if x != "0"]
        if not xs:
            return "0"
        r = xs[0]
        for x in xs[1:]:
            r = self.xor(r, x)
        return r

    def andg(self, a, b):
        if a == "0" or b == "0":
            return "0"
        t = self.tmp()
        self.lines.append(("&", t, a, b))
        return t

    def linear(self, m, ins):
        # common-subexpression-free linear layer (row by row)
        return [self.xorn([ins[c] for c in range(len(ins)) if m[r][c]]) for r in range(len(m))]


def paar(P, targets, ins):
    """Greedy common-subexpression XOR network (Paar): targets are bit masks
    over `ins`; repeatedly materialize the most shared pair."""
    sigs = list(ins)               # signal names
    rows = [set(i for i in range(len(ins)) if (m >> i) & 1) for m in targets]
    while True:
        best, cnt = None, 1
        counts = {}
        for r in rows:
            rl = sorted(r)
            for i in range(len(rl)):
                for j in range(i + 1, len(rl)):
                    k = (rl[i], rl[j])
                    counts[k] = counts.get(k, 0) + 1
        for k, c in counts.items():
            if c > cnt:
                best, cnt = k, c
        if best is None:
            break
        a, b = best
        sigs.append(P.xor(sigs[a], sigs[b]))
        new = len(sigs) - 1
        for r in rows:
            if a in r and b in r:
                r.discard(a)
                r.discard(b)
                r.add(new)
    return [P.xorn([sigs[i] for i in sorted(r)]) for r in rows]


def lin_masks(fn):
    """Bit masks (over the 8 input bits) of a GF(2)-linear byte function fn: int -> int."""
    cols = [fn(1 << c) for c in range(8)]
    return [sum(((cols[c] >> r) & 1) << c for c in range(8)) for r in range(8)]


def gf4_mul_p(P, a, b):  # a = (a1, a0)
    a1, a0 = a
    b1, b0 = b
    t = P.andg(a1, b1)
    # hi = a1b1 ^ a1b0 ^ a0b1 = (a1^a0)(b1^b0) ^ a0b0; lo = a1b1 ^ a0b0
    s = P.andg(P.xor(a1, a0), P.xor(b1, b0))
    u = P.andg(a0, b0)
    return (P.xor(s, u), P.xor(t, u))


def gf4_scale_p(P, a, c):  # multiply by constant c in GF(4) (linear)
    a1, a0 = a
    if c == 1:
        return a
    if c == 2:  # w*(a1 w + a0) = a1 (w+1) + a0 w = (a1^a0) w + a1
        return (P.xor(a1, a0), a1)
    if c == 3:  # (w+1) a = w a + a
        h, l = gf4_scale_p(P, a, 2)
        return (P.xor(h, a1), P.xor(l, a0))
    return ("0", "0")


def gf4_sq_p(P, a):  # (a1 w + a0)^2 = a1 w + (a1 ^ a0)
    a1, a0 = a
    return (a1, P.xor(a1, a0))


def gf4_add(P, a, b):
    return (P.xor(a[0], b[0]), P.xor(a[1], b[1]))


def gf16_mul_p(P, a, b, N):  # a = (ah, al) of GF(4) pairs
    ah, al = a
    bh, bl = b
    hh = gf4_mul_p(P, ah, bh)
    # Karatsuba: hi = (ah+al)(bh+bl) + al bl ; lo = hh*N + al bl
    ll = gf4_mul_p(P, al, bl)
    mm = gf4_mul_p(P, gf4_add(P, ah, al), gf4_add(P, bh, bl))
    hi = gf4_add(P, mm, ll)
    lo = gf4_add(P, gf4_scale_p(P, hh, N), ll)
    return (hi, lo)


def gf16_inv_p(P, a, N):
    ah, al = a
    # d = ah^2 N + ah al + al^2 ; inv = (ah, ah+al) * d^-1 ; d^-1 = d^2 in GF(4)
    d = gf4_add(P, gf4_add(P, gf4_scale_p(P, gf4_sq_p(P, ah), N), gf4_mul_p(P, ah, al)), gf4_sq_p(P, al))
    di = gf4_sq_p(P, d)
    return (gf4_mul_p(P, ah, di), gf4_mul_p(P, gf4_add(P, ah, al), di))


def gf16_add(P, a, b):
    return (gf4_add(P, a[0], b[0]), gf4_add(P, a[1], b[1]))


def main():
    N, M = find_tower()
    imgs = find_iso(N, M)
    T2A = mat_from_images(imgs)          # tower bits -> AES bits
    A2T = mat_inv(T2A)
    # affine map of the S-box: out = Aff * inv ^ 0x63
    aff = [[1 if ((c - r) % 8) in (0, 4, 5, 6, 7) else 0 for c in range(8)] for r in range(8)]
    OUT = mat_mul(aff, T2A)              # tower inverse bits -> S-box output bits (before ^0x63)

    P = Prog()
    x = [f"x[{i}]" for i in range(8)]

    def to_tower(v):  # AES byte -> tower bits (linear)
        r = 0
        for i in range(8):
            if v >> i & 1:
                r ^= sum(A2T[b][i] << b for b in range(8))
        return r

    def gf16_sq_int(a):
        return gf16_mul(a, a, N)

    # top linear layer, all as functions of the AES input bits:
    #   tower bits t (ah = t[7:4], al = t[3:0]); s = ah + al; dl = ah^2 M + al^2
    t_m = lin_masks(to_tower)
    s_m = lin_masks(lambda v: (to_tower(v) >> 4) ^ (to_tower(v) & 15))[:4]
    dl_m = lin_masks(lambda v: gf16_mul(gf16_sq_int(to_tower(v) >> 4), M, N) ^ gf16_sq_int(to_tower(v) & 15))[:4]
    top = paar(P, t_m + s_m + dl_m, x)
    t, sv, dl = top[:8], top[8:12], top[12:16]
    g4 = lambda b: ((b[3], b[2]), (b[1], b[0]))  # 4 bit names (LSB first) -> GF(16) pair of GF(4) pairs
    ah = g4(t[4:8])
    al = g4(t[0:4])
    ahal = g4(sv)
    # d = ah^2 M + al^2 + ah al
    d = gf16_add(P, g4(dl), gf16_mul_p(P, ah, al, N))
    di = gf16_inv_p(P, d, N)
    oh = gf16_mul_p(P, ah, di, N)
    ol = gf16_mul_p(P, ahal, di, N)
    inv_bits = [ol[1][1], ol[1][0], ol[0][1], ol[0][0], oh[1][1], oh[1][0], oh[0][1], oh[0][0]]
    out_masks = [sum(OUT[r][c] << c for c in range(8)) for r in range(8)]
    out = paar(P, out_masks, inv_bits)

    # constant 0x63: complement those output bits
    final = []
    for i in range(8):
        final.append((out[i], (0x63 >> i) & 1))

    # ---- verify by interpretation on all 256 inputs ----
    def run(v):
        env = {f"x[{i}]": (v >> i) & 1 for i in range(8)}
        env["0"] = 0
        for op, dst, a, b in P.lines:
            env[dst] = (env[a] & env[b]) if op == "&" else (env[a] ^ env[b])
        r = 0
        for i, (name, c) in enumerate(final):
            r |= ((env[name] ^ c) & 1) << i
        return r

    bad = [v for v in range(256) if run(v) != sbox(v)]
    if bad:
        raise SystemExit(f"S-box circuit wrong for {len(bad)} inputs, e.g. {bad[:4]}")
    n_and = sum(1 for l in P.lines if l[0] == "&")
    n_xor = len(P.lines) - n_and

    # ---- emit ----
    out_lines = [
        "// Generated by tools/gen_sbox.py -- do not edit. Bitsliced AES S-box:",
        f"// GF(((2^2)^2)^2) tower inversion (N = {N}, M = {M}) plus the affine map,",
        f"// {n_and} AND + {n_xor} XOR gates (+ NOTs folded from 0x63), verified on all 256 inputs.",
        "// x[0..7]: input bit planes (bit i of each byte, LSB first); y[0..7]: output planes.",
        "#pragma once",
        "#define ABY3G_AES_BS_SBOX(T, x, y) \\",
        "    do { \\",
    ]
    for op, dst, a, b in P.lines:
        out_lines.append(f"        const T {dst} = {a} {op} {b}; \\")
    for i, (name, c) in enumerate(final):
        val = name if name != "0" else "T(0)"
        out_lines.append(f"        y[{i}] = {'~' if c else ''}({val}); \\")
    out_lines.append("    } while (0)")
    dst = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "aby3_amd", "csrc",
                                                               "aes_bs_sbox.h")
    open(dst, "w").write("\n".join(out_lines) + "\n")
    print(f"ok: N={N} M={M} gates: {n_and} AND + {n_xor} XOR -> {dst}")


if __name__ == "__main__":
    main()
