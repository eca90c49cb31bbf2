"""Generates the golden fixtures of tests/golden/*.json with the CPU oracle.

The reference cannot be built here (libOTe/cryptoTools,
Eigen and Boost are absent and need the network), so the fixtures come from
the C++ restatement under oracle/, seeded exactly as the reference's unit
tests seed their parties: encryptor toBlock(0, i) / toBlock(0, i+1),
evaluator toBlock(1, i) / toBlock(1, i+1), party 0 owning every input.
Plaintext inputs are words of the cryptoTools PRNG(ZeroBlock) stream
(AES-CTR under the all-zero key), as the reference tests draw theirs.

What pins what:
  * "revealed" values are checked here against the reference tests'
    expectations (exact product, truncation bound, circuit semantics,
    sorted merge) before a fixture is written;
  * the per-party "shares" are pinned only by the Appendix A randomness
    restatement (AES checked against FIPS-197 and OpenSSL): at share level
    parity is unpinned by the reference itself, and the GPU path must
    reproduce them bit for bit.

Run: python tests/golden/make_golden.py   (after `make oracle host`)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.dirname(os.path.dirname(HERE))]

import oracle as orc  # noqa: E402
from aby3_amd import native as nt  # noqa: E402

ZERO = bytes(16)


class Stream:
    """PRNG(ZeroBlock).get<i64>() sequence."""

    def __init__(self):
        self.off = 0

    def i64(self, n):
        v = orc.prng_i64(ZERO, self.off, n)
        self.off += 8 * n
        return v


def L(a):
    return [int(x) for x in np.asarray(a).reshape(-1)]


def arith(st):
    out = {}
    for mode, name in ((1, "gemm_10x10"), (0, "hadamard_10x10")):
        a, b = st.i64(100), st.i64(100)
        sh, plain = orc.sim_mul(mode, False, 0, a, b, 10, 10, 10)
        am, bm = a.reshape(10, 10).astype(object), b.reshape(10, 10).astype(object)
        exp = (am @ bm) if mode == 1 else (am * bm)
        assert L(plain) == [((int(x) + 2**63) % 2**64) - 2**63 for x in exp.reshape(-1)]
        out[name] = dict(mode=mode, trunc=0, d=0, M=10, K=10, N=10, a=L(a), b=L(b), shares=L(sh), revealed=L(plain))
    # 4x4 fixed-point GEMM with truncation at D8 (matrixFixed_test): |x| < 2^20
    a, b = st.i64(16) % (1 << 21) - (1 << 20), st.i64(16) % (1 << 21) - (1 << 20)
    sh, plain = orc.sim_mul(1, True, 8, a, b, 4, 4, 4)
    e = (a.reshape(4, 4) @ b.reshape(4, 4)).reshape(-1) >> 8
    assert np.all(plain - e <= 1) and np.all(e - plain < 4)
    out["trunc_gemm_4x4_D8"] = dict(mode=1, trunc=1, d=8, M=4, K=4, N=4, a=L(a), b=L(b), shares=L(sh),
                                    revealed=L(plain))
    # shared x shared-bit and public x shared-bit (sh3_asyncArithBinMul_test / Pub)
    a, bits = st.i64(64), st.i64(64) & 1
    sh, plain = orc.sim_mul_bit(0, a, 0, bits)
    assert np.array_equal(plain, np.where(bits == 1, a, 0))
    out["mul_bit_64"] = dict(kind=0, a=L(a), apub=0, bits=L(bits), shares=L(sh), revealed=L(plain))
    apub = int(st.i64(1)[0])
    bits = st.i64(64) & 1
    sh, plain = orc.sim_mul_bit(1, np.zeros(64, np.int64), apub, bits)
    assert np.array_equal(plain, np.where(bits == 1, apub, 0))
    out["pub_mul_bit_64"] = dict(kind=1, a=L(np.zeros(64)), apub=apub, bits=L(bits), shares=L(sh), revealed=L(plain))
    return out


def binary(st):
    out = {}
    specs = [
        # (fixture, circuit, bits, rows, plaintext semantics) -- Sh3BinaryEvaluatorTests.cpp:333-424
        ("and8_256", "int_int_bitwiseAnd", 8, 256, lambda a, b: a & b),
        ("add8_256", "int_int_add", 8, 256, lambda a, b: (a + b) & 0xFF),
        ("msb64_256", "int_comp_helper", 64, 256,
         lambda a, b: ((a.view(np.uint64) + b.view(np.uint64)) >> np.uint64(63)).view(np.int64)),
    ]
    for fx, name, bits, rows, f in specs:
        a, b = st.i64(rows), st.i64(rows)
        if bits < 64:
            a, b = a & ((1 << bits) - 1), b & ((1 << bits) - 1)
        cir = nt.circuit(name, bits)
        res, shs = orc.sim_circuit(cir, rows, [a, b], with_shares=True)
        assert np.array_equal(res[0][:, 0], f(a, b)), fx
        out[fx] = dict(circuit=name, size=bits, param=0, rows=rows, gates=len(cir["gates"]), inputs=[L(a), L(b)],
                       shares=[L(s) for s in shs], revealed=[L(r) for r in res])
    # 16-value compare of BoolTest.cpp:21-300 / Test.cpp:74-191: x = i, y = 16 - i
    x = np.arange(16, dtype=np.int64)
    y = 16 - x
    for fx, name, f in (("lt64_16", "int_int_lt", lambda a, b: (a < b).astype(np.int64)),
                        ("eq64_16", "int_eq", lambda a, b: (a == b).astype(np.int64))):
        cir = nt.circuit(name, 64)
        res, shs = orc.sim_circuit(cir, 16, [y, x], with_shares=True)  # bool_cipher_lt(Y, X) = [y < x]
        assert np.array_equal(res[0][:, 0], f(y, x)), fx
        out[fx] = dict(circuit=name, size=64, param=0, rows=16, gates=len(cir["gates"]), inputs=[L(y), L(x)],
                       shares=[L(s) for s in shs], revealed=[L(r) for r in res])
    return out


def fetch_msb(st):
    x = np.arange(16, dtype=np.int64)
    y = 16 - x
    cir = nt.circuit("int_comp_helper", 64)
    plain, sh = orc.sim_fetch_msb(cir, x, y, with_shares=True)
    assert np.array_equal(plain & 1, (x > y).astype(np.int64))  # Test.cpp res_gt
    out = {"cipher_gt_16": dict(a=L(x), b=L(y), shares=L(sh), revealed=L(plain))}
    a, b = st.i64(128), st.i64(128)
    plain, sh = orc.sim_fetch_msb(cir, a, b, with_shares=True)
    d = (b.view(np.uint64) - a.view(np.uint64)) >> np.uint64(63)
    assert np.array_equal(plain.view(np.uint64), d)
    out["cipher_gt_128"] = dict(a=L(a), b=L(b), shares=L(sh), revealed=L(plain))
    return out


def piecewise(st):
    D = 16
    x = np.round(np.linspace(-1.5, 1.5, 64) * (1 << D)).astype(np.int64)  # Sh3PiecewiseTests.cpp:13-83
    cir = nt.circuit("int_Sh3Piecewise_helper", 64, 2)
    sh, plain = orc.sim_piecewise(0, cir, x, D)
    xf = x / float(1 << D)
    exp = np.where(xf < -0.5, 0.0, np.where(xf < 0.5, 0.5 + xf, 1.0))
    assert np.max(np.abs(plain / float(1 << D) - exp)) <= 2.0**-D
    return {"sigmoid_64_D16": dict(kind=0, D=D, x=L(x), shares=L(sh), revealed=L(plain))}


def merge(st):
    # SortTest.cpp:354-487: sorted lists merged; expected = std::sort of the union
    out = {}
    for fx, lens in (("merge_8_8", [8, 8]), ("multi_merge_5_7_8_3", [5, 7, 8, 3])):
        lists = [np.sort((st.i64(n).view(np.uint64) >> np.uint64(21)).view(np.int64)) for n in lens]
        out[fx] = dict(lists=[L(v) for v in lists], sorted=L(np.sort(np.concatenate(lists))))
    # share level: the batched network (aby3_amd/host/Sort.h) with the cmp_swap
    # circuit, the reference tests' seeds; a 16-key sort (mode 1) and a
    # two-dimensional multi-merge of odd list count (mode 2)
    cir = nt.circuit("cmp_swap", 64)
    for fx, mode, dim, lens in (("sort_16", 1, 0, [1] * 16), ("hd_multi_merge_2x3", 2, 2, [4, 2, 3, 5, 1, 4])):
        lists = [np.sort((st.i64(n).view(np.uint64) >> np.uint64(21)).view(np.int64)) for n in lens]
        plain, sh = orc.sim_merge(cir, lists, mode, dim, with_shares=True)
        if mode == 1:
            exp = np.sort(np.concatenate(lists))
        else:
            k = len(lens) // dim
            exp = np.concatenate([np.sort(np.concatenate(lists[i * k:(i + 1) * k])) for i in range(dim)])
        assert np.array_equal(plain, exp)
        out[fx] = dict(lists=[L(v) for v in lists], mode=mode, dim=dim, sorted=L(plain), shares=L(sh))
    return out


def lr():
    # C4 driver (main-logistic.cpp:82-140, Regression.h:24-58, 249-293): the
    # model, the first mini-batches getSubset draws over the 10^6-row dataset,
    # the dataset's first rows, and every party's w shares after 3 iterations
    # on the first 4096 rows (aby3ML seeds, the oracle's batches over 4096 rows)
    X, Y, model = orc.lr_dataset(4096, 128, 16)
    assert list(model[10:]) == [0.0] * 118 and all(abs(v) <= 9 for v in model[:10])
    b_full = orc.lr_batches(10**6, 256, 2)
    assert len(set(L(b_full))) == 512  # without replacement
    b = orc.lr_batches(4096, 256, 3)
    sh, w = orc.sim_lr(nt.circuit("int_Sh3Piecewise_helper", 64, 2), X, Y, b)
    # the revealed model moves along the planted one (first updates)
    assert np.sign(w[0]) == np.sign(model[0]) and np.sign(w[1]) == np.sign(model[1])
    return {"lr_4096x128_B256": dict(n=4096, d=128, B=256, D=16, aB=11, iters=3, model=[float(v) for v in model],
                                     batches_1e6=L(b_full), batches=L(b), x_rows01=L(X[:2]), y_head=L(Y[:64]),
                                     x_sum=int(X.sum()), y_sum=int(Y.sum()), w_shares=L(sh), w=L(w))}


def main():
    st = Stream()
    files = dict(arith=arith(st), binary=binary(st), fetch_msb=fetch_msb(st), piecewise=piecewise(st),
                 merge=merge(st), lr=lr())
    for name, data in files.items():
        path = os.path.join(HERE, f"{name}.json")
        with open(path, "w") as f:
            json.dump(data, f, separators=(",", ":"))
        print(path, os.path.getsize(path))


if __name__ == "__main__":
    main()
