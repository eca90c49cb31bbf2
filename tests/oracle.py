"""ctypes wrapper of the CPU oracle (oracle/build/liborc.so).

TEST INFRASTRUCTURE ONLY: the oracle is the checker. Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_int, c_int64, c_uint32, c_uint64, c_void_p

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORC_LIB = os.path.join(ROOT, "oracle", "build", "liborc.so")

_dll = None


def dll():
    global _dll
    if _dll is None:
        if not os.path.exists(ORC_LIB):
            raise RuntimeError(f"{ORC_LIB} missing: run `make oracle`")
        d = ctypes.CDLL(ORC_LIB)
        d.orc_last_error.restype = c_char_p
        _dll = d
    return _dll


def _p(a: np.ndarray):
    return a.ctypes.data_as(c_void_p)


def _check(rc):
    if rc != 0:
        raise RuntimeError("oracle: " + dll().orc_last_error().decode())


def to_block(hi: int, lo: int) -> bytes:
    """cryptoTools toBlock(hi, lo) = LE64(lo) || LE64(hi)."""
    return (lo & (2**64 - 1)).to_bytes(8, "little") + (hi & (2**64 - 1)).to_bytes(8, "little")


def aes_ref(key: bytes, block: bytes) -> bytes:
    out = ctypes.create_string_buffer(16)
    _check(dll().orc_aes_ref_encrypt(key, block, out))
    return out.raw


def aes_ctr(key: bytes, base: int, n: int, use_ref: bool = False) -> np.ndarray:
    out = np.zeros(2 * n, dtype=np.uint64)
    _check(dll().orc_aes_ctr(key, c_uint64(base), c_uint64(n), _p(out), int(use_ref)))
    return out


def prng_bytes(seed: bytes, off: int, n: int) -> bytes:
    out = ctypes.create_string_buffer(max(n, 1))
    _check(dll().orc_prng_bytes(seed, c_uint64(off), c_uint64(n), out))
    return out.raw[:n]


def prng_i64(seed: bytes, off: int, n: int) -> np.ndarray:
    return np.frombuffer(prng_bytes(seed, off, 8 * n), dtype=np.int64).copy()


def share_draws(kind: int, kprev: bytes, knext: bytes, base: int, n: int):
    o0 = np.zeros(n, dtype=np.int64)
    o1 = np.zeros(n, dtype=np.int64)
    _check(dll().orc_share_draws(kind, kprev, knext, c_uint64(base), c_uint64(n), _p(o0), _p(o1)))
    return o0, o1


def party_keys(prev_seed: bytes, next_seed: bytes):
    """(kSharePrev, kShareNext, kOtPrev, kOtNext) of Sh3ShareGen/Sh3Evaluator::init."""
    out = ctypes.create_string_buffer(64)
    _check(dll().orc_party_keys(prev_seed, next_seed, out))
    r = out.raw
    return r[0:16], r[16:32], r[32:48], r[48:64]


def local_product(mode: int, A0, A1, B0, B1, M, K, N) -> np.ndarray:
    C = np.zeros(M * N, dtype=np.int64)
    arrs = [np.ascontiguousarray(x, dtype=np.int64) for x in (A0, A1, B0, B1)]
    _check(dll().orc_local_product(mode, *[_p(a) for a in arrs], c_uint64(M), c_uint64(K), c_uint64(N), _p(C)))
    return C


def trunc_tuple(next_seed: bytes, next_off: int, prev_seed: bytes, prev_off: int, n: int, d: int):
    R = np.zeros(n, dtype=np.int64)
    RT0 = np.zeros(n, dtype=np.int64)
    RT1 = np.zeros(n, dtype=np.int64)
    _check(dll().orc_trunc_tuple(next_seed, c_uint64(next_off), prev_seed, c_uint64(prev_off), c_uint64(n),
                                 c_uint64(d), _p(R), _p(RT0), _p(RT1)))
    return R, RT0, RT1


def sim_mul(mode: int, trunc: bool, d: int, a: np.ndarray, b: np.ndarray, M: int, K: int, N: int):
    n = M * N if mode == 1 else M * K  # Hadamard: C is M x K
    shares = np.zeros(6 * n, dtype=np.int64)
    plain = np.zeros(n, dtype=np.int64)
    a = np.ascontiguousarray(a, dtype=np.int64)
    b = np.ascontiguousarray(b, dtype=np.int64)
    _check(dll().orc_sim_mul(mode, int(trunc), c_uint64(d), _p(a), _p(b), c_uint64(M), c_uint64(K), c_uint64(N),
                             _p(shares), _p(plain)))
    return shares.reshape(3, 2, n), plain


def sim_mul_bit(kind: int, a: np.ndarray, apub: int, bits: np.ndarray):
    n = len(bits)
    shares = np.zeros(6 * n, dtype=np.int64)
    plain = np.zeros(n, dtype=np.int64)
    a = np.ascontiguousarray(a, dtype=np.int64)
    bits = np.ascontiguousarray(bits, dtype=np.int64)
    _check(dll().orc_sim_mul_bit(kind, _p(a), c_int64(apub), _p(bits), c_uint64(n), _p(shares), _p(plain)))
    return shares.reshape(3, 2, n), plain


def _cir_args(cir):
    """cir: dict with wires, gates (n x 4 uint32), levels, inputs (list of lists), outputs."""
    gates = np.ascontiguousarray(np.asarray(cir["gates"], dtype=np.uint32).reshape(-1, 4))
    levels = np.ascontiguousarray(np.asarray(cir["levels"], dtype=np.uint32))
    inw = np.ascontiguousarray(np.concatenate([np.asarray(b, dtype=np.uint32) for b in cir["inputs"]]))
    ins = np.asarray([len(b) for b in cir["inputs"]], dtype=np.uint32)
    outw = np.ascontiguousarray(np.concatenate([np.asarray(b, dtype=np.uint32) for b in cir["outputs"]]))
    outs = np.asarray([len(b) for b in cir["outputs"]], dtype=np.uint32)
    keep = (gates, levels, inw, ins, outw, outs)
    args = [c_uint32(cir["wires"]), _p(gates), c_uint64(len(gates)), _p(levels), c_uint64(len(levels)), _p(inw),
            _p(ins), c_uint64(len(ins)), _p(outw), _p(outs), c_uint64(len(outs))]
    return args, keep


def sim_circuit(cir, rows: int, inputs: list[np.ndarray], with_shares: bool = False):
    args, keep = _cir_args(cir)
    ins = np.ascontiguousarray(np.concatenate([np.asarray(x, dtype=np.int64).reshape(-1) for x in inputs]))
    out_cols = [(len(b) + 63) // 64 for b in cir["outputs"]]
    outs = np.zeros(rows * sum(out_cols), dtype=np.int64)
    sh = np.zeros(6 * rows * sum(out_cols), dtype=np.int64) if with_shares else None
    _check(dll().orc_sim_circuit(*args, c_uint64(rows), _p(ins), _p(outs), _p(sh) if with_shares else None))
    res, off = [], 0
    for c in out_cols:
        res.append(outs[off:off + rows * c].reshape(rows, c))
        off += rows * c
    if with_shares:
        shs, off = [], 0
        for c in out_cols:
            shs.append(sh[off:off + 6 * rows * c].reshape(3, 2, rows * c))
            off += 6 * rows * c
        return res, shs
    return res


def sim_piecewise(kind: int, cir, x: np.ndarray, D: int):
    args, keep = _cir_args(cir)
    n = len(x)
    x = np.ascontiguousarray(x, dtype=np.int64)
    shares = np.zeros(6 * n, dtype=np.int64)
    plain = np.zeros(n, dtype=np.int64)
    _check(dll().orc_sim_piecewise(kind, *args, _p(x), c_uint64(n), c_uint64(D), _p(shares), _p(plain)))
    return shares.reshape(3, 2, n), plain


def sim_fetch_msb(cir, a: np.ndarray, b: np.ndarray, with_shares: bool = False):
    """cipher_gt(a, b) = MSB(b - a) through fetch_msb (BuildingBlocks.cpp:464-532)."""
    args, keep = _cir_args(cir)
    n = len(a)
    a = np.ascontiguousarray(a, dtype=np.int64)
    b = np.ascontiguousarray(b, dtype=np.int64)
    out = np.zeros(n, dtype=np.int64)
    sh = np.zeros(6 * n, dtype=np.int64)
    _check(dll().orc_sim_fetch_msb(*args, _p(a), _p(b), c_uint64(n), _p(out), _p(sh)))
    return (out, sh.reshape(3, 2, n)) if with_shares else out


def sim_merge(cir, lists, mode: int = 0, dim: int = 0, with_shares: bool = False):
    """The batched merge network (orc_sim_merge): mode 0 odd_even_multi_merge
    of separately shared lists, 1 all keys shared as one matrix, 2
    high_dimensional_odd_even_multi_merge ([dim][k] lists, flattened), 3
    high_dimensional_odd_even_merge, 4 / 5 mode 0 / 2 in the reference's
    sequential merge order. cir: the cmp_swap(64) circuit."""
    args, keep = _cir_args(cir)
    lens = np.asarray([len(x) for x in lists], dtype=np.uint64)
    keys = np.ascontiguousarray(np.concatenate([np.asarray(x, dtype=np.int64) for x in lists]))
    n = len(keys)
    out = np.zeros(n, dtype=np.int64)
    sh = np.zeros(6 * n, dtype=np.int64)
    _check(dll().orc_sim_merge(*args, c_int(mode), _p(lens), c_uint64(len(lists)), c_uint64(dim), _p(keys), _p(out),
                               _p(sh)))
    return (out, sh.reshape(3, 2, n)) if with_shares else out


def lr_dataset(n: int, dim: int = 128, D: int = 16):
    """The oracle's LogisticModelGen restatement: (X [n][dim], Y [n], model [dim])."""
    X = np.zeros((n, dim), dtype=np.int64)
    Y = np.zeros(n, dtype=np.int64)
    m = np.zeros(dim, dtype=np.float64)
    _check(dll().orc_lr_dataset(c_uint64(n), c_uint64(dim), c_uint64(D), _p(X), _p(Y), _p(m)))
    return X, Y, m


def lr_label_margin(n: int, dim: int = 128) -> float:
    """min over the C4 dataset's first n rows of |X m + noise| over twice the
    summation-order error bound of X m: > 1 means every label is the same
    under any summation order (the reference's Eigen GEMV included)."""
    out = ctypes.c_double(0)
    _check(dll().orc_lr_label_margin(c_uint64(n), c_uint64(dim), ctypes.byref(out)))
    return out.value


def lr_batches(n: int, B: int = 256, iters: int = 1):
    """The oracle's getSubset restatement: the first `iters` mini-batches [iters][B]."""
    out = np.zeros((iters, B), dtype=np.uint64)
    _check(dll().orc_lr_batches(c_uint64(n), c_uint64(B), c_uint64(iters), _p(out)))
    return out


def sim_lr(cir, X, Y, batches, D: int = 16, aB: int = 11):
    """SGD_Logistic iterations on the oracle (aby3ML seeds, party 0 shares X, Y,
    w = 0); cir: the int_Sh3Piecewise_helper(64, 2) circuit. Returns
    (w shares [3][2][d], revealed w)."""
    args, keep = _cir_args(cir)
    X = np.ascontiguousarray(X, dtype=np.int64)
    Y = np.ascontiguousarray(Y, dtype=np.int64).reshape(-1)
    batches = np.ascontiguousarray(batches, dtype=np.uint64)
    n, d = X.shape
    iters, B = batches.shape
    sh = np.zeros(6 * d, dtype=np.int64)
    w = np.zeros(d, dtype=np.int64)
    u = c_uint64
    _check(dll().orc_sim_lr(*args, u(n), u(d), u(B), u(D), u(aB), u(iters), _p(X), _p(Y), _p(batches), _p(sh),
                            _p(w)))
    return sh.reshape(3, 2, d), w


def shuffle_permutation(n: int, seed: bytes) -> np.ndarray:
    """get_permutation(n, seed) (BoolBasic.cpp:925-934)."""
    out = np.zeros(n, dtype=np.uint64)
    _check(dll().orc_shuffle_permutation(c_uint64(n), seed, _p(out)))
    return out.astype(np.int64)


def sim_shuffle(x: np.ndarray, mode: int = 0):
    """The shuffles of Shuffle.cpp by three parties (encryptor seeds
    toBlock(0, i)); x [len][unit]. Returns (shares [3][2][len*unit], revealed
    [len][unit], permutation shares [3][2][len] or None)."""
    x = np.ascontiguousarray(np.asarray(x, dtype=np.int64).reshape(len(x), -1))
    n, unit = x.shape
    sh = np.zeros(6 * n * unit, dtype=np.int64)
    plain = np.zeros(n * unit, dtype=np.int64)
    pi = np.zeros(6 * n, dtype=np.int64) if mode == 2 else None
    _check(dll().orc_sim_shuffle(c_int(mode), _p(x), c_uint64(n), c_uint64(unit), _p(sh),
                                 _p(pi) if pi is not None else None, _p(plain)))
    return sh.reshape(3, 2, -1), plain.reshape(n, unit), (pi.reshape(3, 2, -1) if pi is not None else None)


def reference_shuffle_order(n: int, c: int = 0):
    """The expected result of shuffle_test (aby3_tests/Test.cpp:305-340) for
    encryptor seeds toBlock(c, i): party 0's permutation list {next, prev,
    party 1's next} combined (BoolBasic.cpp:946-961); returns final_permutation
    (the scattering plain_permutate puts unit i at final[i])."""
    perms = [shuffle_permutation(n, to_block(c, 1)), shuffle_permutation(n, to_block(c, 0)),
             shuffle_permutation(n, to_block(c, 2))]
    final = np.arange(n, dtype=np.int64)
    for p in reversed(perms):
        inv = np.empty(n, dtype=np.int64)
        inv[p] = np.arange(n)
        tmp = np.empty(n, dtype=np.int64)
        tmp[inv] = final
        final = tmp
    return final
