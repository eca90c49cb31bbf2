"""Protocol-level parity on the GPU, through the host runtime's C entry
points (include/aby3.h):

* aby3h_sim_*: one call by three parties on cuda:0 vs the CPU oracle on the
  same seeds and inputs, every party's shares bit-exact, at sizes the oracle
  finishes in seconds (ragged shapes, one row, the LR shapes, merges);
* aby3h_session_*: every bench job at BASELINE.json's sizes, checked through
  size-independent properties (the revealed product against exact
  arithmetic / the truncation bound; every MSB row; the LR model against a
  plaintext fixed-point restatement; the 2^20-key sort equal to std::sort).
"""
import numpy as np
import pytest

import oracle as orc
from aby3_amd import native as nt

pytestmark = pytest.mark.gpu


def rand(n, seed, bound=None):
    rng = np.random.default_rng(seed)
    if bound is None:
        return rng.integers(-(2**63), 2**63 - 1, size=n, dtype=np.int64, endpoint=True)
    return rng.integers(-bound, bound, size=n, dtype=np.int64)


MUL_CASES = [
    # mode, trunc, d, M, K, N
    (1, False, 0, 1, 1, 1),
    (1, False, 0, 33, 17, 65),
    (1, False, 0, 256, 128, 1),      # LR: xw = X_B w
    (0, False, 0, 128, 128, 128),    # C1 Hadamard
    (1, True, 16, 100, 70, 50),
    (1, True, 27, 128, 256, 1),      # LR: X_B^T err >> (D + aB)
    (0, True, 8, 31, 9, 1),
    (1, True, 16, 256, 256, 256),
    # empty shapes (Eigen's empty matrices in the reference): no rows, no
    # columns, and no inner dimension -- a zero product, then the truncation
    (1, False, 0, 0, 5, 7),
    (1, False, 0, 5, 7, 0),
    (1, True, 16, 5, 0, 7),
    (0, True, 8, 0, 3, 3),
]


@pytest.mark.parametrize("mode,trunc,d,M,K,N", MUL_CASES)
def test_mul_vs_oracle(gpu, mode, trunc, d, M, K, N):
    bound = (1 << 20) if trunc else None
    a = rand(M * K, M + K, bound)
    b = rand((K * N) if mode == 1 else (M * K), N + 7, bound)
    sh_g, plain_g = nt.sim.mul(mode, trunc, d, a, b, M, K, N)
    sh_o, plain_o = orc.sim_mul(mode, trunc, d, a, b, M, K, N)
    assert np.array_equal(sh_g, sh_o)
    assert np.array_equal(plain_g, plain_o)


@pytest.mark.parametrize("kind,n", [(0, 1), (0, 1000), (1, 257)])
def test_mul_bit_vs_oracle(gpu, kind, n):
    a = rand(n, 3)
    bits = np.random.default_rng(4).integers(0, 2, size=n).astype(np.int64)
    sh_g, p_g = nt.sim.mul_bit(kind, a, 0x1234567, bits)
    sh_o, p_o = orc.sim_mul_bit(kind, a, 0x1234567, bits)
    assert np.array_equal(sh_g, sh_o) and np.array_equal(p_g, p_o)


CIRCUITS = [("int_comp_helper", 64, 1), ("int_comp_helper", 64, 5000), ("int_int_lt", 64, 3000),
            ("int_eq", 64, 700), ("int_int_add", 64, 1000), ("int_int_sub", 64, 2048),
            ("bits_nor_helper", 64, 300), ("cmp_swap", 64, 2049), ("int_int_bitwiseOr", 16, 100)]


@pytest.mark.parametrize("name,bits,rows", CIRCUITS)
def test_circuit_vs_oracle(gpu, name, bits, rows):
    cir = nt.circuit(name, bits)
    ins = []
    for k, w in enumerate(cir["inputs"]):
        v = rand(rows, 10 + k)
        if len(w) < 64:
            v &= (1 << len(w)) - 1
        ins.append(v)
    shs_g, res_g = nt.sim.circuit(name, bits, 0, rows, ins)
    res_o, shs_o = orc.sim_circuit(cir, rows, ins, with_shares=True)
    for o in range(len(res_o)):
        assert np.array_equal(shs_g[o], shs_o[o]), f"output {o} shares"
        assert np.array_equal(res_g[o], res_o[o])


def test_circuit_file_vs_oracle(gpu, tmp_path):
    """An externally stored circuit (BetaCircuit binary file, "bin:" name)
    evaluated by the GPU engine, share-exact against the oracle."""
    path = str(tmp_path / "add64.bin")
    nt.circuit_write("int_int_add", path, 64)
    name = "bin:" + path
    cir = nt.circuit(name)
    ins = [rand(3001, 30), rand(3001, 31)]
    shs_g, res_g = nt.sim.circuit(name, 64, 0, 3001, ins)
    res_o, shs_o = orc.sim_circuit(cir, 3001, ins, with_shares=True)
    assert np.array_equal(shs_g[0], shs_o[0]) and np.array_equal(res_g[0], res_o[0])
    assert np.array_equal(res_g[0][:, 0], (ins[0].astype(np.uint64) + ins[1].astype(np.uint64)).astype(np.int64))


@pytest.mark.parametrize("kind,n,D", [(0, 256, 16), (0, 1, 16), (1, 500, 8)])
def test_piecewise_vs_oracle(gpu, kind, n, D):
    x = rand(n, 21, 3 << D)
    cir = nt.circuit("int_Sh3Piecewise_helper", 64, 2 if kind == 0 else 1)
    sh_g, p_g = nt.sim.piecewise(kind, x, D)
    sh_o, p_o = orc.sim_piecewise(kind, cir, x, D)
    assert np.array_equal(sh_g, sh_o) and np.array_equal(p_g, p_o)


def test_cipher_gt_vs_oracle(gpu):
    a, b = rand(4097, 30), rand(4097, 31)
    b[:10] = a[:10]  # equal keys: gt = 0
    sh_g, p_g = nt.sim.cipher_gt(a, b)
    p_o, sh_o = orc.sim_fetch_msb(nt.circuit("int_comp_helper", 64), a, b, with_shares=True)
    assert np.array_equal(sh_g, sh_o) and np.array_equal(p_g, p_o)


MERGE_CASES = [
    # mode, dim, list lengths
    (0, 0, [1, 1]),
    (0, 0, [8, 8]),                   # SortTest.cpp odd_even_merge
    (0, 0, [5, 7, 8, 3]),             # SortTest.cpp odd_even_multi_merge
    (0, 0, [64] * 8),
    (0, 0, [100, 3, 17, 250, 9]),     # odd count, unequal lengths (padding)
    (1, 0, [1] * 4096),               # the sort, 12 levels, 78 rounds
    (1, 0, [1] * 1000),               # sort of a non-power-of-two count
    (1, 0, [3, 1, 4, 1, 5, 9, 2, 6]),
    (2, 3, [16] * 12),                # high_dimensional_odd_even_multi_merge, 3 x 4 lists
    (2, 2, [4, 2, 3, 5, 1, 4]),       # 2 x 3 lists (odd k)
    (3, 4, [8] * 8),                  # high_dimensional_odd_even_merge, 4 dims
    (3, 2, [5, 9, 2, 2]),
    (4, 0, [5, 7, 8, 3]),             # the reference's sequential merge order (MergeOrder::Sequential)
    (4, 0, [100, 3, 17, 250, 9]),
    (4, 0, [64] * 8),
    (5, 3, [16] * 12),                # high-dimensional, sequential order
    (5, 2, [4, 2, 3, 5, 1, 4]),
]


@pytest.mark.parametrize("mode,dim,lens", MERGE_CASES)
def test_merge_vs_oracle(gpu, mode, dim, lens):
    """Every party's shares of the merged output equal the oracle's batched
    restatement (oracle/src/orc_sort.cpp), and the revealed lists are sorted."""
    rng = np.random.default_rng(sum(lens) + mode)
    lists = [np.sort(rng.integers(-(2**62), 2**62, size=n, dtype=np.int64)) for n in lens]
    p_g, sh_g = nt.sim.merge(lists, mode, dim, shares=True)
    p_o, sh_o = orc.sim_merge(nt.circuit("cmp_swap", 64), lists, mode, dim, with_shares=True)
    assert np.array_equal(sh_g, sh_o)
    assert np.array_equal(p_g, p_o)
    if mode in (2, 3, 5):
        k = len(lists) // dim
        exp = np.concatenate([np.sort(np.concatenate(lists[i * k:(i + 1) * k])) for i in range(dim)])
    else:
        exp = np.sort(np.concatenate(lists))
    assert np.array_equal(p_g, exp)


# ---- bench jobs at the BASELINE.json sizes --------------------------------
@pytest.mark.parametrize("job,params,steps", [
    (nt.JOB_MUL_TRUNC, [1024, 1024, 1024, 16, 1], 3),   # C2 GEMM + truncation
    (nt.JOB_MUL_TRUNC, [1024, 1024, 1024, 8, 0], 2),    # Hadamard + truncation, D8
    (nt.JOB_MUL, [128, 128, 128, 0], 3),                # C1 Hadamard
    (nt.JOB_MUL, [128, 128, 128, 1], 3),                # C1 GEMM
    (nt.JOB_MSB, [1 << 20], 2),                         # C3 every row checked
    (nt.JOB_LR, [100000, 128, 256, 16, 11], 20),        # C4 shapes (dataset trimmed)
    (nt.JOB_LR, [1000000, 128, 256, 16, 11], 20),       # C4 at its 10^6 x 128 dataset
    (nt.JOB_LR, [1000000, 128, 256, 16, 11, 1], 40),    # C4 with getSubset inside every step
    (nt.JOB_SORT, [1 << 20], 1),                        # C5 the whole 2^20-key sort, every key checked
    (nt.JOB_SORT, [777], 2),                            # sort of a ragged count
    (nt.JOB_SORT, [777, 1], 1),                         # the reference's sequential merge order
    (nt.JOB_SORT, [1 << 12, 1], 1),
    (nt.JOB_A2B, [1 << 20], 2),                         # toBinaryMatrix, every value checked
    (nt.JOB_A2B, [1000], 3),                            # ragged rows
    (nt.JOB_BITINJ, [1 << 16, 64], 2),                  # bitInjection, every bit checked
    (nt.JOB_BITINJ, [777, 13], 3),                      # ragged rows, 13 bits
])
def test_session_jobs(gpu, job, params, steps):
    with nt.Session(job, params, probe=False) as s:
        s.run(steps)
        assert s.check()
