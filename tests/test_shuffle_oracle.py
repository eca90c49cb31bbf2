"""The oracle's restatement of aby3-Basic/Shuffle.cpp on CPU, pinned by the
reference's own shuffle test (aby3_tests/Test.cpp:262-450): the revealed
shuffle equals the input permuted by combine_permutation of the parties'
permutation lists, and the permutation shares of
efficient_shuffle_with_random_permutation reveal that same permutation."""
import numpy as np
import pytest

import oracle as orc


def units(n, unit, seed):
    rng = np.random.default_rng(seed)
    return rng.integers(-2**63, 2**63, size=(n, unit), dtype=np.int64)


def test_permutation_is_a_permutation():
    p = orc.shuffle_permutation(1000, orc.to_block(0, 1))
    assert sorted(p.tolist()) == list(range(1000))
    assert orc.shuffle_permutation(1, orc.to_block(0, 1)).tolist() == [0]


@pytest.mark.parametrize("n,unit", [(1, 1), (2, 1), (16, 1), (16, 4), (100, 3), (1025, 1)])
def test_shuffle_matches_reference_test(n, unit):
    x = units(n, unit, n + unit)
    final = orc.reference_shuffle_order(n)
    expect = np.empty_like(x)
    expect[final] = x  # plain_permutate(final_permutation, shuffle_res) (Test.cpp:335-340)
    for mode in (0, 2):
        sh, plain, pi = orc.sim_shuffle(x, mode)
        assert np.array_equal(plain, expect), f"mode {mode}"
        if mode == 2:
            # revealed permutation shares = final_permutation (Test.cpp:382-410)
            assert np.array_equal(pi[0, 0] ^ pi[1, 0] ^ pi[2, 0], final)


def test_shuffle_test_inputs():
    """TEST_SIZE units holding their index (Test.cpp:286-292)."""
    n, unit = 20, 5
    x = np.repeat(np.arange(n, dtype=np.int64)[:, None], unit, axis=1)
    _, plain, _ = orc.sim_shuffle(x, 0)
    final = orc.reference_shuffle_order(n)
    assert np.array_equal(plain[final, 0], np.arange(n))


@pytest.mark.parametrize("n", [1, 5, 300])
def test_row_shuffle_is_a_permutation(n):
    """efficient_shuffle(sbMatrix) (Shuffle.cpp:229-385): no reference test
    pins its order; its output is the input under the parties' gathering
    permutations."""
    x = units(n, 1, 7 + n)
    sh, plain, _ = orc.sim_shuffle(x, 1)
    assert sorted(plain[:, 0].tolist()) == sorted(x[:, 0].tolist())
    # the X path composes P0's gathers (next, then prev) and P1's next; the Y
    # path (P1's prev, P2's next, P2's prev) uses the same three seeds in the
    # same order: toBlock(0, 1), toBlock(0, 0), toBlock(0, 2)
    order = np.arange(n)
    for k in (1, 0, 2):
        order = order[orc.shuffle_permutation(n, orc.to_block(0, k))]
    assert np.array_equal(plain[:, 0], x[order, 0])
