"""The 3-party shuffle (aby3-Basic/Shuffle.cpp) on the GPU engine against
the oracle's restatement, share for share, in all four forms (the reference's
vector<sbMatrix> and sbMatrix forms, the shuffle with the permutation's
shares, and the packed units the engine runs them on); at 2^20 units the
packed form is checked against the reference test's expected order
(aby3_tests/Test.cpp:305-340) computed from the parties' permutations."""
import numpy as np
import pytest

import oracle as orc
from aby3_amd import native as nt

pytestmark = pytest.mark.gpu


def units(n, unit, seed):
    rng = np.random.default_rng(seed)
    return rng.integers(-2**63, 2**63, size=(n, unit), dtype=np.int64)


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
@pytest.mark.parametrize("n,unit", [(1, 1), (2, 1), (7, 3), (1000, 1), (4097, 2)])
def test_shuffle_vs_oracle(gpu, mode, n, unit):
    if mode == 1 and unit != 1:
        pytest.skip("the sbMatrix form shuffles one word per row")
    x = units(n, unit, 100 * n + unit)
    sh_g, plain_g, pi_g = nt.sim.shuffle(x, mode)
    sh_o, plain_o, pi_o = orc.sim_shuffle(x, 0 if mode == 3 else mode)
    assert np.array_equal(sh_g, sh_o), "shares"
    assert np.array_equal(plain_g, plain_o)
    if mode == 2:
        assert np.array_equal(pi_g, pi_o), "permutation shares"


def test_shuffle_2_20_units(gpu):
    n = 1 << 20
    x = units(n, 1, 5)
    _, plain, _ = nt.sim.shuffle(x, 3)
    final = orc.reference_shuffle_order(n)
    expect = np.empty_like(x)
    expect[final] = x
    assert np.array_equal(plain, expect)
