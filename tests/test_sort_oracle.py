"""CPU checks of the merge network (aby3-Basic/Sort.cpp:327-628) and of the
oracle's batched restatement (oracle/src/orc_sort.cpp).

* The reference's round schedule (t = ceil(log2(length) + 1), q = 2^(t-1),
  d = 1 then q - 1 with q halving, r = 1 after the first round) restated in
  plain Python sorts every input it is given: merges of unequal lengths
  (padding with max(last1, last2)) and multi-merges of odd list counts.
* The 2^20-key sort (C5) is 20 levels, 210 rounds.
* The oracle's three-party restatement reveals the sorted lists in every mode
  (merge, multi-merge, high-dimensional forms), with consistent shares.
"""
import math

import numpy as np
import pytest

import oracle as orc
from aby3_amd import native as nt


def rounds(length):
    # Sort.cpp:361-398
    t = math.ceil(math.log2(length) + 1)
    q, d, r, out = 2 ** (t - 1), 1, 0, []
    while d > 0:
        out.append((d, r))
        d, q, r = q - 1, q >> 1, 1
    return out


def merge_plain(a, b):
    L = max(len(a), len(b))
    res = [max(a[-1], b[-1])] * (2 * L)
    res[0:2 * len(a):2] = a
    res[1:2 * len(b):2] = b
    for d, r in rounds(L):
        for i in range(r, 2 * L - d, 2):
            if res[i] > res[i + d]:
                res[i], res[i + d] = res[i + d], res[i]
    return res[:len(a) + len(b)]


def multi_plain(lists):
    k = len(lists)
    while k != 1:  # Sort.cpp:413-437
        if k % 2:
            lists[k - 2] = merge_plain(lists[k - 2], lists[k - 1])
            k -= 1
        else:
            lists = [merge_plain(lists[i], lists[i + 1]) for i in range(0, k, 2)]
            k //= 2
    return lists[0]


def test_schedule_sorts():
    rng = np.random.default_rng(1)
    for n in list(range(1, 70)) + [127, 128, 129, 1000]:
        keys = [int(x) for x in rng.integers(0, 1 << 40, size=n)]
        assert multi_plain([[x] for x in keys]) == sorted(keys), n
    for _ in range(300):
        l1, l2 = (int(x) for x in rng.integers(1, 50, size=2))
        a = sorted(int(x) for x in rng.integers(0, 100, size=l1))
        b = sorted(int(x) for x in rng.integers(0, 100, size=l2))
        assert merge_plain(a, b) == sorted(a + b)


def test_c5_round_count():
    assert sum(len(rounds(2 ** lv)) for lv in range(20)) == 210


@pytest.mark.parametrize("mode,dim,lens", [
    (0, 0, [8, 8]), (0, 0, [5, 7, 8, 3]), (0, 0, [100, 3, 17, 250, 9]), (1, 0, [1] * 300),
    (2, 3, [6] * 9), (3, 2, [5, 9, 2, 2]), (4, 0, [5, 7, 8, 3]), (4, 0, [100, 3, 17, 250, 9]),
    (5, 3, [6] * 12),
])
def test_oracle_merge_sorted(mode, dim, lens):
    rng = np.random.default_rng(len(lens))
    lists = [np.sort(rng.integers(-(2**62), 2**62, size=n, dtype=np.int64)) for n in lens]
    plain, sh = orc.sim_merge(nt.circuit("cmp_swap", 64), lists, mode, dim, with_shares=True)
    if mode in (2, 3, 5):
        k = len(lists) // dim
        exp = np.concatenate([np.sort(np.concatenate(lists[i * k:(i + 1) * k])) for i in range(dim)])
    else:
        exp = np.sort(np.concatenate(lists))
    assert np.array_equal(plain, exp)
    for p in range(3):  # party p's share 1 is party p-1's share 0
        assert np.array_equal(sh[p, 1], sh[(p + 2) % 3, 0])


def test_oracle_merge_orders():
    """The reference's sequential order of a level's merges (Sort.cpp:423-429)
    and the batched one reveal the same list from different randomness draws;
    with a single merge per level (two lists) they are the same computation."""
    rng = np.random.default_rng(7)
    cir = nt.circuit("cmp_swap", 64)
    lists = [np.sort(rng.integers(-(2**62), 2**62, size=n, dtype=np.int64)) for n in (5, 7, 8, 3)]
    pb, sb = orc.sim_merge(cir, lists, 0, 0, with_shares=True)
    ps, ss = orc.sim_merge(cir, lists, 4, 0, with_shares=True)
    assert np.array_equal(pb, ps) and not np.array_equal(sb, ss)
    two = lists[:2]
    assert np.array_equal(orc.sim_merge(cir, two, 0, 0, with_shares=True)[1],
                          orc.sim_merge(cir, two, 4, 0, with_shares=True)[1])
