"""The C4 driver around the SGD iteration (aby3-ML): LogisticModelGen data
(LinearModelGen.cpp:49-93, main-logistic.cpp:82-100), getSubset mini-batches
(Regression.h:24-40), aby3ML::init seeds, and SGD_Logistic's iterations.

CPU: the product's host-side generator and sampler (libaby3.so) equal the
oracle's restatement and the committed fixture (tests/golden/lr.json: the
model, the first two mini-batches over the 10^6-row dataset, the dataset's
head and sums); the oracle regenerates the fixture's w shares.
GPU: three parties on cuda:0 reproduce every party's w shares bit for bit
after k iterations (the fixture, and the oracle directly on 20000 rows).
"""
import json
import os

import numpy as np
import pytest

import oracle as orc
from aby3_amd import native as nt

FX = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lr.json")))["lr_4096x128_B256"]


def A(x, dt=np.int64):
    return np.asarray(x, dtype=dt)


@pytest.mark.parametrize("n", [FX["n"], 1_000_000])
def test_labels_independent_of_summation_order(n):
    # The reference labels rows by Eigen's GEMV X * mModel + noise
    # (LinearModelGen.cpp:75); the restatements sum left to right. Every row's
    # |sum + noise| exceeds twice the error bound any summation order can
    # reach, so the labels -- of the fixture's rows and of the whole 10^6-row
    # C4 dataset -- are the reference's whatever order Eigen sums in.
    assert orc.lr_label_margin(n, FX["d"]) > 1.0


def test_dataset_product_equals_oracle_and_fixture():
    X, Y, m = nt.lr_dataset(FX["n"], FX["d"], FX["D"])
    Xo, Yo, mo = orc.lr_dataset(FX["n"], FX["d"], FX["D"])
    assert np.array_equal(X, Xo) and np.array_equal(Y, Yo) and np.array_equal(m, mo)
    assert list(m) == FX["model"]
    assert np.array_equal(X[:2].reshape(-1), A(FX["x_rows01"]))
    assert np.array_equal(Y[:64], A(FX["y_head"]))
    assert int(X.sum()) == FX["x_sum"] and int(Y.sum()) == FX["y_sum"]
    # labels are 0 / 1 in fixed point, features ~ N(1, 1)
    assert set(np.unique(Y).tolist()) <= {0, 1 << FX["D"]}
    assert abs(X.mean() / (1 << FX["D"]) - 1.0) < 0.02


def test_batches_product_equals_oracle_and_fixture():
    b = nt.lr_batches(10**6, 256, 2)
    assert np.array_equal(b, orc.lr_batches(10**6, 256, 2))
    assert np.array_equal(b.reshape(-1), A(FX["batches_1e6"], np.uint64))
    small = nt.lr_batches(FX["n"], FX["B"], FX["iters"])
    assert np.array_equal(small.reshape(-1), A(FX["batches"], np.uint64))
    # without replacement within an epoch; the pool reshuffles when exhausted
    e = nt.lr_batches(1000, 100, 10)
    assert sorted(e.reshape(-1).tolist()) == list(range(1000))
    assert len(set(nt.lr_batches(1000, 300, 4).reshape(-1)[:900].tolist())) == 900


def test_oracle_w_shares_match_fixture():
    X, Y, _ = orc.lr_dataset(FX["n"], FX["d"], FX["D"])
    b = A(FX["batches"], np.uint64).reshape(FX["iters"], FX["B"])
    sh, w = orc.sim_lr(nt.circuit("int_Sh3Piecewise_helper", 64, 2), X, Y, b, FX["D"], FX["aB"])
    assert np.array_equal(sh.reshape(-1), A(FX["w_shares"]))
    assert np.array_equal(w, A(FX["w"]))


@pytest.mark.gpu
def test_lr_gpu_matches_fixture(gpu):
    X, Y, _ = nt.lr_dataset(FX["n"], FX["d"], FX["D"])
    b = A(FX["batches"], np.uint64).reshape(FX["iters"], FX["B"])
    sh, w = nt.sim.lr(X, Y, b, FX["D"], FX["aB"])
    assert np.array_equal(sh.reshape(-1), A(FX["w_shares"]))
    assert np.array_equal(w, A(FX["w"]))


@pytest.mark.gpu
@pytest.mark.parametrize("n,B,iters", [(20000, 256, 5), (3000, 64, 4), (1000000, 256, 3)])
def test_lr_vs_oracle(gpu, n, B, iters):
    # (1000000, 256, 3): C4's own dataset (BASELINE configs[3]), 2 GB of shares per party
    X, Y, _ = nt.lr_dataset(n, 128, 16)
    b = nt.lr_batches(n, B, iters)
    sh_g, w_g = nt.sim.lr(X, Y, b)
    sh_o, w_o = orc.sim_lr(nt.circuit("int_Sh3Piecewise_helper", 64, 2), X, Y, b)
    assert np.array_equal(sh_g, sh_o)
    assert np.array_equal(w_g, w_o)
