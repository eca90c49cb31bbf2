"""Committed golden fixtures (tests/golden/*.json, made by make_golden.py).

CPU: the oracle regenerates every fixture bit for bit, and the revealed
values meet the reference tests' expectations.
GPU: the product path (three parties on cuda:0 through libaby3.so and the
gfx950 kernels) reproduces every party's shares and the revealed values of
every fixture bit for bit.
"""
import json
import os

import numpy as np
import pytest

import oracle as orc
from aby3_amd import native as nt

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(HERE, name + ".json")) as f:
        return json.load(f)


def A(x):
    return np.asarray(x, dtype=np.int64)


def cases(name):
    return sorted(load(name).items())


# ---- arithmetic -----------------------------------------------------------
@pytest.mark.parametrize("name,fx", cases("arith"))
def test_arith_oracle(name, fx):
    if "mode" in fx:
        sh, plain = orc.sim_mul(fx["mode"], fx["trunc"], fx["d"], A(fx["a"]), A(fx["b"]), fx["M"], fx["K"], fx["N"])
    else:
        sh, plain = orc.sim_mul_bit(fx["kind"], A(fx["a"]), fx["apub"], A(fx["bits"]))
    assert np.array_equal(sh.reshape(-1), A(fx["shares"]))
    assert np.array_equal(plain, A(fx["revealed"]))


@pytest.mark.gpu
@pytest.mark.parametrize("name,fx", cases("arith"))
def test_arith_gpu(gpu, name, fx):
    if "mode" in fx:
        sh, plain = nt.sim.mul(fx["mode"], fx["trunc"], fx["d"], A(fx["a"]), A(fx["b"]), fx["M"], fx["K"], fx["N"])
    else:
        sh, plain = nt.sim.mul_bit(fx["kind"], A(fx["a"]), fx["apub"], A(fx["bits"]))
    assert np.array_equal(sh.reshape(-1), A(fx["shares"])), "shares differ from the fixture"
    assert np.array_equal(plain, A(fx["revealed"]))


# ---- binary circuits ------------------------------------------------------
def _cir_inputs(fx):
    return [A(x) for x in fx["inputs"]]


@pytest.mark.parametrize("name,fx", cases("binary"))
def test_binary_oracle(name, fx):
    cir = nt.circuit(fx["circuit"], fx["size"], fx["param"])
    assert len(cir["gates"]) == fx["gates"], "circuit library changed: regenerate the fixtures"
    res, shs = orc.sim_circuit(cir, fx["rows"], _cir_inputs(fx), with_shares=True)
    for o in range(len(res)):
        assert np.array_equal(res[o].reshape(-1), A(fx["revealed"][o]))
        assert np.array_equal(shs[o].reshape(-1), A(fx["shares"][o]))


@pytest.mark.gpu
@pytest.mark.parametrize("name,fx", cases("binary"))
def test_binary_gpu(gpu, name, fx):
    shs, res = nt.sim.circuit(fx["circuit"], fx["size"], fx["param"], fx["rows"], _cir_inputs(fx))
    for o in range(len(res)):
        assert np.array_equal(shs[o].reshape(-1), A(fx["shares"][o])), f"output {o} shares differ"
        assert np.array_equal(res[o].reshape(-1), A(fx["revealed"][o]))


@pytest.mark.parametrize("name,fx", cases("fetch_msb"))
def test_cipher_gt_oracle(name, fx):
    plain, sh = orc.sim_fetch_msb(nt.circuit("int_comp_helper", 64), A(fx["a"]), A(fx["b"]), with_shares=True)
    assert np.array_equal(plain, A(fx["revealed"]))
    assert np.array_equal(sh.reshape(-1), A(fx["shares"]))


@pytest.mark.gpu
@pytest.mark.parametrize("name,fx", cases("fetch_msb"))
def test_cipher_gt_gpu(gpu, name, fx):
    sh, plain = nt.sim.cipher_gt(A(fx["a"]), A(fx["b"]))
    assert np.array_equal(sh.reshape(-1), A(fx["shares"]))
    assert np.array_equal(plain, A(fx["revealed"]))


# ---- piecewise and merge --------------------------------------------------
@pytest.mark.parametrize("name,fx", cases("piecewise"))
def test_piecewise_oracle(name, fx):
    cir = nt.circuit("int_Sh3Piecewise_helper", 64, 2)
    sh, plain = orc.sim_piecewise(fx["kind"], cir, A(fx["x"]), fx["D"])
    assert np.array_equal(sh.reshape(-1), A(fx["shares"]))
    assert np.array_equal(plain, A(fx["revealed"]))


@pytest.mark.gpu
@pytest.mark.parametrize("name,fx", cases("piecewise"))
def test_piecewise_gpu(gpu, name, fx):
    sh, plain = nt.sim.piecewise(fx["kind"], A(fx["x"]), fx["D"])
    assert np.array_equal(sh.reshape(-1), A(fx["shares"]))
    assert np.array_equal(plain, A(fx["revealed"]))


@pytest.mark.parametrize("name,fx", cases("merge"))
def test_merge_fixture_is_sorted_union(name, fx):
    lists = [A(v) for v in fx["lists"]]
    assert all(np.all(np.diff(v) >= 0) for v in lists)
    dim = fx.get("dim", 0)
    if fx.get("mode", 0) == 2:
        k = len(lists) // dim
        exp = np.concatenate([np.sort(np.concatenate(lists[i * k:(i + 1) * k])) for i in range(dim)])
    else:
        exp = np.sort(np.concatenate(lists))
    assert np.array_equal(exp, A(fx["sorted"]))


@pytest.mark.parametrize("name,fx", [c for c in cases("merge") if "shares" in c[1]])
def test_merge_oracle(name, fx):
    plain, sh = orc.sim_merge(nt.circuit("cmp_swap", 64), [A(v) for v in fx["lists"]], fx["mode"], fx["dim"],
                              with_shares=True)
    assert np.array_equal(plain, A(fx["sorted"]))
    assert np.array_equal(sh.reshape(-1), A(fx["shares"]))


@pytest.mark.gpu
@pytest.mark.parametrize("name,fx", cases("merge"))
def test_merge_gpu(gpu, name, fx):
    plain, sh = nt.sim.merge([A(v) for v in fx["lists"]], fx.get("mode", 0), fx.get("dim", 0), shares=True)
    assert np.array_equal(plain, A(fx["sorted"]))
    if "shares" in fx:
        assert np.array_equal(sh.reshape(-1), A(fx["shares"]))
