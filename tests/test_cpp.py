"""Runs the C++ test programs (built by `make tests`): the scheduler contract
and the circuit library on CPU; the 3-party protocol parity suites on GPU."""
import os
import subprocess

import pytest

BUILD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp", "build")


def _run(name, timeout):
    exe = os.path.join(BUILD, name)
    assert os.path.exists(exe), f"{exe} missing: run `make tests`"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=timeout)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "FAIL" not in r.stdout


def test_runtime_schedule():
    _run("test_runtime", 60)


def test_circuit_library_plaintext():
    _run("test_circuits", 120)


@pytest.mark.gpu
def test_arith_protocols_gpu():
    _run("test_arith", 600)


@pytest.mark.gpu
def test_binary_protocols_gpu():
    _run("test_binary", 600)


@pytest.mark.gpu
def test_oram_gpu():
    # sqrt-ORAM and its position map at the reference tests' revealed checks
    _run("test_oram", 600)


@pytest.mark.gpu
def test_lr_iteration_both_forms_gpu():
    # SGD_Logistic op by op and fused (aby3g_lr_iteration), share-exact vs the oracle
    _run("test_lr", 600)


@pytest.mark.gpu
def test_convert_protocols_gpu():
    _run("test_convert", 600)


def test_convert_oracle_revealed():
    # the oracle's share conversions against the reference tests' revealed checks (CPU)
    _run("test_convert_oracle", 120)


def test_random_shuffle_restatements():
    # product and oracle batch sampling / shuffle permutations against libstdc++'s
    # own std::random_shuffle on the same PRNG stream (CPU)
    _run("test_random_shuffle", 120)
