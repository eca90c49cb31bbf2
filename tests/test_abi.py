"""The C-ABI libraries load on a CPU-only host and export every symbol their
headers declare (no compute calls without a GPU)."""
import ctypes
import os
import re

from aby3_amd import native as nt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header, prefix):
    text = open(os.path.join(ROOT, "include", header)).read()
    return sorted(set(re.findall(r"\b(" + prefix + r"[a-z0-9_]+)\s*\(", text)))


def test_gpu_lib_exports_every_declared_symbol():
    dll = ctypes.CDLL(nt.GPU_LIB)
    names = _declared("aby3gpu.h", "aby3g_")
    assert len(names) > 40
    missing = [n for n in names if not hasattr(dll, n)]
    assert not missing, missing


def test_binding_covers_header():
    # the ctypes signature table is complete, so no call goes out untyped
    names = set(_declared("aby3gpu.h", "aby3g_"))
    assert names == set(nt._SIGS), names ^ set(nt._SIGS)


def test_host_lib_exports_every_declared_symbol():
    nt.lib()
    dll = ctypes.CDLL(nt.HOST_LIB)
    names = _declared("aby3.h", "aby3h_")
    missing = [n for n in names if not hasattr(dll, n)]
    assert not missing, missing


def test_host_key_derivation_matches_oracle():
    # aby3g_aes_block_host runs on the CPU: keys of Sh3ShareGen::init
    import oracle as orc

    lib = nt.lib()
    seed = orc.to_block(0, 2)
    out = (ctypes.c_uint8 * 16)()
    lib.aes_block_host(nt.key16(seed), 0, out)
    assert bytes(out) == orc.prng_bytes(seed, 0, 16)


def test_errors_are_reported_not_thrown():
    lib = nt.lib()
    rc = lib.dll.aby3g_prng_fill(nt.key16(bytes(16)), 3, 8, None, None)  # misaligned offset
    assert rc != 0
    assert b"multiples of 8" in lib.dll.aby3g_last_error()
