"""ctypes binding of the gfx950 C-ABI (include/aby3gpu.h).

The shared library is built in-tree by ``make`` (``__graft_entry__.build()``)
into ``aby3_amd/lib/``. There is no fallback: if the library is missing or a
symbol is absent, importing this module raises, so nothing can silently run
on a CPU path.
"""
from __future__ import annotations

import ctypes
import os
import re
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int64, c_size_t, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "lib")
GPU_LIB = os.path.join(LIB_DIR, "libaby3gpu.so")
HOST_LIB = os.path.join(LIB_DIR, "libaby3.so")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "aby3gpu.h")

c_u8p = POINTER(ctypes.c_uint8)

MUL_HADAMARD, MUL_GEMM = 0, 1
DRAW_ARITH, DRAW_BIN, DRAW_RANDPAIR = 0, 1, 2
GATE = dict(XOR=0, NXOR=1, AND=2, OR=3, NOR=4, NA_AND=5, COPY=6, INV=7)
PROBE_GEMM, PROBE_EPILOGUE, PROBE_BINARY, PROBE_AES, PROBE_OTHER = range(5)


class ZeroShare(ctypes.Structure):
    _fields_ = [("k_prev", ctypes.c_uint8 * 16), ("k_next", ctypes.c_uint8 * 16), ("draw_base", c_uint64)]


class TruncStreams(ctypes.Structure):
    _fields_ = [
        ("next_seed", ctypes.c_uint8 * 16),
        ("next_off", c_uint64),
        ("prev_seed", ctypes.c_uint8 * 16),
        ("prev_off", c_uint64),
    ]


class StreamPos(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint8 * 16), ("off", c_uint64)]


class Gate(ctypes.Structure):
    _fields_ = [("in0", c_uint32), ("in1", c_uint32), ("out", c_uint32), ("type", c_uint32),
                ("z_row", c_uint32), ("send_row", c_uint32)]


def key16(b: bytes):
    assert len(b) == 16
    return (ctypes.c_uint8 * 16)(*b)


_SIGS = {
    "aby3g_last_error": (c_char_p, []),
    "aby3g_version": (c_int, []),
    "aby3g_device_count": (c_int, [POINTER(c_int)]),
    "aby3g_set_device": (c_int, [c_int]),
    "aby3g_malloc": (c_int, [POINTER(c_void_p), c_size_t]),
    "aby3g_free": (c_int, [c_void_p]),
    "aby3g_host_malloc": (c_int, [POINTER(c_void_p), c_size_t]),
    "aby3g_host_free": (c_int, [c_void_p]),
    "aby3g_memcpy": (c_int, [c_void_p, c_void_p, c_size_t, c_int, c_void_p]),
    "aby3g_memset": (c_int, [c_void_p, c_int, c_size_t, c_void_p]),
    "aby3g_stream_create": (c_int, [POINTER(c_void_p)]),
    "aby3g_stream_destroy": (c_int, [c_void_p]),
    "aby3g_stream_sync": (c_int, [c_void_p]),
    "aby3g_device_sync": (c_int, []),
    "aby3g_event_create": (c_int, [POINTER(c_void_p)]),
    "aby3g_event_destroy": (c_int, [c_void_p]),
    "aby3g_event_record": (c_int, [c_void_p, c_void_p]),
    "aby3g_event_sync": (c_int, [c_void_p]),
    "aby3g_stream_wait_event": (c_int, [c_void_p, c_void_p]),
    "aby3g_event_elapsed_ms": (c_int, [c_void_p, c_void_p, POINTER(c_float)]),
    "aby3g_probe_enable": (c_int, [c_int]),
    "aby3g_probe_read": (c_int, [c_int, POINTER(c_double), POINTER(c_uint64)]),
    "aby3g_probe_reset": (c_int, []),
    "aby3g_aes_block_host": (c_int, [c_u8p, c_uint64, c_u8p]),
    "aby3g_aes_ctr": (c_int, [c_u8p, c_uint64, c_uint64, c_void_p, c_void_p]),
    "aby3g_prng_fill": (c_int, [c_u8p, c_uint64, c_uint64, c_void_p, c_void_p]),
    "aby3g_share_draws": (c_int, [c_int, c_u8p, c_u8p, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "aby3g_mul_workspace_bytes": (c_size_t, [c_int, c_uint64, c_uint64, c_uint64]),
    "aby3g_mul_local": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_uint64, c_uint64, c_uint64,
                                POINTER(ZeroShare), c_void_p, c_size_t, c_void_p]),
    "aby3g_trunc_tuple": (c_int, [POINTER(TruncStreams), c_uint64, ctypes.c_uint, c_void_p, c_void_p, c_void_p]),
    "aby3g_mul_trunc_local": (c_int, [c_int, c_void_p, c_void_p, c_uint64, c_uint64, c_uint64, ctypes.c_uint,
                                      POINTER(TruncStreams), c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "aby3g_trunc_finalize": (c_int, [c_int, c_void_p, c_void_p, c_void_p, ctypes.c_uint, c_void_p, c_uint64,
                                     c_void_p]),
    "aby3g_bitmul_p0": (c_int, [c_void_p, c_void_p, c_uint64, POINTER(StreamPos), POINTER(StreamPos), c_u8p,
                                c_uint64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "aby3g_bitmul_p2": (c_int, [c_void_p, c_void_p, c_uint64, POINTER(StreamPos), c_u8p, c_uint64, c_void_p,
                                c_void_p, c_void_p, c_void_p]),
    "aby3g_ot_recv": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, c_int, c_void_p, c_void_p]),
    "aby3g_pubmul_p0": (c_int, [c_int64, c_void_p, c_uint64, POINTER(ZeroShare), c_u8p, c_uint64, c_u8p, c_uint64,
                                c_void_p, c_void_p, c_void_p]),
    "aby3g_pubmul_helper": (c_int, [c_void_p, c_uint64, POINTER(ZeroShare), c_u8p, c_uint64, c_void_p, c_void_p,
                                    c_void_p]),
    "aby3g_bin_gates": (c_int, [c_void_p, c_uint32, c_void_p, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p]),
    "aby3g_bin_unpack": (c_int, [c_void_p, c_void_p, c_uint32, c_void_p, c_uint64, c_uint64, c_void_p]),
    "aby3g_bits_to_wires": (c_int, [c_void_p, c_uint64, c_uint64, c_uint32, c_void_p, c_uint64, c_void_p]),
    "aby3g_wires_to_bits": (c_int, [c_void_p, c_void_p, c_uint32, c_uint64, c_void_p, c_uint64, c_void_p]),
    "aby3g_i64_lincomb": (c_int, [c_uint64, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p]),
    "aby3g_u64_bitop": (c_int, [c_int, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "aby3g_u64_gather": (c_int, [c_uint64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "aby3g_u64_scatter": (c_int, [c_uint64, c_void_p, c_void_p, c_void_p, c_void_p]),
}


def declared_symbols(header: str = HEADER) -> list[str]:
    """Every function name include/aby3gpu.h declares."""
    text = open(header).read()
    return sorted(set(re.findall(r"\b(aby3g_[a-z0-9_]+)\s*\(", text)))


class NativeError(RuntimeError):
    pass


class _Lib:
    def __init__(self, path: str = GPU_LIB):
        if not os.path.exists(path):
            raise NativeError(f"{path} missing: run `make` (or __graft_entry__.build()) first; there is no CPU fallback")
        self.path = path
        self.dll = ctypes.CDLL(path)
        for name, (res, args) in _SIGS.items():
            fn = getattr(self.dll, name)  # raises AttributeError if not exported
            fn.restype = res
            fn.argtypes = args

    def __getattr__(self, name):
        fn = getattr(self.dll, "aby3g_" + name)

        def call(*args):
            rc = fn(*args)
            if fn.restype is c_int and rc != 0:
                raise NativeError(f"aby3g_{name} failed ({rc}): {self.dll.aby3g_last_error().decode()}")
            return rc

        return call


_lib = None


def lib() -> _Lib:
    global _lib
    if _lib is None:
        _lib = _Lib()
    return _lib
