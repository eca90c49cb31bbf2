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

# HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues (default 4). Three
# co-located parties use one stream each plus the shared AND-mask draw stream
# -- four -- so the default fits; 8 queues measured the same, and extra
# per-party streams with them far slower. Left to the
# caller's environment.

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "lib")
GPU_LIB = os.path.join(LIB_DIR, "libaby3gpu.so")
HOST_LIB = os.path.join(LIB_DIR, "libaby3.so")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "aby3gpu.h")

c_u8p = POINTER(ctypes.c_uint8)

MUL_HADAMARD, MUL_GEMM = 0, 1
DRAW_ARITH, DRAW_BIN, DRAW_RANDPAIR = 0, 1, 2
GATE = dict(XOR=0, NXOR=1, AND=2, OR=3, NOR=4, NA_AND=5, COPY=6, INV=7)
PROBE_GEMM, PROBE_EPILOGUE, PROBE_BINARY, PROBE_AES, PROBE_OTHER, PROBE_DIGITS = range(6)


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


class Handoff(ctypes.Structure):
    _fields_ = [("flags", c_void_p), ("seq", c_uint64), ("wait_ticks", c_void_p)]


class RowMap(ctypes.Structure):
    """aby3g_rowmap: element p -> idx[first + p], or the affine
    start + rep * rep_stride + k * step with (rep, k) = divmod(first + p, per_rep)."""
    _fields_ = [("first", c_uint64), ("start", c_uint64), ("step", c_uint64), ("per_rep", c_uint64),
                ("rep_stride", c_uint64), ("idx", c_void_p)]


class WireSrc(ctypes.Structure):
    """aby3g_wire_src: one source of aby3g_bits_to_wires_lin."""
    _fields_ = [("term", ctypes.POINTER(ctypes.c_int64) * 4), ("coef", ctypes.c_int64 * 4),
                ("constant", ctypes.c_int64), ("cols64", c_uint64), ("nbits", c_uint32),
                ("wire_rows", ctypes.POINTER(c_uint64)), ("copy_out", ctypes.POINTER(ctypes.c_int64))]


def key16(b: bytes):
    assert len(b) == 16
    return (ctypes.c_uint8 * 16)(*b)


_SIGS = {
    "aby3g_last_error": (c_char_p, []),
    "aby3g_version": (c_int, []),
    "aby3g_recent_calls": (c_int, [c_char_p, c_size_t]),
    "aby3g_set_draw_workgroups": (c_int, [c_int]),
    "aby3g_device_count": (c_int, [POINTER(c_int)]),
    "aby3g_set_device": (c_int, [c_int]),
    "aby3g_get_device": (c_int, [POINTER(c_int)]),
    "aby3g_api_time": (c_int, [POINTER(c_double), POINTER(c_uint64)]),
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
    "aby3g_event_create_timed": (c_int, [POINTER(c_void_p)]),
    "aby3g_event_destroy": (c_int, [c_void_p]),
    "aby3g_event_record": (c_int, [c_void_p, c_void_p]),
    "aby3g_event_sync": (c_int, [c_void_p]),
    "aby3g_stream_wait_event": (c_int, [c_void_p, c_void_p]),
    "aby3g_event_elapsed_ms": (c_int, [c_void_p, c_void_p, POINTER(c_float)]),
    "aby3g_signal_alloc": (c_int, [POINTER(c_void_p)]),
    "aby3g_stream_write_value": (c_int, [c_void_p, c_void_p, c_uint64]),
    "aby3g_stream_wait_value": (c_int, [c_void_p, c_void_p, c_uint64]),
    "aby3g_ipc_get_handle": (c_int, [c_void_p, c_void_p]),
    "aby3g_ipc_open": (c_int, [c_void_p, POINTER(c_void_p)]),
    "aby3g_ipc_close": (c_int, [c_void_p]),
    "aby3g_host_register": (c_int, [c_void_p, c_size_t, POINTER(c_void_p)]),
    "aby3g_host_unregister": (c_int, [c_void_p]),
    "aby3g_enable_peer_access": (c_int, [c_int, c_int]),
    "aby3g_set_gemm_sharing": (c_int, [c_int]),
    "aby3g_u64_xor_gather_units": (c_int, [c_uint64, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                           c_void_p, c_void_p]),
    "aby3g_probe_enable": (c_int, [c_int]),
    "aby3g_probe_enable_mask": (c_int, [ctypes.c_uint32]),
    "aby3g_probe_read": (c_int, [c_int, POINTER(c_double), POINTER(c_uint64)]),
    "aby3g_probe_reset": (c_int, []),
    "aby3g_aes_block_host": (c_int, [c_u8p, c_uint64, c_u8p]),
    "aby3g_aes_ctr_host": (c_int, [c_u8p, c_uint64, c_uint64, c_void_p]),
    "aby3g_aes_ctr": (c_int, [c_u8p, c_uint64, c_uint64, c_void_p, c_void_p]),
    "aby3g_prng_fill": (c_int, [c_u8p, c_uint64, c_uint64, c_void_p, c_void_p]),
    "aby3g_share_draws": (c_int, [c_int, c_u8p, c_u8p, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "aby3g_share_draws_rows": (c_int, [c_int, c_u8p, c_u8p, c_uint64, c_uint64, c_uint64, c_uint64, c_void_p,
                                       c_void_p]),
    "aby3g_mul_workspace_bytes": (c_size_t, [c_int, c_uint64, c_uint64, c_uint64]),
    "aby3g_mul_local": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_uint64, c_uint64, c_uint64,
                                POINTER(ZeroShare), c_void_p, c_size_t, c_void_p]),
    "aby3g_trunc_tuple": (c_int, [POINTER(TruncStreams), c_uint64, ctypes.c_uint, c_void_p, c_void_p, c_void_p]),
    "aby3g_mul_prefers_fused": (c_int, [c_int, c_uint64, c_uint64, c_uint64]),
    "aby3g_mfma_turn": (c_int, [c_int]),
    "aby3g_mul_sub_local": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_uint64,
                                    c_uint64, c_void_p, c_size_t, c_void_p]),
    "aby3g_mul_trunc_local": (c_int, [c_int, c_void_p, c_void_p, c_uint64, c_uint64, c_uint64, ctypes.c_uint,
                                      POINTER(TruncStreams), c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "aby3g_trunc_finalize": (c_int, [c_int, c_void_p, c_void_p, c_void_p, ctypes.c_uint, c_void_p, c_uint64,
                                     c_void_p]),
    "aby3g_bitmul_p0": (c_int, [c_void_p, c_void_p, c_uint64, POINTER(StreamPos), POINTER(StreamPos), c_u8p,
                                c_uint64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "aby3g_bitmul_p2": (c_int, [c_void_p, c_void_p, c_uint64, POINTER(StreamPos), c_u8p, c_uint64, c_void_p,
                                c_void_p, c_void_p, c_void_p]),
    "aby3g_ot_recv": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, c_int, c_void_p, c_void_p]),
    "aby3g_a2b_reshare": (c_int, [POINTER(StreamPos), c_uint64, c_uint64, c_uint64, c_void_p, c_void_p, c_int,
                                  c_void_p, c_void_p, c_void_p]),
    "aby3g_bitinj_send": (c_int, [c_void_p, c_uint64, c_uint64, c_uint64, POINTER(StreamPos), POINTER(StreamPos),
                                  c_u8p, c_uint64, c_u8p, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "aby3g_prng_i32": (c_int, [POINTER(StreamPos), c_uint64, c_int64, c_void_p, c_void_p]),
    "aby3g_b2a_open": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p, c_void_p]),
    "aby3g_ot_help_bits": (c_int, [c_void_p, c_uint64, c_uint64, c_uint64, c_u8p, c_uint64, c_void_p, c_void_p]),
    "aby3g_ot_recv_bits": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, c_uint64, c_uint64, c_void_p,
                                   c_void_p]),
    "aby3g_pubmul_p0": (c_int, [c_int64, c_void_p, c_uint64, POINTER(ZeroShare), c_u8p, c_uint64, c_u8p, c_uint64,
                                c_void_p, c_void_p, c_void_p]),
    "aby3g_pubmul_helper": (c_int, [c_void_p, c_uint64, POINTER(ZeroShare), c_u8p, c_uint64, c_void_p, c_void_p,
                                    c_void_p]),
    "aby3g_bin_gates": (c_int, [c_void_p, c_uint32, c_void_p, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p]),
    "aby3g_bin_level": (c_int, [c_void_p, c_void_p, ctypes.c_uint32, c_void_p, c_void_p, ctypes.c_uint32, c_void_p,
                                c_uint64, c_uint64, c_void_p, c_void_p, c_void_p]),
    "aby3g_bin_level_rr": (c_int, [c_void_p, c_void_p, c_void_p, ctypes.c_uint32, c_void_p, c_void_p, ctypes.c_uint32,
                                   c_void_p, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p]),
    # the aby3g_handoff / aby3g_lr_iter / aby3g_lr_circuit structs go by pointer
    "aby3g_bin_level_hs": (c_int, [c_void_p, c_void_p, c_void_p, ctypes.c_uint32, c_void_p, c_void_p, ctypes.c_uint32,
                                   c_void_p, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "aby3g_handoff_status": (c_int, [POINTER(ctypes.c_uint32)]),
    "aby3g_set_handoff_timeout_us": (c_int, [c_uint64]),
    "aby3g_bin_level_residency": (c_int, [POINTER(c_int), POINTER(c_int), POINTER(c_int), POINTER(c_int)]),
    "aby3g_stream_count": (c_int, [c_int, POINTER(c_int)]),
    "aby3g_null_queue_init": (c_int, []),
    "aby3g_malloc_uncached": (c_int, [POINTER(c_void_p), c_size_t]),
    "aby3g_device_uuid": (c_int, [c_int, c_void_p]),
    "aby3g_event_query": (c_int, [c_void_p, POINTER(c_int)]),
    "aby3g_lr_mailbox_bytes": (c_uint64, [ctypes.c_uint32, ctypes.c_uint32, c_void_p]),
    "aby3g_lr_scratch_bytes": (c_uint64, [ctypes.c_uint32, ctypes.c_uint32, c_void_p]),
    "aby3g_lr_iteration": (c_int, [c_void_p, c_void_p]),
    "aby3g_bits_to_wires2": (c_int, [c_void_p, c_uint64, c_uint64, ctypes.c_uint32, c_void_p, c_uint64, c_uint64,
                                     c_void_p]),
    "aby3g_wires_to_bits2": (c_int, [c_void_p, c_uint64, c_void_p, ctypes.c_uint32, c_uint64, c_void_p, c_uint64,
                                     c_void_p]),
    "aby3g_bits_to_wires_map_n": (c_int, [c_void_p, c_uint64, c_uint64, ctypes.c_uint32, c_void_p, c_void_p,
                                          ctypes.c_uint32, c_uint64, c_uint64, c_uint64, c_void_p]),
    "aby3g_wires_to_bits_map_n": (c_int, [c_void_p, c_uint64, c_void_p, ctypes.c_uint32, c_uint64, c_void_p,
                                          c_uint64, c_void_p, ctypes.c_uint32, c_uint64, c_void_p]),
    "aby3g_bits_to_wires_map": (c_int, [c_void_p, c_uint64, c_uint64, ctypes.c_uint32, POINTER(RowMap), c_uint64,
                                        c_void_p, c_uint64, c_uint64, c_void_p]),
    "aby3g_wires_to_bits_map": (c_int, [c_void_p, c_uint64, c_void_p, ctypes.c_uint32, c_uint64, c_void_p, c_uint64,
                                        POINTER(RowMap), c_uint64, c_void_p]),
    "aby3g_bin_unpack": (c_int, [c_void_p, c_void_p, c_uint32, c_void_p, c_uint64, c_uint64, c_void_p]),
    # aby3g_wire_src / aby3g_level_run arrays and aby3g_handoff go by pointer
    "aby3g_lin_copy_out": (c_int, [c_void_p, c_uint32, c_uint64, c_void_p]),
    "aby3g_bin_level_in": (c_int, [c_void_p, c_uint32, c_uint64, c_uint32, c_uint32, c_int, c_void_p, c_void_p,
                                   c_uint32, c_void_p, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "aby3g_bits_to_wires_lin": (c_int, [c_void_p, c_uint32, c_uint64, c_uint64, c_void_p]),
    "aby3g_bits_to_wires": (c_int, [c_void_p, c_uint64, c_uint64, c_uint32, c_void_p, c_uint64, c_void_p]),
    "aby3g_wires_to_bits": (c_int, [c_void_p, c_void_p, c_uint32, c_uint64, c_void_p, c_uint64, c_void_p]),
    "aby3g_i64_lincomb": (c_int, [c_uint64, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p]),
    "aby3g_u64_bitop": (c_int, [c_int, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "aby3g_i64_gather_rows": (c_int, [c_void_p, c_uint64, c_uint64, c_void_p, c_uint64, c_void_p, c_void_p]),
    "aby3g_i64_transpose": (c_int, [c_void_p, c_uint64, c_uint64, c_void_p, c_void_p]),
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


JOB_MUL_TRUNC, JOB_MUL, JOB_MSB, JOB_LR, JOB_SORT, JOB_A2B, JOB_BITINJ = range(7)
INFO = dict(mults_per_step=0, gemm_int8_ops=1, and_words=2, gate_words=3, gate_bytes=4, bytes_sent=5,
            host_enqueue_us=6, host_drain_us=7, host_recv_wait_us=8, host_api_us=9, host_api_calls=10,
            device_wait_us=11, lr_fused=12, lr_sys_scope=13)

_HOST_SIGS = {
    "aby3h_last_error": (c_char_p, []),
    "aby3h_session_create": (c_void_p, [c_int, POINTER(c_uint64), c_int, POINTER(c_int), c_int]),
    "aby3h_party_create": (c_void_p, [c_int, POINTER(c_uint64), c_int, c_int, c_int, c_char_p, c_int, c_int]),
    "aby3h_session_run": (c_int, [c_void_p, c_uint64]),
    "aby3h_session_probe": (c_int, [c_void_p, c_int, POINTER(c_double), POINTER(c_uint64)]),
    "aby3h_session_probe_reset": (c_int, [c_void_p]),
    "aby3h_session_info": (c_int, [c_void_p, POINTER(c_double), c_int]),
    "aby3h_session_check": (c_int, [c_void_p]),
    "aby3h_session_digest": (c_int, [c_void_p, c_int, c_void_p]),
    "aby3h_session_result": (c_int, [c_void_p, c_int, c_int, c_void_p, c_uint64, c_void_p]),
    "aby3h_session_destroy": (None, [c_void_p]),
    "aby3h_circuit": (c_int, [c_char_p, c_uint64, c_uint64, POINTER(c_uint64), c_void_p, c_void_p, c_void_p,
                              c_void_p, c_void_p, c_void_p]),
    "aby3h_circuit_write": (c_int, [c_char_p, c_uint64, c_uint64, c_char_p]),
    "aby3h_sim_last_error": (c_char_p, []),
    "aby3h_sim_mul": (c_int, [c_int, c_int, c_int, c_uint64, c_void_p, c_void_p, c_uint64, c_uint64, c_uint64,
                              c_void_p, c_void_p]),
    "aby3h_sim_mul_bit": (c_int, [c_int, c_int, c_void_p, c_int64, c_void_p, c_uint64, c_void_p, c_void_p]),
    "aby3h_sim_circuit": (c_int, [c_int, c_char_p, c_uint64, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p]),
    "aby3h_sim_piecewise": (c_int, [c_int, c_int, c_void_p, c_uint64, c_uint64, c_void_p, c_void_p]),
    "aby3h_sim_cipher_gt": (c_int, [c_int, c_void_p, c_void_p, c_uint64, c_void_p, c_void_p]),
    "aby3h_sim_lr": (c_int, [c_int, c_uint64, c_uint64, c_uint64, c_uint64, c_uint64, c_uint64, c_void_p, c_void_p,
                             c_void_p, c_void_p, c_void_p]),
    "aby3h_lr_dataset": (c_int, [c_uint64, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p]),
    "aby3h_lr_batches": (c_int, [c_uint64, c_uint64, c_uint64, c_void_p]),
    "aby3h_sim_shuffle": (c_int, [c_int, c_int, c_void_p, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p]),
    "aby3h_sim_merge": (c_int, [c_int, c_int, c_void_p, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p]),
}

_host = None


def host():
    """The C++ host runtime (include/aby3.h)."""
    global _host
    if _host is None:
        lib()  # the GPU library must load first (libaby3.so links it)
        if not os.path.exists(HOST_LIB):
            raise NativeError(f"{HOST_LIB} missing: run `make`")
        d = ctypes.CDLL(HOST_LIB)
        for name, (res, args) in _HOST_SIGS.items():
            fn = getattr(d, name)
            fn.restype = res
            fn.argtypes = args
        _host = d
    return _host


class Session:
    """Three in-process parties running one job of the hot path (include/aby3.h)."""

    def __init__(self, job: int, params, devices=(0, 0, 0), probe=True):
        """probe: False / True (all kernel families) or a family bitmask
        (1 << PROBE_GEMM, ...): only those launches are bracketed by events."""
        h = host()
        p = (c_uint64 * len(params))(*params)
        dv = (c_int * 3)(*devices)
        mask = 0xFF if probe is True else int(probe)
        self._h = h.aby3h_session_create(job, p, len(params), dv, mask)
        if not self._h:
            raise NativeError("aby3h_session_create: " + h.aby3h_last_error().decode())
        self.host = h

    @classmethod
    def party(cls, job: int, params, party: int, link: str, device: int = 0, colocated: int = 1,
              probe=False):
        """One party of a session in this process (aby3h_party_create): the
        three processes pass the same job, params and link name. colocated:
        0 parties on different GPUs, 1 on this one, 2 on this one taking the
        cross-GPU branches (aby3.h)."""
        self = cls.__new__(cls)
        h = host()
        p = (c_uint64 * len(params))(*params)
        mask = 0xFF if probe is True else int(probe)
        self._h = h.aby3h_party_create(job, p, len(params), party, device, link.encode(), int(colocated), mask)
        if not self._h:
            raise NativeError("aby3h_party_create: " + h.aby3h_last_error().decode())
        self.host = h
        return self

    def run(self, steps: int):
        if self.host.aby3h_session_run(self._h, steps) != 0:
            raise NativeError("aby3h_session_run: " + self.host.aby3h_last_error().decode())

    def probe(self, family: int):
        ms, n = c_double(), c_uint64()
        if self.host.aby3h_session_probe(self._h, family, ctypes.byref(ms), ctypes.byref(n)) != 0:
            raise NativeError("aby3h_session_probe: " + self.host.aby3h_last_error().decode())
        return ms.value, n.value

    def probe_reset(self):
        self.host.aby3h_session_probe_reset(self._h)

    def info(self) -> dict:
        out = (c_double * len(INFO))()
        self.host.aby3h_session_info(self._h, out, len(INFO))
        return {k: out[v] for k, v in INFO.items()}

    def check(self) -> bool:
        rc = self.host.aby3h_session_check(self._h)
        if rc == 2:
            raise NativeError("aby3h_session_check: " + self.host.aby3h_last_error().decode())
        return rc == 0

    def digest(self, party: int) -> int:
        """FNV-1a digest of `party`'s two shares of the last step's result."""
        out = c_uint64()
        if self.host.aby3h_session_digest(self._h, party, ctypes.byref(out)) != 0:
            raise NativeError("aby3h_session_digest: " + self.host.aby3h_last_error().decode())
        return out.value

    def result(self, party: int):
        """`party`'s two shares of the last step's result, as two int64
        numpy arrays (row-major)."""
        import numpy as np

        out = []
        for share in (0, 1):
            n = c_uint64()
            if self.host.aby3h_session_result(self._h, party, share, None, 0, ctypes.byref(n)) != 0:
                raise NativeError("aby3h_session_result: " + self.host.aby3h_last_error().decode())
            a = np.empty(n.value, dtype=np.int64)
            if self.host.aby3h_session_result(self._h, party, share, a.ctypes.data_as(c_void_p), n.value,
                                              ctypes.byref(n)) != 0:
                raise NativeError("aby3h_session_result: " + self.host.aby3h_last_error().decode())
            out.append(a)
        return out[0], out[1]

    def close(self):
        if self._h:
            self.host.aby3h_session_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def circuit_write(name: str, path: str, size: int = 64, param: int = 0):
    """Store a library circuit in the BetaCircuit binary format; "bin:" + path
    then names it for circuit() / sim.circuit()."""
    h = host()
    if h.aby3h_circuit_write(name.encode(), size, param, path.encode()) != 0:
        raise NativeError(h.aby3h_last_error().decode())


def circuit(name: str, size: int = 64, param: int = 0) -> dict:
    """A library circuit as flat arrays (levelized gate list), CPU only."""
    import numpy as np

    h = host()
    counts = (c_uint64 * 6)()
    if h.aby3h_circuit(name.encode(), size, param, counts, None, None, None, None, None, None) != 0:
        raise NativeError(h.aby3h_last_error().decode())
    wires, ngates, nlev, nin, nout, _ = list(counts)
    gates = np.zeros(4 * ngates, dtype=np.uint32)
    levels = np.zeros(nlev, dtype=np.uint32)
    insz = np.zeros(nin, dtype=np.uint32)
    outsz = np.zeros(nout, dtype=np.uint32)
    inw = np.zeros(counts[5], dtype=np.uint32)
    outw = np.zeros(counts[5], dtype=np.uint32)
    P = lambda a: a.ctypes.data_as(c_void_p)
    h.aby3h_circuit(name.encode(), size, param, counts, P(gates), P(levels), P(insz), P(inw), P(outsz), P(outw))
    ins, outs, o = [], [], 0
    for s in insz:
        ins.append(inw[o:o + s].tolist())
        o += s
    o = 0
    for s in outsz:
        outs.append(outw[o:o + s].tolist())
        o += s
    return dict(wires=int(wires), gates=gates.reshape(-1, 4), levels=levels, inputs=ins, outputs=outs)


class sim:
    """One protocol call by three in-process parties on one GPU, with the
    reference unit tests' seeds (include/aby3.h aby3h_sim_*). Each returns
    (shares[3][2][n], revealed) as numpy int64, in the oracle's layout."""

    @staticmethod
    def _np():
        import numpy as np

        return np

    @staticmethod
    def _call(fn, *args):
        h = host()
        if getattr(h, fn)(*args) != 0:
            raise NativeError(f"{fn}: " + h.aby3h_sim_last_error().decode())

    @staticmethod
    def _p(a):
        return a.ctypes.data_as(c_void_p)

    @classmethod
    def mul(cls, mode, trunc, d, a, b, M, K, N, device=0):
        np = cls._np()
        a, b = np.ascontiguousarray(a, np.int64), np.ascontiguousarray(b, np.int64)
        n = M * N if mode == 1 else M * K  # Hadamard: a, b and C are M x K
        if a.size != M * K or b.size != (K * N if mode == 1 else M * K):
            raise ValueError("sim.mul: operand sizes do not match M, K, N")
        sh, plain = np.zeros(6 * n, np.int64), np.zeros(n, np.int64)
        cls._call("aby3h_sim_mul", device, mode, int(trunc), d, cls._p(a), cls._p(b), M, K, N, cls._p(sh),
                  cls._p(plain))
        return sh.reshape(3, 2, -1), plain

    @classmethod
    def mul_bit(cls, kind, a, apub, bits, device=0):
        np = cls._np()
        n = len(bits)
        a = np.ascontiguousarray(a if a is not None else np.zeros(n), np.int64)
        bits = np.ascontiguousarray(bits, np.int64)
        sh, plain = np.zeros(6 * n, np.int64), np.zeros(n, np.int64)
        cls._call("aby3h_sim_mul_bit", device, kind, cls._p(a), apub, cls._p(bits), n, cls._p(sh), cls._p(plain))
        return sh.reshape(3, 2, -1), plain

    @classmethod
    def circuit(cls, name, size, param, rows, inputs, device=0):
        """inputs: one [rows, ceil(bits/64)] int64 array per input bundle;
        returns (shares per output bundle, revealed per output bundle)."""
        np = cls._np()
        cir = circuit(name, size, param)
        ins = np.ascontiguousarray(np.concatenate([np.asarray(x, np.int64).reshape(-1) for x in inputs]))
        cols = [(len(o) + 63) // 64 for o in cir["outputs"]]
        outs, sh = np.zeros(rows * sum(cols), np.int64), np.zeros(6 * rows * sum(cols), np.int64)
        cls._call("aby3h_sim_circuit", device, name.encode(), size, param, rows, cls._p(ins), cls._p(outs),
                  cls._p(sh))
        res, shs, o = [], [], 0
        for c in cols:
            res.append(outs[o:o + rows * c].reshape(rows, c))
            shs.append(sh[6 * o:6 * (o + rows * c)].reshape(3, 2, rows * c))
            o += rows * c
        return shs, res

    @classmethod
    def piecewise(cls, kind, x, D, device=0):
        np = cls._np()
        x = np.ascontiguousarray(x, np.int64)
        n = len(x)
        sh, plain = np.zeros(6 * n, np.int64), np.zeros(n, np.int64)
        cls._call("aby3h_sim_piecewise", device, kind, cls._p(x), n, D, cls._p(sh), cls._p(plain))
        return sh.reshape(3, 2, -1), plain

    @classmethod
    def shuffle(cls, x, mode=0, device=0):
        """x [len][unit] int64; returns (shares [3][2][len*unit], revealed
        [len][unit], permutation shares [3][2][len] or None)."""
        np = cls._np()
        x = np.ascontiguousarray(np.asarray(x, np.int64).reshape(len(x), -1))
        n, unit = x.shape
        sh, plain = np.zeros(6 * n * unit, np.int64), np.zeros(n * unit, np.int64)
        pi = np.zeros(6 * n, np.int64) if mode == 2 else None
        cls._call("aby3h_sim_shuffle", device, mode, cls._p(x), n, unit, cls._p(sh),
                  cls._p(pi) if pi is not None else None, cls._p(plain))
        return sh.reshape(3, 2, -1), plain.reshape(n, unit), (pi.reshape(3, 2, -1) if pi is not None else None)

    @classmethod
    def cipher_gt(cls, a, b, device=0):
        np = cls._np()
        a, b = np.ascontiguousarray(a, np.int64), np.ascontiguousarray(b, np.int64)
        n = len(a)
        sh, plain = np.zeros(6 * n, np.int64), np.zeros(n, np.int64)
        cls._call("aby3h_sim_cipher_gt", device, cls._p(a), cls._p(b), n, cls._p(plain), cls._p(sh))
        return sh.reshape(3, 2, -1), plain

    @classmethod
    def lr(cls, X, Y, batches, D=16, aB=11, device=0):
        """SGD_Logistic iterations on (X [n][d], Y [n]) fixed point, one per row
        of batches [iters][B]; returns (w shares [3][2][d], revealed w)."""
        np = cls._np()
        X = np.ascontiguousarray(X, np.int64)
        Y = np.ascontiguousarray(Y, np.int64).reshape(-1)
        batches = np.ascontiguousarray(batches, np.uint64)
        n, d = X.shape
        iters, B = batches.shape
        sh = np.zeros(6 * d, np.int64)
        w = np.zeros(d, np.int64)
        cls._call("aby3h_sim_lr", device, n, d, B, D, aB, iters, cls._p(X), cls._p(Y), cls._p(batches), cls._p(sh),
                  cls._p(w))
        return sh.reshape(3, 2, d), w

    @classmethod
    def merge(cls, lists, mode=0, dim=0, shares=False, device=0):
        """The merge network (aby3h_sim_merge): mode 0 odd_even_multi_merge of
        separately shared lists, 1 the flat form (singletons: the sort),
        2 high_dimensional_odd_even_multi_merge (lists [dim][k], flattened),
        3 high_dimensional_odd_even_merge, 4 / 5 mode 0 / 2 in the
        reference's sequential merge order. Returns the revealed result, and
        with shares=True also every party's shares [3][2][n]."""
        np = cls._np()
        lens = np.asarray([len(x) for x in lists], np.uint64)
        keys = np.ascontiguousarray(np.concatenate([np.asarray(x, np.int64) for x in lists]))
        out = np.zeros(len(keys), np.int64)
        sh = np.zeros(6 * len(keys), np.int64) if shares else None
        cls._call("aby3h_sim_merge", device, mode, cls._p(lens), len(lists), dim, cls._p(keys), cls._p(out),
                  cls._p(sh) if shares else None)
        return (out, sh.reshape(3, 2, len(keys))) if shares else out


_lib = None


def lr_dataset(n: int, dim: int = 128, D: int = 16):
    """The C4 dataset (LogisticModelGen, fixed point D): (X [n][dim], Y [n], model [dim])."""
    import numpy as np

    X = np.zeros((n, dim), np.int64)
    Y = np.zeros(n, np.int64)
    m = np.zeros(dim, np.float64)
    if host().aby3h_lr_dataset(n, dim, D, X.ctypes.data_as(c_void_p), Y.ctypes.data_as(c_void_p),
                               m.ctypes.data_as(c_void_p)):
        raise NativeError(host().aby3h_sim_last_error().decode())
    return X, Y, m


def lr_batches(n: int, B: int = 256, iters: int = 1):
    """getSubset's first `iters` mini-batches of B rows over n: [iters][B]."""
    import numpy as np

    out = np.zeros((iters, B), np.uint64)
    if host().aby3h_lr_batches(n, B, iters, out.ctypes.data_as(c_void_p)):
        raise NativeError(host().aby3h_sim_last_error().decode())
    return out


def lib() -> _Lib:
    global _lib
    if _lib is None:
        _lib = _Lib()
    return _lib
