"""Kernel-level parity: every C-ABI entry point against the CPU oracle on the
same seeded inputs, bit-exact (all arithmetic is integer)."""
import ctypes

import numpy as np
import pytest

import oracle as orc
from aby3_amd import native as nt

pytestmark = pytest.mark.gpu

U64 = 2**64


_KEEP = []  # device tensors whose pointers were handed to a kernel stay alive


@pytest.fixture(autouse=True)
def _release():
    yield
    _KEEP.clear()


def dev(a):
    import torch

    t = torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to("cuda")
    _KEEP.append(t)
    return t


def empty(n):
    import torch

    return torch.zeros(n, dtype=torch.int64, device="cuda")


def host(t):
    import torch

    torch.cuda.synchronize()
    return t.cpu().numpy()


def P(t):
    return ctypes.c_void_p(t.data_ptr())


def rnd(seed, n):
    return np.random.default_rng(seed).integers(-(2**63), 2**63 - 1, size=n, dtype=np.int64, endpoint=True)


def k16(seed):
    return bytes(np.random.default_rng(seed).integers(0, 256, size=16, dtype=np.uint8))


@pytest.mark.parametrize("base,n", [(0, 1), (5, 1000), (2**40 + 3, 4097), (2047, 70001), (2**64 - 100000, 99999)])
def test_aes_ctr(gpu, base, n):
    key = k16(1)
    out = empty(2 * n)
    gpu.aes_ctr(nt.key16(key), base, n, P(out), None)
    assert np.array_equal(host(out).view(np.uint64), orc.aes_ctr(key, base, n))


@pytest.mark.parametrize("off,n", [(0, 8), (8, 24), (16, 1000), (40, 4096 * 8 + 8)])
def test_prng_fill(gpu, off, n):
    seed = k16(2)
    out = empty(n // 8)
    gpu.prng_fill(nt.key16(seed), off, n, P(out), None)
    assert host(out).tobytes() == orc.prng_bytes(seed, off, n)


@pytest.mark.parametrize("kind", [nt.DRAW_ARITH, nt.DRAW_BIN, nt.DRAW_RANDPAIR])
@pytest.mark.parametrize("base,n", [(0, 1), (1, 2), (513, 5000), (3, 200003)])
def test_share_draws(gpu, kind, base, n):
    kp, kn = k16(3), k16(4)
    o0, o1 = empty(n), empty(n)
    gpu.share_draws(kind, nt.key16(kp), nt.key16(kn), base, n, None, P(o0), P(o1), None)
    r0, r1 = orc.share_draws(kind, kp, kn, base, n)
    assert np.array_equal(host(o0), r0)
    if kind == nt.DRAW_RANDPAIR:
        assert np.array_equal(host(o1), r1)
    if kind != nt.DRAW_RANDPAIR:
        add = rnd(5, n)
        gpu.share_draws(kind, nt.key16(kp), nt.key16(kn), base, n, P(dev(add)), P(o0), None, None)
        exp = (r0.view(np.uint64) + add.view(np.uint64)) if kind == nt.DRAW_ARITH else (r0 ^ add).view(np.uint64)
        assert np.array_equal(host(o0).view(np.uint64), exp)


@pytest.mark.parametrize("kind", [nt.DRAW_ARITH, nt.DRAW_BIN])
@pytest.mark.parametrize("base,row_len,stride,nrows", [(0, 32, 64, 5), (64, 96, 512, 181), (1024, 2, 2, 7),
                                                       (6, 4096, 16384, 3), (0, 0, 64, 4), (8, 64, 64, 0)])
def test_share_draws_rows(gpu, kind, base, row_len, stride, nrows):
    """A row slice of the binary engine's masks (aby3g_share_draws_rows):
    row r of the output is draws [base + r*stride, base + r*stride + row_len)
    of the oracle's stream."""
    kp, kn = k16(7), k16(8)
    out = empty(max(row_len * nrows, 1))
    gpu.share_draws_rows(kind, nt.key16(kp), nt.key16(kn), base, row_len, stride, nrows, P(out), None)
    if not row_len or not nrows:
        return
    r0, _ = orc.share_draws(kind, kp, kn, base, stride * (nrows - 1) + row_len)
    exp = np.concatenate([r0[r * stride:r * stride + row_len] for r in range(nrows)])
    assert np.array_equal(host(out), exp)


def test_share_draws_rows_rejects_odd(gpu):
    out = empty(8)
    for args in [(1, 2, 2, 1), (0, 3, 4, 1), (0, 2, 3, 2), (0, 4, 2, 2)]:  # odd base / length / stride, overlap
        with pytest.raises(nt.NativeError):
            gpu.share_draws_rows(nt.DRAW_BIN, nt.key16(k16(7)), nt.key16(k16(8)), *args, P(out), None)


def _zs(kp, kn, base):
    z = nt.ZeroShare()
    z.k_prev[:] = kp
    z.k_next[:] = kn
    z.draw_base = base
    return z


def _mats(M, K, N, mode, seed):
    A = rnd(seed, 2 * M * K)
    B = rnd(seed + 1, 2 * (K * N if mode == nt.MUL_GEMM else M * K))
    return A, B


SHAPES = [(nt.MUL_HADAMARD, 128, 128, 128), (nt.MUL_HADAMARD, 7, 3, 3), (nt.MUL_GEMM, 10, 10, 10),
          (nt.MUL_GEMM, 33, 17, 65), (nt.MUL_GEMM, 256, 128, 1), (nt.MUL_GEMM, 128, 256, 1),
          (nt.MUL_GEMM, 192, 512, 320), (nt.MUL_GEMM, 1024, 1024, 1024),
          # MFMA path with ragged edges (M, N off the 128 x 64 tile, K off 32),
          # and a long K: 564 K'-stages over 32 split-K slabs
          (nt.MUL_GEMM, 257, 200, 250), (nt.MUL_GEMM, 64, 9000, 64)]


@pytest.mark.parametrize("mode,M,K,N", SHAPES)
@pytest.mark.parametrize("with_zs", [False, True])
def test_mul_local(gpu, mode, M, K, N, with_zs):
    if mode == nt.MUL_HADAMARD:
        K = N
    A, B = _mats(M, K, N, mode, 10 + M + K + N)
    n = M * N
    kb = K * N if mode == nt.MUL_GEMM else M * N
    exp = orc.local_product(mode, A[:M * K], A[M * K:], B[:kb], B[kb:], M, K, N)
    ws_bytes = gpu.dll.aby3g_mul_workspace_bytes(mode, M, K, N)
    ws = empty(max(ws_bytes // 8, 1))
    C0 = empty(n)
    zs = None
    if with_zs:
        kp, kn = k16(6), k16(7)
        zs = ctypes.byref(_zs(kp, kn, 77))
        exp = (exp.view(np.uint64) + orc.share_draws(0, kp, kn, 77, n)[0].view(np.uint64)).view(np.int64)
    gpu.mul_local(mode, P(dev(A)), P(dev(B)), P(C0), M, K, N, zs, P(ws), ws_bytes, None)
    assert np.array_equal(host(C0), exp)


def test_gemm_digit_extremes(gpu):
    """Operands at the digit-carry corners: all-ones, 2^63, 0x7f/0x80 bytes."""
    M = K = N = 64
    vals = np.array([-1, -(2**63), 2**63 - 1, 0x7F7F7F7F7F7F7F7F, -0x7F7F7F7F7F7F7F80, 0x8080808080808080 - 2**64,
                     1, 0], dtype=np.int64)
    rng = np.random.default_rng(9)
    A = vals[rng.integers(0, len(vals), 2 * M * K)]
    B = vals[rng.integers(0, len(vals), 2 * K * N)]
    exp = orc.local_product(nt.MUL_GEMM, A[:M * K], A[M * K:], B[:K * N], B[K * N:], M, K, N)
    ws_bytes = gpu.dll.aby3g_mul_workspace_bytes(nt.MUL_GEMM, M, K, N)
    ws = empty(ws_bytes // 8)
    C0 = empty(M * N)
    gpu.mul_local(nt.MUL_GEMM, P(dev(A)), P(dev(B)), P(C0), M, K, N, None, P(ws), ws_bytes, None)
    assert np.array_equal(host(C0), exp)


def _ts(ns, noff, ps, poff):
    t = nt.TruncStreams()
    t.next_seed[:] = ns
    t.next_off = noff
    t.prev_seed[:] = ps
    t.prev_off = poff
    return t


@pytest.mark.parametrize("noff,poff", [(32, 32), (40, 32), (32, 48)])
@pytest.mark.parametrize("d", [8, 16, 27])
@pytest.mark.parametrize("n", [3001, 140001])
def test_trunc_tuple(gpu, noff, poff, d, n):
    ns, ps = k16(11), k16(12)
    R, RT = empty(n), empty(2 * n)
    gpu.trunc_tuple(ctypes.byref(_ts(ns, noff, ps, poff)), n, d, P(R), P(RT), None)
    eR, e0, e1 = orc.trunc_tuple(ns, noff, ps, poff, n, d)
    rt = host(RT)
    assert np.array_equal(host(R), eR)
    assert np.array_equal(rt[:n], e0) and np.array_equal(rt[n:], e1)


@pytest.mark.parametrize("mode,M,K,N", [SHAPES[0], SHAPES[3], SHAPES[4], SHAPES[7]])
def test_mul_trunc_local(gpu, mode, M, K, N):
    if mode == nt.MUL_HADAMARD:
        K = N
    d = 16
    A, B = _mats(M, K, N, mode, 20 + M)
    n = M * N
    kb = K * N if mode == nt.MUL_GEMM else M * N
    prod = orc.local_product(mode, A[:M * K], A[M * K:], B[:kb], B[kb:], M, K, N)
    ns, ps = k16(13), k16(14)
    eR, e0, e1 = orc.trunc_tuple(ns, 32, ps, 40, n, d)
    ws_bytes = gpu.dll.aby3g_mul_workspace_bytes(mode, M, K, N)
    ws = empty(max(ws_bytes // 8, 1))
    z, C = empty(n), empty(2 * n)
    gpu.mul_trunc_local(mode, P(dev(A)), P(dev(B)), M, K, N, d, ctypes.byref(_ts(ns, 32, ps, 40)), P(z), P(C), P(ws),
                        ws_bytes, None)
    assert np.array_equal(host(z), (prod.view(np.uint64) - eR.view(np.uint64)).view(np.int64))
    c = host(C)
    assert np.array_equal(c[:n], e0) and np.array_equal(c[n:], e1)


@pytest.mark.parametrize("party", [0, 1, 2])
def test_trunc_finalize(gpu, party):
    n, d = 999, 13
    za, zb, zo, C = rnd(1, n), rnd(2, n), rnd(3, n), rnd(4, 2 * n)
    Cd = dev(C)
    gpu.trunc_finalize(party, P(dev(za)), P(dev(zb)), P(dev(zo)), d, P(Cd), n, None)
    s = (za.view(np.uint64) + zb.view(np.uint64) + zo.view(np.uint64)).view(np.int64) >> d
    exp = C.copy()
    if party < 2:
        exp[party * n:(party + 1) * n] = (exp[party * n:(party + 1) * n].view(np.uint64) + s.view(np.uint64)).view(
            np.int64)
    assert np.array_equal(host(Cd), exp)


def _bits_ref(x, nbits, words):
    rows = x.shape[0]
    out = np.zeros((nbits, words), dtype=np.uint64)
    xu = x.view(np.uint64)
    sh = np.arange(64, dtype=np.uint64)
    for b in range(nbits):
        col = np.zeros(words * 64, dtype=np.uint64)
        col[:rows] = (xu[:, b // 64] >> np.uint64(b % 64)) & np.uint64(1)
        out[b] = np.bitwise_or.reduce(col.reshape(words, 64) << sh, axis=1)
    return out


@pytest.mark.parametrize("rows,nbits", [(1, 1), (100, 64), (2048, 64), (3000, 70)])
def test_transposes(gpu, rows, nbits):
    cols = (nbits + 63) // 64
    x = rnd(rows + nbits, rows * cols).reshape(rows, cols)
    if nbits % 64:
        x[:, -1] &= np.int64((1 << (nbits % 64)) - 1)
    words = 32 * ((rows + 2047) // 2048)
    W = empty(nbits * words)
    gpu.bits_to_wires(P(dev(x)), rows, cols, nbits, P(W), words, None)
    w = host(W).view(np.uint64).reshape(nbits, words)
    assert np.array_equal(w, _bits_ref(x, nbits, words))
    import torch

    wires = torch.arange(nbits, dtype=torch.int32, device="cuda")
    out = empty(rows * cols)
    gpu.wires_to_bits(P(W), P(wires), nbits, words, P(out), rows, None)
    assert np.array_equal(host(out).reshape(rows, cols), x)


@pytest.mark.parametrize("rows,nbits", [(1, 1), (3000, 70), (4096, 64), (70001, 64), (5000, 130), (70001, 1),
                                        (5000, 7), (2048, 8), (100, 9)])
def test_transposes_both_shares(gpu, rows, nbits):
    """bits_to_wires2 / wires_to_bits2 (both shares, engine memory layout)."""
    import torch

    cols = (nbits + 63) // 64
    x = rnd(rows + 7, 2 * rows * cols).reshape(2, rows, cols)
    if nbits % 64:
        x[:, :, -1] &= np.int64((1 << (nbits % 64)) - 1)
    words = 32 * ((rows + 2047) // 2048)
    wires = nbits + 5  # the input lands at wire 3 of a 2 x wires x words memory
    mem = empty(2 * wires * words)
    gpu.bits_to_wires2(P(dev(x)), rows, cols, nbits, ctypes.c_void_p(mem.data_ptr() + 3 * words * 8), wires * words,
                       words, None)
    m = host(mem).view(np.uint64).reshape(2, wires, words)
    for s in range(2):
        assert np.array_equal(m[s, 3:3 + nbits], _bits_ref(x[s], nbits, words))
    ids = torch.arange(3, 3 + nbits, dtype=torch.int32, device="cuda")
    out = empty(2 * rows * cols)
    gpu.wires_to_bits2(P(mem), wires * words, P(ids), nbits, words, P(out), rows, None)
    assert np.array_equal(host(out).reshape(2, rows, cols), x)


@pytest.mark.parametrize("rows", [1, 4096, 70001])
def test_bits_to_wires_lin(gpu, rows):
    """bits_to_wires_lin: per source the wire rows of sum_t coef_t term_t + c
    (zero wires for a source without terms) and the copy-out, against numpy."""
    import torch

    words = 32 * ((rows + 2047) // 2048)
    t = [rnd(rows + k, rows) for k in range(3)]
    dt = [dev(x) for x in t]
    mem = dev(rnd(9, 3 * 64 * words))  # garbage: every source row must be written
    cp = empty(rows)
    Src = nt.WireSrc * 3
    s = Src()
    at = lambda k: ctypes.cast(mem.data_ptr() + 8 * k * 64 * words, ctypes.POINTER(ctypes.c_uint64))
    i64p = lambda x: ctypes.cast(x.data_ptr(), ctypes.POINTER(ctypes.c_int64))
    for k in range(3):
        s[k].cols64, s[k].nbits, s[k].wire_rows = 1, 64, at(k)
    s[0].term[0], s[0].term[1], s[0].coef[0], s[0].coef[1] = i64p(dt[0]), i64p(dt[1]), 3, -1
    s[0].constant, s[0].copy_out = 1234567, i64p(cp)
    s[2].term[2], s[2].coef[2], s[2].constant = i64p(dt[2]), 1, -5
    gpu.bits_to_wires_lin(s, 3, rows, words, None)
    m = host(mem).view(np.uint64).reshape(3, 64, words)
    with np.errstate(over="ignore"):
        v0 = (3 * t[0].view(np.uint64) - t[1].view(np.uint64))
        e0 = (v0 + np.uint64(1234567)).view(np.int64).reshape(rows, 1)
        e2 = (t[2].view(np.uint64) - np.uint64(5)).view(np.int64).reshape(rows, 1)
    assert np.array_equal(host(cp).view(np.uint64), v0)
    assert np.array_equal(m[0], _bits_ref(e0, 64, words))
    assert not m[1].any()
    assert np.array_equal(m[2], _bits_ref(e2, 64, words))


def test_bits_to_wires_lin_two_columns(gpu):
    """bits_to_wires_lin over a 2-column (100-bit) source: the strided row
    path of the register transpose, trimmed to nbits."""
    rows, nbits, cols = 3001, 100, 2
    words = 32 * ((rows + 2047) // 2048)
    t = rnd(77, rows * cols)
    t.reshape(rows, cols)[:, 1] &= np.int64((1 << (nbits - 64)) - 1)
    mem = dev(rnd(78, nbits * words))
    Src = nt.WireSrc * 1
    s = Src()
    dt = dev(t)
    s[0].cols64, s[0].nbits = cols, nbits
    s[0].wire_rows = ctypes.cast(mem.data_ptr(), ctypes.POINTER(ctypes.c_uint64))
    s[0].term[0] = ctypes.cast(dt.data_ptr(), ctypes.POINTER(ctypes.c_int64))
    s[0].coef[0] = 1
    gpu.bits_to_wires_lin(s, 1, rows, words, None)
    m = host(mem).view(np.uint64).reshape(nbits, words)
    assert np.array_equal(m, _bits_ref(t.reshape(rows, cols), nbits, words))


def _map_rows(first, start, step, per_rep, rep_stride, n):
    q = first + np.arange(n, dtype=np.int64)
    return start + (q // per_rep) * rep_stride + (q % per_rep) * step


@pytest.mark.parametrize("in_rows,rows,mp,padded", [
    (4096, 2048, (0, 0, 1, 1024, 2048), True),      # merge round 0: first halves of 2 lists of 1024
    (4096, 1500, (0, 1, 2, 1500, 4096), True),      # odd slots, one rep
    (5000, 1999, (17, 3, 2, 7, 16), True),          # chunk offset, short reps
    (300, 300, None, True),                          # explicit index list (a permutation)
    (2049, 1, (0, 2048, 1, 1, 0), True),
    (5000, 150, (0, 7, 3, 150, 5000), False),       # 3 words a wire: odd rows of words, unaligned pairs
    (5000, 190, (1, 0, 1, 95, 200), False),
])
def test_transposes_mapped(gpu, in_rows, rows, mp, padded):
    """bits_to_wires_map / wires_to_bits_map (the merge rounds' fused gather
    and scatter) against numpy; the scatter leaves unmapped rows untouched.
    Unpadded word counts (odd, so every other wire row starts 8 bytes off a
    16-byte boundary) take the kernels' one-word paths."""
    import torch

    x = rnd(in_rows + rows, 2 * in_rows).reshape(2, in_rows, 1)
    if mp is None:
        src = np.random.default_rng(rows).permutation(in_rows)[:rows].astype(np.int64)
        idx = torch.from_numpy(src.astype(np.uint32).view(np.int32)).cuda()
        rm = nt.RowMap(0, 0, 0, 1, 0, idx.data_ptr())
    else:
        src = _map_rows(*mp, rows)
        rm = nt.RowMap(*mp, None)
    words = 32 * ((rows + 2047) // 2048) if padded else (rows + 63) // 64
    mem = empty(2 * 64 * words)
    gpu.bits_to_wires_map(P(dev(x)), in_rows, 1, 64, ctypes.byref(rm), rows, P(mem), 64 * words, words, None)
    m = host(mem).view(np.uint64).reshape(2, 64, words)
    for s in range(2):
        assert np.array_equal(m[s], _bits_ref(x[s, src], 64, words))
    ids = torch.arange(64, dtype=torch.int32, device="cuda")
    out_np = rnd(in_rows, 2 * in_rows).reshape(2, in_rows, 1)
    out = dev(out_np)
    gpu.wires_to_bits_map(P(mem), 64 * words, P(ids), 64, words, P(out), in_rows, ctypes.byref(rm), rows, None)
    exp = out_np.copy()
    exp[:, src] = x[:, src]
    assert np.array_equal(host(out).reshape(2, in_rows, 1), exp)


@pytest.mark.parametrize("in_rows,half", [(4096, 2048), (5000, 2400)])
def test_transposes_mapped_pair(gpu, in_rows, half):
    """bits_to_wires_map_n / wires_to_bits_map_n: a compare-exchange round's
    two gathers (first / second elements of each pair) and two scatters in
    one launch each, against numpy."""
    import torch

    x = rnd(in_rows + half, 2 * in_rows).reshape(2, in_rows, 1)
    maps = [(0, 0, 2, half, 0), (0, 1, 2, half, 0)]  # even rows, odd rows
    rms = (nt.RowMap * 2)(*[nt.RowMap(*m, None) for m in maps])
    srcs = [_map_rows(*m, half) for m in maps]
    words = 32 * ((half + 2047) // 2048)
    mem = dev(rnd(3, 2 * 128 * words))  # input 0 at wires 0..63, input 1 at wires 64..127
    dst = (ctypes.c_void_p * 2)(mem.data_ptr(), mem.data_ptr() + 8 * 64 * words)
    gpu.bits_to_wires_map_n(P(dev(x)), in_rows, 1, 64, rms, dst, 2, half, 128 * words, words, None)
    m = host(mem).view(np.uint64).reshape(2, 128, words)
    for s in range(2):
        for k in range(2):
            assert np.array_equal(m[s, 64 * k:64 * k + 64], _bits_ref(x[s, srcs[k]], 64, words))
    # scatter input k's wires back through the other map: rows swap within each pair
    ids = [torch.arange(64 * k, 64 * k + 64, dtype=torch.int32, device="cuda") for k in range(2)]
    wl = (ctypes.c_void_p * 2)(ids[0].data_ptr(), ids[1].data_ptr())
    swapped = (nt.RowMap * 2)(rms[1], rms[0])
    out_np = rnd(in_rows + 1, 2 * in_rows).reshape(2, in_rows, 1)
    out = dev(out_np)
    gpu.wires_to_bits_map_n(P(mem), 128 * words, wl, 64, words, P(out), in_rows, swapped, 2, half, None)
    exp = out_np.copy()
    exp[:, srcs[1]] = x[:, srcs[0]]
    exp[:, srcs[0]] = x[:, srcs[1]]
    assert np.array_equal(host(out).reshape(2, in_rows, 1), exp)


def test_transposes_mapped_rejects_out_of_range(gpu):
    x = empty(2 * 100)
    mem = empty(2 * 64 * 32)
    rm = nt.RowMap(0, 50, 1, 100, 0, None)  # rows 50 .. 149 of a 100-row matrix
    with pytest.raises(nt.NativeError, match="past the matrix"):
        gpu.bits_to_wires_map(P(x), 100, 1, 64, ctypes.byref(rm), 100, P(mem), 64 * 32, 32, None)


@pytest.mark.parametrize("next_off,prev_off,rows,bits,two", [
    (8, 0, 70, 3, 0),      # next word offset odd, prev at 0: the straddling path's first counter
    (16, 8, 33, 64, 1),    # offsets of different parity, one OT
    (24, 40, 50, 7, 0),    # same parity (both odd words)
])
def test_bitinj_send_vs_oracle(gpu, next_off, prev_off, rows, bits, two):
    """bitInjection sender (Sh3Converter.cpp:319-361) through the C-ABI:
    dest words from the next / prev streams at the given offsets, OT messages
    m[c] = -d0 - d1 + (c ^ b) padded with AES(key, ctr + k)."""
    cols = (bits + 63) // 64
    x = rnd(rows + bits, 2 * rows * cols).reshape(2, rows, cols)
    if bits % 64:
        x[:, :, -1] &= np.int64((1 << (bits % 64)) - 1)
    n = rows * bits
    sn, sp, ka, kb = k16(1), k16(2), k16(3), k16(4)
    nxt = nt.StreamPos(nt.key16(sn), next_off)
    prv = nt.StreamPos(nt.key16(sp), prev_off)
    dest, ma = empty(2 * n), empty(2 * n)
    mb = None if two else empty(2 * n)
    gpu.bitinj_send(P(dev(x)), rows, cols, bits, ctypes.byref(nxt), ctypes.byref(prv), nt.key16(ka), 5,
                    nt.key16(kb), 9, P(dest), P(ma), P(mb) if mb is not None else None, None)
    d0 = orc.prng_i64(sn, next_off, n).view(np.uint64)
    d1 = orc.prng_i64(sp, prev_off, n).view(np.uint64)
    xv = (x[0] ^ x[1]).view(np.uint64)
    k = np.arange(n)
    b = (xv[k // bits, (k % bits) // 64] >> (k % bits % 64).astype(np.uint64)) & np.uint64(1)
    base = (np.uint64(0) - d0 - d1)
    m = np.stack([base + b, base + (b ^ np.uint64(1))], axis=1).reshape(-1)
    got = host(dest).view(np.uint64).reshape(2, n)
    assert np.array_equal(got[0], d0) and np.array_equal(got[1], d1)
    pa = orc.aes_ctr(ka, 5, n)
    assert np.array_equal(host(ma).view(np.uint64), pa ^ m)
    if mb is not None:
        assert np.array_equal(host(mb).view(np.uint64), orc.aes_ctr(kb, 9, n) ^ m)


def _gate_ref(t, x0, x1, y0, y1, z):
    if t == 0:
        return x0 ^ y0, x1 ^ y1
    if t == 1:
        return ~(x0 ^ y0), ~(x1 ^ y1)
    if t == 6:
        return x0, x1
    if t == 7:
        return ~x0, ~x1
    if t == 2:
        r = (x0 & y0) ^ (x0 & y1) ^ (x1 & y0)
    elif t == 3:
        r = (x0 & y0) ^ (x0 & y1) ^ (x1 & y0) ^ x0 ^ y0
    elif t == 4:
        r = (~x0 & ~y0) ^ (~x0 & ~y1) ^ (~x1 & ~y0)
    else:
        r = (~x0 & y0) ^ (~x0 & y1) ^ (~x1 & y0)
    return r ^ z, None


def test_bin_gates_and_unpack(gpu):
    import torch

    wires, words = 40, 64
    rng = np.random.default_rng(3)
    mem = rng.integers(0, 2**64, size=2 * wires * words, dtype=np.uint64)
    z = rng.integers(0, 2**64, size=4 * words, dtype=np.uint64)
    gates = [(0, 1, 20, 0), (2, 3, 21, 1), (4, 5, 22, 2), (6, 7, 23, 3), (8, 9, 24, 4), (10, 11, 25, 5),
             (12, 0, 26, 6), (13, 0, 27, 7)]
    arr = (nt.Gate * len(gates))()
    zrow = 0
    for i, (a, b, o, t) in enumerate(gates):
        arr[i].in0, arr[i].in1, arr[i].out, arr[i].type = a, b, o, t
        if t in (2, 3, 4, 5):
            arr[i].z_row = arr[i].send_row = zrow
            zrow += 1
    gdev = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to("cuda")
    memd = dev(mem.view(np.int64))
    send = empty(4 * words)
    gpu.bin_gates(P(gdev), len(gates), P(memd), wires, words, P(dev(z.view(np.int64))), P(send), None)
    out = host(memd).view(np.uint64).reshape(2, wires, words)
    snd = host(send).view(np.uint64).reshape(4, words)
    m = mem.reshape(2, wires, words)
    zr = 0
    for a, b, o, t in gates:
        r0, r1 = _gate_ref(t, m[0, a], m[1, a], m[0, b], m[1, b], z.reshape(4, words)[zr] if t in (2, 3, 4, 5) else 0)
        assert np.array_equal(out[0, o], r0), t
        if r1 is not None:
            assert np.array_equal(out[1, o], r1), t
        else:
            assert np.array_equal(snd[zr], r0)
            zr += 1
    # unpack: share-1 rows of the AND outputs <- a received buffer
    recv = rng.integers(0, 2**64, size=4 * words, dtype=np.uint64)
    outw = torch.tensor([22, 23, 24, 25], dtype=torch.int32, device="cuda")
    gpu.bin_unpack(P(dev(recv.view(np.int64))), P(outw), 4, P(memd), wires, words, None)
    out = host(memd).view(np.uint64).reshape(2, wires, words)
    assert np.array_equal(out[1, 22:26], recv.reshape(4, words))


@pytest.mark.parametrize("words", [32, 4096])
def test_bin_level_matches_unpack_then_batches(gpu, words):
    """aby3g_bin_level == aby3g_bin_unpack + one aby3g_bin_gates per batch,
    with a dependent chain across batches (XOR of an earlier AND output)."""
    import torch

    wires = 48
    rng = np.random.default_rng(words)
    mem = rng.integers(0, 2**64, size=2 * wires * words, dtype=np.uint64)
    z = rng.integers(0, 2**64, size=4 * words, dtype=np.uint64)
    recv = rng.integers(0, 2**64, size=3 * words, dtype=np.uint64)
    unpack = [30, 31, 32]
    # batch 0: independent gates reading unpacked wires; batch 1 consumes batch 0
    batches = [[(30, 1, 20, 2), (31, 3, 21, 0), (32, 5, 22, 5), (6, 7, 23, 7), (8, 9, 24, 3)],
               [(20, 21, 25, 0), (22, 23, 26, 4), (24, 0, 27, 6)],
               [(25, 26, 28, 1)]]
    flat = [g for b in batches for g in b]
    arr = (nt.Gate * len(flat))()
    zrow = 0
    for i, (a, b, o, t) in enumerate(flat):
        arr[i].in0, arr[i].in1, arr[i].out, arr[i].type = a, b, o, t
        if t in (2, 3, 4, 5):
            arr[i].z_row = arr[i].send_row = zrow
            zrow += 1
    gdev = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to("cuda")
    ends = torch.tensor(np.cumsum([len(b) for b in batches]).tolist(), dtype=torch.int32, device="cuda")
    uw = torch.tensor(unpack, dtype=torch.int32, device="cuda")
    zd, rd = dev(z.view(np.int64)), dev(recv.view(np.int64))
    # reference: the separate kernels
    m1, s1 = dev(mem.view(np.int64)), empty(4 * words)
    gpu.bin_unpack(P(rd), P(uw), 3, P(m1), wires, words, None)
    gsz = ctypes.sizeof(nt.Gate)
    first = 0
    for b in batches:
        gpu.bin_gates(ctypes.c_void_p(gdev.data_ptr() + gsz * first), len(b), P(m1), wires, words, P(zd), P(s1), None)
        first += len(b)
    m2, s2 = dev(mem.view(np.int64)), empty(4 * words)
    gpu.bin_level(P(gdev), P(ends), len(batches), P(rd), P(uw), 3, P(m2), wires, words, P(zd), P(s2), None)
    assert np.array_equal(host(m1), host(m2))
    assert np.array_equal(host(s1)[:zrow * words], host(s2)[:zrow * words])
    # aby3g_bin_level_rr: share 1 of the unpacked wires read from the recv rows
    rows = {w: j for j, w in enumerate(unpack)}
    rr = np.array([[rows.get(a, 0xFFFFFFFF), rows.get(b, 0xFFFFFFFF)] for a, b, _, _ in flat], dtype=np.uint32)
    rrd = torch.from_numpy(rr.reshape(-1).view(np.int32).copy()).to("cuda")
    m3, s3 = dev(mem.view(np.int64)), empty(4 * words)
    gpu.bin_level_rr(P(gdev), P(rrd), P(ends), len(batches), P(rd), P(uw), 3, P(m3), wires, words, P(zd), P(s3), None)
    assert np.array_equal(host(m1), host(m3))
    assert np.array_equal(host(s1)[:zrow * words], host(s3)[:zrow * words])


def _timeouts():
    n = ctypes.c_uint32(0)
    nt.lib().handoff_status(ctypes.byref(n))
    return n.value


def test_handoff_residency_rule(gpu):
    """The device's residency figures behind the in-kernel hand-off budget
    (Channel.h handoffResidencyOk): printed for the log, and the C3 / C5
    messages (<= 512 chunks) must still qualify, else a register regression
    of k_bin_level has silently moved them back to stream hand-offs."""
    cus, small, large, smax = (ctypes.c_int() for _ in range(4))
    nt.lib().bin_level_residency(ctypes.byref(cus), ctypes.byref(small), ctypes.byref(large), ctypes.byref(smax))
    print(f"residency: {cus.value} CUs, k_bin_level<32,true,1> {small.value}/CU, <8,true,2,2> {large.value}/CU, "
          f"small form below {smax.value} workgroups")
    assert cus.value >= 1 and small.value >= 1 and large.value >= 1
    per = lambda c: small.value if c < smax.value else large.value  # noqa: E731
    ok = lambda c: 2 * -(-c // per(c)) + 4 + 1 <= cus.value  # noqa: E731
    assert ok(64) and ok(512), "C3/C5 level messages no longer fit the residency rule"


def test_handoff_timeout_gives_up_and_counts(gpu):
    """A level launch waiting on a hand-off whose flags are never written
    gives up after the (shortened) timeout instead of hanging, the device's
    timeout count goes up by one, and a launch enqueued after that -- whose
    flags are set -- runs normally without being aborted by the old timeout."""
    import time

    import torch

    words, wires = 32, 8
    lib = nt.lib()
    gates = (nt.Gate * 1)()
    gates[0].in0, gates[0].in1, gates[0].out, gates[0].type = 0, 1, 2, 0  # one XOR
    gdev = torch.frombuffer(bytearray(bytes(gates)), dtype=torch.uint8).to("cuda")
    ends = torch.tensor([1], dtype=torch.int32, device="cuda")
    uw = torch.tensor([3], dtype=torch.int32, device="cuda")
    mem, recv = empty(2 * wires * words), empty(words)
    flags = empty(4)  # zero: never posted
    before = _timeouts()
    lib.set_handoff_timeout_us(20000)
    try:
        wait = nt.Handoff(ctypes.c_void_p(flags.data_ptr()), 1, None)
        t0 = time.perf_counter()
        lib.bin_level_hs(P(gdev), None, P(ends), 1, P(recv), P(uw), 1, P(mem), wires, words, None, None,
                         ctypes.byref(wait), None, None)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        assert _timeouts() == before + 1
        assert dt < 5, f"the wait took {dt:.2f} s with a 20 ms limit"
        # posted flags now: a fresh wait completes and counts nothing
        flags.fill_(1)
        torch.cuda.synchronize()
        lib.bin_level_hs(P(gdev), None, P(ends), 1, P(recv), P(uw), 1, P(mem), wires, words, None, None,
                         ctypes.byref(wait), None, None)
        torch.cuda.synchronize()
        assert _timeouts() == before + 1
    finally:
        lib.set_handoff_timeout_us(5000000)
    # and a three-party call after it is unaffected by the earlier timeout
    a = np.arange(64, dtype=np.int64).reshape(8, 8)
    sh, plain = nt.sim.mul(1, 0, 0, a, a, 8, 8, 8)
    assert np.array_equal(plain.reshape(8, 8), a @ a)


def test_lincomb_bitops(gpu):
    import torch

    n = 1000
    a, b = rnd(1, n), rnd(2, n)
    o = empty(n)
    gpu.i64_lincomb(n, 3, P(dev(a)), -5, P(dev(b)), 7, P(o), None)
    exp = (np.uint64(3) * a.view(np.uint64) + np.uint64(2**64 - 5) * b.view(np.uint64) + np.uint64(7)).view(np.int64)
    assert np.array_equal(host(o), exp)
    for op, f in [(0, lambda x, y: x ^ y), (1, lambda x, y: x & y), (2, lambda x, y: ~x),
                  (3, lambda x, y: -(x & 1)), (4, lambda x, y: x)]:
        gpu.u64_bitop(op, n, P(dev(a)), P(dev(b)), P(o), None)
        assert np.array_equal(host(o), f(a, b)), op
    idx = np.random.default_rng(4).permutation(n).astype(np.int32)
    idxd = torch.from_numpy(idx).to("cuda")
    gpu.u64_gather(n, P(idxd), P(dev(a)), P(o), None)
    assert np.array_equal(host(o), a[idx])
    gpu.u64_scatter(n, P(idxd), P(dev(a)), P(o), None)
    exp = np.zeros(n, dtype=np.int64)
    exp[idx] = a
    assert np.array_equal(host(o), exp)
