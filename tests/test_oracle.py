"""Pins the CPU oracle (test infrastructure) before it is trusted:
  * AES-128 against the FIPS-197 known-answer vectors and OpenSSL's libcrypto;
  * the cryptoTools PRNG / ShareGen / SharedOT semantics of SURVEY.md
    Appendix A (stream = AES-CTR bytes, zero-sum shares, OT pad layout);
  * every protocol at the revealed level against the reference's own
    test expectations (Sh3EvaluatorTests.cpp, Sh3BinaryEvaluatorTests.cpp,
    CircuitTests.cpp, Sh3PiecewiseTests.cpp, Test.cpp, BoolTest.cpp).
CPU only."""
import ctypes
import ctypes.util

import numpy as np
import pytest

import oracle as orc

FIPS197 = [
    # (key, plaintext, ciphertext): FIPS-197 Appendix B and C.1, and the all-zero KAT
    ("2b7e151628aed2a6abf7158809cf4f3c", "3243f6a8885a308d313198a2e0370734", "3925841d02dc09fbdc118597196a0b32"),
    ("000102030405060708090a0b0c0d0e0f", "00112233445566778899aabbccddeeff", "69c4e0d86a7b0430d8cdb78070b4c55a"),
    ("00000000000000000000000000000000", "00000000000000000000000000000000", "66e94bd4ef8a2c3b884cfa59ca342b2e"),
]


@pytest.mark.parametrize("k,p,c", FIPS197)
def test_aes_fips197(k, p, c):
    assert orc.aes_ref(bytes.fromhex(k), bytes.fromhex(p)).hex() == c


def test_aesni_matches_reference():
    key = bytes(range(16))
    assert np.array_equal(orc.aes_ctr(key, 123456789, 333), orc.aes_ctr(key, 123456789, 333, use_ref=True))


def _openssl_ecb(key: bytes, data: bytes) -> bytes:
    name = ctypes.util.find_library("crypto")
    if not name:
        pytest.skip("libcrypto not present")
    L = ctypes.CDLL(name)
    L.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
    L.EVP_aes_128_ecb.restype = ctypes.c_void_p
    ctx = L.EVP_CIPHER_CTX_new()
    assert L.EVP_EncryptInit_ex(ctypes.c_void_p(ctx), ctypes.c_void_p(L.EVP_aes_128_ecb()), None, key, None) == 1
    L.EVP_CIPHER_CTX_set_padding(ctypes.c_void_p(ctx), 0)
    out = ctypes.create_string_buffer(len(data) + 16)
    n = ctypes.c_int(0)
    assert L.EVP_EncryptUpdate(ctypes.c_void_p(ctx), out, ctypes.byref(n), data, len(data)) == 1
    L.EVP_CIPHER_CTX_free(ctypes.c_void_p(ctx))
    return out.raw[:n.value]


def test_aes_ctr_matches_openssl():
    key = bytes.fromhex("0f1e2d3c4b5a69788796a5b4c3d2e1f0")
    blocks = b"".join(int(c).to_bytes(8, "little") + bytes(8) for c in range(1000, 1256))
    assert _openssl_ecb(key, blocks) == orc.aes_ctr(key, 1000, 256).tobytes()


def test_prng_stream_is_aes_counter_mode():
    seed = orc.to_block(3488535245, 2454523)
    s = orc.prng_bytes(seed, 0, 64)
    assert s == orc.aes_ctr(seed, 0, 4).tobytes()
    # byte-contiguous: any window is a slice of the stream
    assert orc.prng_bytes(seed, 24, 16) == s[24:40]


def test_to_block_layout():
    # toBlock(hi, lo) = LE64(lo) || LE64(hi)
    assert orc.to_block(1, 2) == (2).to_bytes(8, "little") + (1).to_bytes(8, "little")


def _keys(c):
    return [orc.party_keys(orc.to_block(c, i), orc.to_block(c, (i + 1) % 3)) for i in range(3)]


def test_zero_shares_sum_to_zero():
    # Sh3ShareGen: nextSeed_i == prevSeed_{i+1}, so getShare() over the parties sums to 0
    keys = _keys(0)
    draws = [orc.share_draws(0, k[0], k[1], 0, 1000)[0].view(np.uint64) for k in keys]
    assert np.all(draws[0] + draws[1] + draws[2] == 0)
    bins = [orc.share_draws(1, k[0], k[1], 7, 1000)[0] for k in keys]
    assert np.all(bins[0] ^ bins[1] ^ bins[2] == 0)


def test_rand_int_share_is_replicated():
    # getRandIntShare: party i's r[1] equals party i-1's r[0] (Sh3ShareGen.h:95-109)
    keys = _keys(5)
    r = [orc.share_draws(2, k[0], k[1], 3, 100) for k in keys]
    for i in range(3):
        assert np.array_equal(r[i][1], r[(i + 2) % 3][0])


def test_ot_keys_shared_between_sender_and_helper():
    # P0's mOtNextRecver key (prev stream block 1) == P2's mOtPrevRecver key (next stream block 1)
    keys = _keys(1)
    assert keys[0][3] == keys[2][2]
    assert keys[1][3] == keys[0][2]


def _rand(n, seed, bound=None):
    rng = np.random.default_rng(seed)
    if bound is None:
        return rng.integers(-(2**63), 2**63 - 1, size=n, dtype=np.int64, endpoint=True)
    return rng.integers(-bound, bound, size=n, dtype=np.int64)


@pytest.mark.parametrize("mode,M,K,N", [(1, 10, 10, 10), (1, 7, 13, 5), (0, 10, 10, 10), (0, 31, 9, 1)])
def test_sim_mul_reveals_product(mode, M, K, N):
    # Sh3_Evaluator_mul_test (GEMM, :594-690) / the fork's Hadamard (Test.cpp:116)
    a = _rand(M * K, 1)
    b = _rand(K * N if mode == 1 else M * K, 2)
    _, plain = orc.sim_mul(mode, False, 0, a, b, M, K, N)
    if mode == 1:
        exp = (a.reshape(M, K).astype(object) @ b.reshape(K, N).astype(object)).reshape(-1)
    else:
        exp = a.astype(object) * b.astype(object)
    exp = np.array([int(x) % 2**64 for x in exp], dtype=np.uint64).view(np.int64)
    assert np.array_equal(plain, exp)


@pytest.mark.parametrize("d", [8, 16])
def test_sim_mul_trunc_error_bound(d):
    # Sh3_Evaluator_truncationPai_test bound (:396-407) and matrixFixed (:551)
    M = K = N = 4
    a = _rand(M * K, 3, 1 << 20)
    b = _rand(K * N, 4, 1 << 20)
    _, plain = orc.sim_mul(1, True, d, a, b, M, K, N)
    exact = (a.reshape(M, K) @ b.reshape(K, N)).reshape(-1) >> d
    diff = plain - exact
    assert np.all(diff <= 1) and np.all(diff > -4)


def test_sim_mul_bits():
    n = 100
    a = _rand(n, 5)
    bits = np.random.default_rng(6).integers(0, 2, size=n).astype(np.int64)
    _, plain = orc.sim_mul_bit(0, a, 0, bits)
    assert np.array_equal(plain, np.where(bits == 1, a, 0))
    _, plain = orc.sim_mul_bit(1, a, 123456789, bits)
    assert np.array_equal(plain, np.where(bits == 1, 123456789, 0))
