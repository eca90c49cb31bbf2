// Share conversions (aby3/sh3/Sh3Converter.cpp) on the GPU: the randomized
// arithmetic-to-binary resharing that feeds the adder circuit of
// toBinaryMatrix (:61-207), and the per-bit 3-party OT of bitInjection
// (:209-371) whose choice bits come straight from packed sbMatrix rows.
//
// All element-wise and HBM/AES bound: one element (or one stream counter)
// per thread, grid-stride, the AES T-tables in LDS as every other randomness
// kernel (common.h). Bit k of a packed [rows][cols64] share matrix with
// `bits` bits per row is row k / bits, bit k % bits (BitVector::append of
// each row's first `bits` bits, Sh3Converter.cpp:240-247).
#include "common.h"

namespace aby3g {

namespace {

constexpr u32 kBlock = 256;

__device__ __forceinline__ u32 packed_bit(const i64* __restrict__ p, u64 k, u64 bits, u64 cols64) {
    const u64 i = k / bits, j = k - i * bits;
    return (u32)(((u64)p[i * cols64 + (j >> 6)] >> (j & 63)) & 1);
}

// toBinaryMatrix's resharing, one party's part (Sh3Converter.cpp:73-197):
// r = stream word (w0 + e) (when the key is given), then
//   out_r[e] = r & m(e)
//   out_x[e] = ((a[e] + b[e]) ^ (xor_r ? r : 0)) & m(e)     (b optional)
// with m(e) = last_mask on the last word of a row, all ones elsewhere.
__global__ void __launch_bounds__(kBlock, 4) k_a2b_reshare(const u32* __restrict__ T0g, AesKey k, int draw, u64 w0,
                                                          u64 n, u64 cols64, u64 last_mask, const i64* __restrict__ a,
                                                          const i64* __restrict__ b, int xor_r, i64* __restrict__ out_x,
                                                          i64* __restrict__ out_r) {
    __shared__ u32 lds[kAesLdsWords];
    if (draw) aes_fill_lds(lds, T0g);
    const u32 lane32 = threadIdx.x & 31;
    auto emit = [&](u64 e, u64 r) {
        const u64 m = (e % cols64 == cols64 - 1) ? last_mask : ~0ull;
        if (out_r) out_r[e] = (i64)(r & m);
        if (out_x) {
            u64 v = (u64)a[e];
            if (b) v += (u64)b[e];
            if (xor_r) v ^= r;
            out_x[e] = (i64)(v & m);
        }
    };
    const u64 stride = (u64)gridDim.x * blockDim.x;
    if (!draw) {
        for (u64 e = (u64)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) emit(e, 0);
        return;
    }
    // one counter per thread: stream words 2c and 2c + 1
    const u64 c_first = w0 >> 1, c_last = (w0 + n - 1) >> 1;
    for (u64 c = c_first + (u64)blockIdx.x * blockDim.x + threadIdx.x; c <= c_last; c += stride) {
        u64 lo, hi;
        aes_ctr_block(lds, lane32, k, c, lo, hi);
        const u64 j = 2 * c;
        if (j >= w0) emit(j - w0, lo);
        if (j + 1 - w0 < n) emit(j + 1 - w0, hi);
    }
}

// bitInjection, sender P2 (Sh3Converter.cpp:319-361): d0 = next word
// (nw0 + k), d1 = prev word (pw0 + k); b = bit k of in0 ^ in1;
// m[c] = -d0 - d1 + (c ^ b); msgs_x[k] = pad(key_x, ctr_x + k) ^ m.
// One thread per next-stream block: its two words are bits k and k + 1, so
// each stream block is encrypted once (the prev stream's two words share a
// block too when both offsets have the same parity, the usual case).
__global__ void __launch_bounds__(kBlock, 4) k_bitinj_send(const u32* __restrict__ T0g, const i64* __restrict__ in0,
                                                          const i64* __restrict__ in1, u64 n, u64 bits, u64 cols64,
                                                          AesKey kn, u64 nw0, AesKey kp, u64 pw0, AesKey ka, u64 ca,
                                                          AesKey kb, u64 cb, int have_b, i64* __restrict__ d0,
                                                          i64* __restrict__ d1, i64* __restrict__ msgs_a,
                                                          i64* __restrict__ msgs_b) {
    __shared__ u32 lds[kAesLdsWords];
    aes_fill_lds(lds, T0g);
    const u32 lane32 = threadIdx.x & 31;
    const bool sameParity = ((nw0 ^ pw0) & 1) == 0;
    const u64 c_first = nw0 >> 1, c_last = (nw0 + n - 1) >> 1;
    for (u64 c = c_first + (u64)blockIdx.x * blockDim.x + threadIdx.x; c <= c_last;
         c += (u64)gridDim.x * blockDim.x) {
        const u64 kbase = 2 * c - nw0;  // bit of word 2c (wraps to ~0 when nw0 is odd and c == c_first)
        const u64 pwb = pw0 + kbase;    // prev word of that bit
        u64 nv[2], pv[2];
        if (sameParity) {
            aes_ctr_block2(lds, lane32, kn, c, kp, pwb >> 1, nv[0], nv[1], pv[0], pv[1]);
        } else {  // prev words pwb (odd) and pwb + 1 straddle two blocks
            u64 alo, ahi, blo, bhi;
            aes_ctr_block(lds, lane32, kn, c, nv[0], nv[1]);
            // the second word's block from its own index: pwb wraps to ~0 when
            // nw0 is odd and pw0 == 0 (bit -1 of the first counter is not emitted)
            aes_ctr_block2(lds, lane32, kp, pwb >> 1, kp, (pwb + 1) >> 1, alo, ahi, blo, bhi);
            pv[0] = ahi;
            pv[1] = blo;
        }
#pragma unroll
        for (u32 h = 0; h < 2; ++h) {
            const u64 k = kbase + h;
            if (k >= n) continue;
            const u32 b = packed_bit(in0, k, bits, cols64) ^ packed_bit(in1, k, bits, cols64);
            const u64 x0 = nv[h], x1 = pv[h];
            d0[k] = (i64)x0;
            d1[k] = (i64)x1;
            const u64 base = 0 - x0 - x1;
            const u64 m0 = base + b, m1 = base + (b ^ 1);
            u64 alo, ahi, blo, bhi;
            if (have_b) {
                aes_ctr_block2(lds, lane32, ka, ca + k, kb, cb + k, alo, ahi, blo, bhi);
                msgs_b[2 * k] = (i64)(blo ^ m0);
                msgs_b[2 * k + 1] = (i64)(bhi ^ m1);
            } else {
                aes_ctr_block(lds, lane32, ka, ca + k, alo, ahi);
            }
            msgs_a[2 * k] = (i64)(alo ^ m0);
            msgs_a[2 * k + 1] = (i64)(ahi ^ m1);
        }
    }
}

// SharedOT::help with packed choice bits (SharedOT.cpp:30-94)
__global__ void __launch_bounds__(kBlock, 4) k_ot_help_bits(const u32* __restrict__ T0g, const i64* __restrict__ in,
                                                           u64 n, u64 bits, u64 cols64, AesKey k, u64 ctr,
                                                           i64* __restrict__ mc) {
    __shared__ u32 lds[kAesLdsWords];
    aes_fill_lds(lds, T0g);
    const u32 lane32 = threadIdx.x & 31;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        u64 lo, hi;
        aes_ctr_block(lds, lane32, k, ctr + i, lo, hi);
        mc[i] = (i64)(packed_bit(in, i, bits, cols64) ? hi : lo);
    }
}

// SharedOT::recv with packed choice bits: out[k] = msgs[k][c_k] ^ mc[k]
__global__ void k_ot_recv_bits(const i64* __restrict__ msgs, const i64* __restrict__ mc, const i64* __restrict__ in,
                               u64 n, u64 bits, u64 cols64, i64* __restrict__ out) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x)
        out[i] = msgs[2 * i + packed_bit(in, i, bits, cols64)] ^ mc[i];
}

// bool2arith's correlated r (BoolBasic.cpp:530-545): PRNG(seed).get<int32_t>()
// sign-extended, times `scale`; one counter (four int32 draws) per thread.
__global__ void __launch_bounds__(kBlock, 4) k_prng_i32(const u32* __restrict__ T0g, AesKey k, u64 w0, u64 n,
                                                       i64 scale, i64* __restrict__ out) {
    __shared__ u32 lds[kAesLdsWords];
    aes_fill_lds(lds, T0g);
    const u32 lane32 = threadIdx.x & 31;
    const u64 c_first = w0 >> 2, c_last = (w0 + n - 1) >> 2;
    for (u64 c = c_first + (u64)blockIdx.x * blockDim.x + threadIdx.x; c <= c_last;
         c += (u64)gridDim.x * blockDim.x) {
        u64 lo, hi;
        aes_ctr_block(lds, lane32, k, c, lo, hi);
        const u32 w[4] = {(u32)lo, (u32)(lo >> 32), (u32)hi, (u32)(hi >> 32)};
#pragma unroll
        for (u32 q = 0; q < 4; ++q) {
            const u64 j = 4 * c + q;
            if (j >= w0 && j - w0 < n) out[j - w0] = (i64)((u64)scale * (u64)(i64)(int32_t)w[q]);
        }
    }
}

// bool2arith, P2 (BoolBasic.cpp:573-587): c = c0 ^ c1 ^ recv, out = c - t
__global__ void k_b2a_open(const i64* __restrict__ c0, const i64* __restrict__ c1, const i64* __restrict__ recv,
                           const i64* __restrict__ t, u64 n, i64* __restrict__ out) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x)
        out[i] = (i64)(((u64)c0[i] ^ (u64)c1[i] ^ (u64)recv[i]) - (u64)t[i]);
}

void check_packed(uint64_t rows, uint64_t cols64, uint64_t bits) {
    ABY3G_REQUIRE(bits >= 1 && (bits + 63) / 64 <= cols64, "bits per row exceed the packed row");
    ABY3G_REQUIRE(rows <= (~0ull) / bits, "rows x bits overflows");
}

}  // namespace

}  // namespace aby3g

using namespace aby3g;

extern "C" {

int aby3g_a2b_reshare(const aby3g_stream_pos* draws, uint64_t n, uint64_t cols64, uint64_t last_mask,
                      const int64_t* a, const int64_t* b, int xor_draws, int64_t* out_x, int64_t* out_r,
                      aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(cols64 >= 1, "cols64 must be >= 1");
        ABY3G_REQUIRE(!draws || draws->off % 8 == 0, "stream offset must be a multiple of 8");
        ABY3G_REQUIRE(draws || (!xor_draws && !out_r), "draws requested without a stream");
        ABY3G_REQUIRE(!out_x || a, "out_x needs a");
        if (!n) return;
        const bool draw = draws != nullptr;
        AesKey k = draw ? expand_key(draws->seed) : AesKey{};
        const u64 w0 = draw ? draws->off / 8 : 0;
        const u64 items = draw ? ((w0 + n - 1) >> 1) - (w0 >> 1) + 1 : n;
        launch(PROBE_AES, k_a2b_reshare, dim3(aes_grid(items, kBlock)), dim3(kBlock), 0, S(stream), aes_table(), k,
               (int)draw, w0, n, cols64, last_mask, a, b, xor_draws, out_x, out_r);
    });
}

int aby3g_bitinj_send(const int64_t* in, uint64_t rows, uint64_t cols64, uint64_t bits,
                      const aby3g_stream_pos* next, const aby3g_stream_pos* prev, const uint8_t key_a[16],
                      uint64_t ctr_a, const uint8_t key_b[16], uint64_t ctr_b, int64_t* dest, int64_t* msgs_a,
                      int64_t* msgs_b, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(in && next && prev && key_a && msgs_a && dest, "null argument");
        ABY3G_REQUIRE(!msgs_b || key_b, "msgs_b needs key_b");
        ABY3G_REQUIRE(next->off % 8 == 0 && prev->off % 8 == 0, "stream offsets must be multiples of 8");
        check_packed(rows, cols64, bits);
        const u64 n = rows * bits;
        if (!n) return;
        AesKey kn = expand_key(next->seed), kp = expand_key(prev->seed), ka = expand_key(key_a);
        AesKey kb = msgs_b ? expand_key(key_b) : ka;
        const u64 nw0 = next->off / 8, items = ((nw0 + n - 1) >> 1) - (nw0 >> 1) + 1;
        launch(PROBE_AES, k_bitinj_send, dim3(aes_grid(items, kBlock)), dim3(kBlock), 0, S(stream), aes_table(), in,
               in + rows * cols64, n, bits, cols64, kn, next->off / 8, kp, prev->off / 8, ka, ctr_a, kb, ctr_b,
               (int)(msgs_b != nullptr), dest, dest + n, msgs_a, msgs_b);
    });
}

int aby3g_ot_help_bits(const int64_t* choice_rows, uint64_t rows, uint64_t cols64, uint64_t bits,
                       const uint8_t ot_key[16], uint64_t ctr, int64_t* mc, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(choice_rows && ot_key && mc, "null argument");
        check_packed(rows, cols64, bits);
        const u64 n = rows * bits;
        if (!n) return;
        AesKey k = expand_key(ot_key);
        launch(PROBE_AES, k_ot_help_bits, dim3(aes_grid(n, kBlock)), dim3(kBlock), 0, S(stream), aes_table(),
               choice_rows, n, bits, cols64, k, ctr, mc);
    });
}

int aby3g_ot_recv_bits(const int64_t* msgs, const int64_t* mc, const int64_t* choice_rows, uint64_t rows,
                       uint64_t cols64, uint64_t bits, int64_t* out, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(msgs && mc && choice_rows && out, "null argument");
        check_packed(rows, cols64, bits);
        const u64 n = rows * bits;
        if (!n) return;
        launch(PROBE_OTHER, k_ot_recv_bits, dim3(aes_grid(n, kBlock)), dim3(kBlock), 0, S(stream), msgs, mc,
               choice_rows, n, bits, cols64, out);
    });
}

int aby3g_prng_i32(const aby3g_stream_pos* s, uint64_t n, int64_t scale, int64_t* out, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(s && out, "null argument");
        ABY3G_REQUIRE(s->off % 4 == 0, "stream offset must be a multiple of 4");
        if (!n) return;
        AesKey k = expand_key(s->seed);
        const u64 w0 = s->off / 4, items = ((w0 + n - 1) >> 2) - (w0 >> 2) + 1;
        launch(PROBE_AES, k_prng_i32, dim3(aes_grid(items, kBlock)), dim3(kBlock), 0, S(stream), aes_table(), k, w0,
               n, (i64)scale, out);
    });
}

int aby3g_b2a_open(const int64_t* c0, const int64_t* c1, const int64_t* recv, const int64_t* t, uint64_t n,
                   int64_t* out, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(c0 && c1 && recv && t && out, "null argument");
        if (!n) return;
        launch(PROBE_OTHER, k_b2a_open, dim3(aes_grid(n, kBlock)), dim3(kBlock), 0, S(stream), c0, c1, recv, t, n,
               out);
    });
}

}  // extern "C"
