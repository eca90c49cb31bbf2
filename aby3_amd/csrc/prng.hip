// AES-CTR correlated randomness on the GPU: PRNG streams, ShareGen draws,
// truncation pairs and the SharedOT pads of the 3-party OT multiplications.
//
// Every kernel here is a grid-stride loop over "windows" of elements; a
// workgroup first builds the 32 KiB replicated T-table in LDS (common.h), then
// produces, for each window, the AES blocks that cover it. Stream word j
// (8 bytes) of PRNG(k) is half (j & 1) of AES(k, j >> 1).
#include "epilogue.h"

namespace aby3g {

namespace {

constexpr u32 kBlock = kEpiBlock;
constexpr u32 kWin = kEpiWin;

__global__ void __launch_bounds__(kBlock, 4) k_aes_ctr(const u32* __restrict__ T0g, AesKey k, u64 base, u64 n,
                                                    u64* __restrict__ out) {
    __shared__ u32 lds[kAesLdsWords];  // static: lookups fold the table base into ds_read's offset
    aes_fill_lds(lds, T0g);
    const u32 lane32 = threadIdx.x & 31;
    const u64 stride = (u64)gridDim.x * blockDim.x;
    // two counters per step, interleaved: i and i + stride
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += 2 * stride) {
        const u64 i2 = i + stride;
        u64 lo, hi, lo2, hi2;
        aes_ctr_block2(lds, lane32, k, base + i, k, base + i2, lo, hi, lo2, hi2);
        out[2 * i] = lo;
        out[2 * i + 1] = hi;
        if (i2 < n) {
            out[2 * i2] = lo2;
            out[2 * i2 + 1] = hi2;
        }
    }
}

// out[i] = stream word (w0 + i), i < n
__global__ void __launch_bounds__(kBlock, 4) k_prng_words(const u32* __restrict__ T0g, AesKey k, u64 w0, u64 n,
                                                       u64* __restrict__ out) {
    __shared__ u32 lds[kAesLdsWords];  // static: lookups fold the table base into ds_read's offset
    aes_fill_lds(lds, T0g);
    const u32 lane32 = threadIdx.x & 31;
    const u64 c_first = w0 >> 1, c_last = (w0 + n - 1) >> 1;
    for (u64 c = c_first + (u64)blockIdx.x * blockDim.x + threadIdx.x; c <= c_last;
         c += (u64)gridDim.x * blockDim.x) {
        u64 lo, hi;
        aes_ctr_block(lds, lane32, k, c, lo, hi);
        u64 j = 2 * c;
        if (j >= w0) out[j - w0] = lo;
        if (j + 1 - w0 < n) out[j + 1 - w0] = hi;
    }
}

// ShareGen draws (Sh3ShareGen.h:60-109). Draw j of either key is word j of
// its AES-CTR stream, so a thread encrypts ONE counter c under both keys
// (the prev schedule in SGPRs, the next one copied to VGPRs: two in SGPRs
// spill) and emits draws 2c and 2c + 1 -- no LDS windows,
// no barriers, and the grid-stride loop balances to one counter.
__global__ void __launch_bounds__(kBlock, 4) k_share_draws(const u32* __restrict__ T0g, AesKeyPair kk, int kind,
                                                           u64 base, u64 n, const i64* __restrict__ addend,
                                                           i64* __restrict__ out0, i64* __restrict__ out1) {
    __shared__ u32 lds[kAesLdsWords];  // static: lookups fold the table base into ds_read's offset
    aes_fill_lds(lds, T0g);
    const u32 lane32 = threadIdx.x & 31;
    const AesKeyV kn = key_to_vgprs(kk.k[1]);
    const u64 c_first = base >> 1, c_last = (base + n - 1) >> 1;
    for (u64 c = c_first + (u64)blockIdx.x * blockDim.x + threadIdx.x; c <= c_last;
         c += (u64)gridDim.x * blockDim.x) {
        u64 p[2], q[2];
        aes_ctr_block(lds, lane32, kk.k[0], c, p[0], p[1]);
        aes_ctr_block_v(lds, lane32, kn, c, q[0], q[1]);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const u64 j = 2 * c + h;
            if (j < base || j - base >= n) continue;
            const u64 i = j - base;
            if (kind == ABY3G_DRAW_ARITH) {
                u64 v = p[h] - q[h];
                if (addend) v += (u64)addend[i];
                out0[i] = (i64)v;
            } else if (kind == ABY3G_DRAW_BIN) {
                u64 v = p[h] ^ q[h];
                if (addend) v ^= (u64)addend[i];
                out0[i] = (i64)v;
            } else {
                out0[i] = (i64)q[h];
                out1[i] = (i64)p[h];
            }
        }
    }
}

// Rows of draws (one party's row slice of the binary engine's masks):
// out0[r * rowLen + i] = draw (base + r * rowStride + i), r < nRows, i < rowLen;
// base, rowLen and rowStride even, so every row is whole counters. A thread
// encrypts one counter under both keys, as k_share_draws.
__global__ void __launch_bounds__(kBlock, 4) k_share_draws_rows(const u32* __restrict__ T0g, AesKeyPair kk, int kind,
                                                                u64 base, u64 rowLen, u64 rowStride, u64 nRows,
                                                                i64* __restrict__ out0) {
    __shared__ u32 lds[kAesLdsWords];  // static: lookups fold the table base into ds_read's offset
    aes_fill_lds(lds, T0g);
    const u32 lane32 = threadIdx.x & 31;
    const AesKeyV kn = key_to_vgprs(kk.k[1]);
    const u64 cpr = rowLen >> 1, total = cpr * nRows;
    for (u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (u64)gridDim.x * blockDim.x) {
        const u64 r = t / cpr, q = t - r * cpr;
        const u64 c = ((base + r * rowStride) >> 1) + q;
        u64 p[2], v[2];
        aes_ctr_block(lds, lane32, kk.k[0], c, p[0], p[1]);
        aes_ctr_block_v(lds, lane32, kn, c, v[0], v[1]);
        i64* o = out0 + r * rowLen + 2 * q;
        o[0] = (i64)(kind == ABY3G_DRAW_ARITH ? p[0] - v[0] : p[0] ^ v[0]);
        o[1] = (i64)(kind == ABY3G_DRAW_ARITH ? p[1] - v[1] : p[1] ^ v[1]);
    }
}

// --- 3-party OT multiplication, party 0 (Sh3Evaluator.cpp:132-163, SharedOT.cpp:6-94)
__global__ void __launch_bounds__(kBlock, 4) k_bitmul_p0(const u32* __restrict__ T0g, const i64* __restrict__ A0,
                                                      const i64* __restrict__ A1, const i64* __restrict__ B0,
                                                      const i64* __restrict__ B1, u64 n, AesKey kprev, u64 pw0,
                                                      AesKey knext, u64 nw0, AesKey kot, u64 ctr,
                                                      i64* __restrict__ C0, i64* __restrict__ C1,
                                                      i64* __restrict__ send, i64* __restrict__ help) {
    __shared__ u32 lds[kAesLdsWords];  // static: lookups fold the table base into ds_read's offset
    aes_fill_lds(lds, T0g);
    constexpr u32 E = kWin / 2;  // 256 elements: 512 prev words, 256 next words
    __shared__ u64 wp[2 * E + 2], wn[E + 2];
    const u32 lane32 = threadIdx.x & 31;
    for (u64 e0 = (u64)blockIdx.x * E; e0 < n; e0 += (u64)gridDim.x * E) {
        const u32 En = (u32)min((u64)E, n - e0);
        __syncthreads();
        stream_window2(lds, kprev, pw0 + 2 * e0, 2 * En, wp, knext, nw0 + e0, En, wn);
        __syncthreads();
        const u32 op = (u32)((pw0 + 2 * e0) & 1), on = (u32)((nw0 + e0) & 1);
        for (u32 e = threadIdx.x; e < En; e += blockDim.x) {
            const u64 i = e0 + e;
            const u32 bb0 = (u32)((B0[i] ^ B1[i]) & 1), bb1 = (u32)(B0[i] & 1);
            const u64 a = (u64)A0[i] + (u64)A1[i];
            const u64 zr = wp[op + 2 * e], c1 = wp[op + 2 * e + 1], c0 = wn[on + e];
            C0[i] = (i64)c0;
            C1[i] = (i64)c1;
            const u64 zz = 0 - (c0 + c1) - zr;
            u64 s[2];
            s[bb0] = zz;
            s[bb0 ^ 1] = a + zz;
            u64 lo, hi, hlo, hhi;  // send pads, help pads
            aes_ctr_block2(lds, lane32, kot, ctr + i, kot, ctr + n + i, lo, hi, hlo, hhi);
            send[2 * i] = (i64)(lo ^ s[0]);
            send[2 * i + 1] = (i64)(hi ^ s[1]);
            help[i] = (i64)(bb1 ? hhi : hlo);
        }
    }
}

// party 2 (Sh3Evaluator.cpp:202-240): help first, then send.
__global__ void __launch_bounds__(kBlock, 4) k_bitmul_p2(const u32* __restrict__ T0g, const i64* __restrict__ A1,
                                                      const i64* __restrict__ B0, const i64* __restrict__ B1, u64 n,
                                                      AesKey knext, u64 nw0, AesKey kot, u64 ctr,
                                                      i64* __restrict__ C0, i64* __restrict__ help,
                                                      i64* __restrict__ send) {
    __shared__ u32 lds[kAesLdsWords];  // static: lookups fold the table base into ds_read's offset
    aes_fill_lds(lds, T0g);
    constexpr u32 E = kWin / 2;
    __shared__ u64 wn[2 * E + 2];
    const u32 lane32 = threadIdx.x & 31;
    for (u64 e0 = (u64)blockIdx.x * E; e0 < n; e0 += (u64)gridDim.x * E) {
        const u32 En = (u32)min((u64)E, n - e0);
        __syncthreads();
        stream_window(lds, knext, nw0 + 2 * e0, 2 * En, wn);
        __syncthreads();
        const u32 on = (u32)((nw0 + 2 * e0) & 1);
        for (u32 e = threadIdx.x; e < En; e += blockDim.x) {
            const u64 i = e0 + e;
            const u32 bb0 = (u32)(B1[i] & 1), bb1 = (u32)((B0[i] ^ B1[i]) & 1);
            const u64 zr = wn[on + 2 * e], c0 = wn[on + 2 * e + 1];
            C0[i] = (i64)c0;
            u64 s[2];
            s[bb1] = zr;
            s[bb1 ^ 1] = (u64)A1[i] + zr;
            u64 lo, hi, hlo, hhi;  // help pads, send pads
            aes_ctr_block2(lds, lane32, kot, ctr + i, kot, ctr + n + i, hlo, hhi, lo, hi);
            help[i] = (i64)(bb0 ? hhi : hlo);
            send[2 * i] = (i64)(lo ^ s[0]);
            send[2 * i + 1] = (i64)(hi ^ s[1]);
        }
    }
}

__global__ void k_ot_recv(const i64* __restrict__ msgs, const i64* __restrict__ mc, const i64* __restrict__ choice,
                          u64 n, int acc, i64* __restrict__ out) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const u32 c = (u32)(choice[i] & 1);
        u64 v = (u64)(msgs[2 * i + c] ^ mc[i]);
        if (acc) v += (u64)out[i];
        out[i] = (i64)v;
    }
}

// public a x shared bit, party 0 (Sh3Evaluator.cpp:430-447)
__global__ void __launch_bounds__(kBlock, 4) k_pubmul_p0(const u32* __restrict__ T0g, i64 a, const i64* __restrict__ B0,
                                                      const i64* __restrict__ B1, u64 n, AesKey kp, AesKey kn,
                                                      u64 dbase, AesKey kon, u64 ctrn, AesKey kop, u64 ctrp,
                                                      i64* __restrict__ mnext, i64* __restrict__ mprev) {
    __shared__ u32 lds[kAesLdsWords];  // static: lookups fold the table base into ds_read's offset
    aes_fill_lds(lds, T0g);
    const u32 lane32 = threadIdx.x & 31;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const u64 j = dbase + i;
        u64 p[2], q[2];
        aes_ctr_block2(lds, lane32, kp, j >> 1, kn, j >> 1, p[0], p[1], q[0], q[1]);
        const u64 zs = p[j & 1] - q[j & 1];
        const u32 bb = (u32)((B0[i] ^ B1[i]) & 1);
        u64 s[2];
        s[bb] = zs;
        s[bb ^ 1] = (u64)a + zs;
        u64 lo, hi, lo2, hi2;
        aes_ctr_block2(lds, lane32, kon, ctrn + i, kop, ctrp + i, lo, hi, lo2, hi2);
        mnext[2 * i] = (i64)(lo ^ s[0]);
        mnext[2 * i + 1] = (i64)(hi ^ s[1]);
        mprev[2 * i] = (i64)(lo2 ^ s[0]);
        mprev[2 * i + 1] = (i64)(hi2 ^ s[1]);
    }
}

// parties 1/2 (Sh3Evaluator.cpp:452-487): share <- getShare(), help pads.
__global__ void __launch_bounds__(kBlock, 4) k_pubmul_helper(const u32* __restrict__ T0g, const i64* __restrict__ choice,
                                                          u64 n, AesKey kp, AesKey kn, u64 dbase, AesKey kot, u64 ctr,
                                                          i64* __restrict__ share, i64* __restrict__ help) {
    __shared__ u32 lds[kAesLdsWords];  // static: lookups fold the table base into ds_read's offset
    aes_fill_lds(lds, T0g);
    const u32 lane32 = threadIdx.x & 31;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const u64 j = dbase + i;
        u64 p[2], q[2];
        aes_ctr_block2(lds, lane32, kp, j >> 1, kn, j >> 1, p[0], p[1], q[0], q[1]);
        share[i] = (i64)(p[j & 1] - q[j & 1]);
        u64 lo, hi;
        aes_ctr_block(lds, lane32, kot, ctr + i, lo, hi);
        help[i] = (i64)((choice[i] & 1) ? hi : lo);
    }
}

}  // namespace

// the share draws' workgroup cap for this thread (aby3g_set_draw_workgroups):
// 256 (one per CU) beside co-located parties' work, more for a party alone
// on its stream (one party per process), where the draws stand in its path
thread_local u32 t_draw_wgs = 256;
inline u32 aes_grid_wide(u64 items, u32 block, u32 cap) {
    u64 g = (items + block - 1) / block;
    if (g > cap) g = cap;
    return (u32)(g ? g : 1);
}

void share_draws_launch(int kind, const u8* kprev, const u8* knext, u64 base, u64 n, const i64* addend, i64* out0,
                        i64* out1, hipStream_t s, int family) {
    ABY3G_REQUIRE(kind >= 0 && kind <= 2, "bad draw kind");
    ABY3G_REQUIRE(kind != ABY3G_DRAW_RANDPAIR || out1, "RANDPAIR needs out1");
    if (!n) return;
    const AesKeyPair kk{{expand_key(kprev), expand_key(knext)}};
    u64 counters = ((base + n - 1) >> 1) - (base >> 1) + 1;
    // at most one workgroup per CU: the draws run beside other work (a
    // circuit's masks beside the previous comparison's latency-bound levels),
    // and fewer 64 KiB-LDS workgroups leave the levels more CUs (C3
    // 0.2999-0.3024 against 0.3088-0.3115 ms with aes_grid's 512, same box;
    // 128 measured 0.344-0.352)
    const u32 grid = std::min<u32>(aes_grid_wide(counters, kBlock, t_draw_wgs), t_draw_wgs);
    launch(family, k_share_draws, dim3(grid), dim3(kBlock), 0, s, aes_table(), kk, kind, base, n, addend, out0, out1);
}

}  // namespace aby3g

using namespace aby3g;

extern "C" {

int aby3g_aes_ctr(const uint8_t key[16], uint64_t ctr_base, uint64_t nblocks, void* out, aby3g_stream stream) {
    return guarded([&] {
        if (!nblocks) return;
        AesKey k = expand_key(key);
        launch(PROBE_AES, k_aes_ctr, dim3(aes_grid(nblocks, kBlock)), dim3(kBlock), 0, S(stream), aes_table(),
               k, ctr_base, nblocks, (u64*)out);
    });
}

int aby3g_prng_fill(const uint8_t seed[16], uint64_t byte_off, uint64_t nbytes, void* out, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(byte_off % 8 == 0 && nbytes % 8 == 0, "offset and length must be multiples of 8");
        if (!nbytes) return;
        AesKey k = expand_key(seed);
        u64 w0 = byte_off / 8, n = nbytes / 8;
        u64 counters = ((w0 + n - 1) >> 1) - (w0 >> 1) + 1;
        launch(PROBE_AES, k_prng_words, dim3(aes_grid(counters, kBlock)), dim3(kBlock), 0, S(stream),
               aes_table(), k, w0, n, (u64*)out);
    });
}

int aby3g_set_draw_workgroups(int cap) {
    return guarded([&] {
        ABY3G_REQUIRE(cap >= 1 && cap <= 4096, "workgroup cap must be 1 .. 4096");
        t_draw_wgs = (u32)cap;
    });
}

int aby3g_share_draws(int kind, const uint8_t k_prev[16], const uint8_t k_next[16], uint64_t draw_base, uint64_t n,
                      const int64_t* addend, int64_t* out0, int64_t* out1, aby3g_stream stream) {
    return guarded(
        [&] { share_draws_launch(kind, k_prev, k_next, draw_base, n, addend, out0, out1, S(stream), PROBE_AES); });
}

int aby3g_share_draws_rows(int kind, const uint8_t k_prev[16], const uint8_t k_next[16], uint64_t draw_base,
                           uint64_t row_len, uint64_t row_stride, uint64_t nrows, int64_t* out0, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(kind == ABY3G_DRAW_ARITH || kind == ABY3G_DRAW_BIN, "row draws: ARITH or BIN only");
        ABY3G_REQUIRE(draw_base % 2 == 0 && row_len % 2 == 0 && row_stride % 2 == 0,
                      "row draws: base, row length and row stride must be even");
        ABY3G_REQUIRE(nrows <= 1 || row_stride >= row_len, "row draws: rows overlap");
        if (!row_len || !nrows) return;
        const AesKeyPair kk{{expand_key(k_prev), expand_key(k_next)}};
        const u64 counters = row_len / 2 * nrows;
        const u32 grid = std::min<u32>(aes_grid_wide(counters, kBlock, t_draw_wgs), t_draw_wgs);
        launch(PROBE_AES, k_share_draws_rows, dim3(grid), dim3(kBlock), 0, S(stream), aes_table(), kk, kind,
               draw_base, row_len, row_stride, nrows, out0);
    });
}

int aby3g_trunc_tuple(const aby3g_trunc_streams* ts, uint64_t n, unsigned d, int64_t* R, int64_t* RT,
                      aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(ts != nullptr, "null trunc streams");
        launch_finish_trunc(SrcNone{}, *ts, n, d, R, RT, RT + n, nullptr, S(stream));
    });
}

int aby3g_bitmul_p0(const int64_t* A, const int64_t* B, uint64_t n, const aby3g_stream_pos* prev,
                    const aby3g_stream_pos* next, const uint8_t ot_key[16], uint64_t ot_ctr, int64_t* C,
                    int64_t* send_msgs, int64_t* help_msgs, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(prev && next, "null stream position");
        ABY3G_REQUIRE(prev->off % 8 == 0 && next->off % 8 == 0, "stream offsets must be multiples of 8");
        if (!n) return;
        AesKey kp = expand_key(prev->seed), kn = expand_key(next->seed), ko = expand_key(ot_key);
        u32 grid = aes_grid((n + 255) / 256, 1);
        launch(PROBE_AES, k_bitmul_p0, dim3(grid), dim3(kBlock), 0, S(stream), aes_table(), A, A + n, B, B + n,
               n, kp, prev->off / 8, kn, next->off / 8, ko, ot_ctr, C, C + n, send_msgs, help_msgs);
    });
}

int aby3g_bitmul_p2(const int64_t* A, const int64_t* B, uint64_t n, const aby3g_stream_pos* next,
                    const uint8_t ot_key[16], uint64_t ot_ctr, int64_t* C, int64_t* help_msgs, int64_t* send_msgs,
                    aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(next != nullptr, "null stream position");
        ABY3G_REQUIRE(next->off % 8 == 0, "stream offset must be a multiple of 8");
        if (!n) return;
        AesKey kn = expand_key(next->seed), ko = expand_key(ot_key);
        u32 grid = aes_grid((n + 255) / 256, 1);
        launch(PROBE_AES, k_bitmul_p2, dim3(grid), dim3(kBlock), 0, S(stream), aes_table(), A + n, B, B + n, n,
               kn, next->off / 8, ko, ot_ctr, C, help_msgs, send_msgs);
    });
}

int aby3g_ot_recv(const int64_t* msgs, const int64_t* mc, const int64_t* choice_src, uint64_t n, int accumulate,
                  int64_t* out, aby3g_stream stream) {
    return guarded([&] {
        if (!n) return;
        launch(PROBE_OTHER, k_ot_recv, dim3(aes_grid(n, 256)), dim3(256), 0, S(stream), msgs, mc, choice_src, n,
               accumulate, out);
    });
}

int aby3g_pubmul_p0(int64_t a, const int64_t* B, uint64_t n, const aby3g_zero_share* zs,
                    const uint8_t ot_next_key[16], uint64_t ctr_next, const uint8_t ot_prev_key[16],
                    uint64_t ctr_prev, int64_t* msgs_next, int64_t* msgs_prev, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(zs != nullptr, "null zero-share keys");
        if (!n) return;
        AesKey kp = expand_key(zs->k_prev), kn = expand_key(zs->k_next);
        AesKey kon = expand_key(ot_next_key), kop = expand_key(ot_prev_key);
        launch(PROBE_AES, k_pubmul_p0, dim3(aes_grid(n, kBlock)), dim3(kBlock), 0, S(stream), aes_table(), a, B,
               B + n, n, kp, kn, zs->draw_base, kon, ctr_next, kop, ctr_prev, msgs_next, msgs_prev);
    });
}

int aby3g_pubmul_helper(const int64_t* choice_src, uint64_t n, const aby3g_zero_share* zs, const uint8_t ot_key[16],
                        uint64_t ctr, int64_t* share_out, int64_t* help_msgs, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(zs != nullptr, "null zero-share keys");
        if (!n) return;
        AesKey kp = expand_key(zs->k_prev), kn = expand_key(zs->k_next), ko = expand_key(ot_key);
        launch(PROBE_AES, k_pubmul_helper, dim3(aes_grid(n, kBlock)), dim3(kBlock), 0, S(stream), aes_table(),
               choice_src, n, kp, kn, zs->draw_base, ko, ctr, share_out, help_msgs);
    });
}

}  // extern "C"
