// Element-wise epilogues of asyncMul that need AES-CTR randomness: the
// zero-share add (Sh3Evaluator.cpp:101-105) and the truncation pair
// (Sh3Evaluator.cpp:503-566, 670-673). They are templated on the source of
// the local share product so that the Hadamard mode computes it in place and
// the GEMM mode reduces its split-K partial slabs in the same pass.
#pragma once
#include "common.h"

namespace aby3g {

// 512-thread workgroups: with the 64 KiB AES table two fit a CU, 16 waves.
constexpr u32 kEpiBlock = 512;
// generic windows (OT kernels): 512 stream words
constexpr u32 kEpiWin = 512;

// win[0 .. 2*nc) <- words of PRNG stream k covering stream words
// [wbase, wbase + E); the word of element e is win[(wbase & 1) + e].
__device__ __forceinline__ void stream_window(const u32* T, const AesKey& k, u64 wbase, u32 E, u64* win) {
    const u64 c0 = wbase >> 1;
    const u32 nc = (u32)(((wbase + E - 1) >> 1) - c0 + 1);
    const u32 lane32 = threadIdx.x & 31;
    for (u32 j = threadIdx.x; j < nc; j += blockDim.x) {
        u64 lo, hi;
        aes_ctr_block(T, lane32, k, c0 + j, lo, hi);
        win[2 * j] = lo;
        win[2 * j + 1] = hi;
    }
}

// Two stream windows at once: wn <- words [nw, nw + En) of kn's stream,
// wp <- words [pw, pw + Ep) of kp's, two AES blocks interleaved per step.
__device__ __forceinline__ void stream_window2(const u32* T, const AesKey& kn, u64 nw, u32 En, u64* wn,
                                               const AesKey& kp, u64 pw, u32 Ep, u64* wp) {
    const u64 cn0 = nw >> 1, cp0 = pw >> 1;
    const u32 ncn = (u32)(((nw + En - 1) >> 1) - cn0 + 1), ncp = (u32)(((pw + Ep - 1) >> 1) - cp0 + 1);
    const u32 nc = ncn > ncp ? ncn : ncp;
    const u32 lane32 = threadIdx.x & 31;
    for (u32 j = threadIdx.x; j < nc; j += blockDim.x) {
        u64 a0, a1, b0, b1;
        aes_ctr_block2(T, lane32, kn, cn0 + j, kp, cp0 + j, a0, a1, b0, b1);
        if (j < ncn) {
            wn[2 * j] = a0;
            wn[2 * j + 1] = a1;
        }
        if (j < ncp) {
            wp[2 * j] = b0;
            wp[2 * j + 1] = b1;
        }
    }
}

// Two AES windows staged in LDS by the two halves of the workgroup: threads
// [0, 256) encrypt counters c00 + j under kk.k[0] into w0, threads
// [256, 512) counters c01 + j under kk.k[1] into w1, j < nc0 / nc1 <= 256.
// Each wave holds one key schedule (two would not fit the SGPR file).
constexpr u32 kPairWin = kEpiBlock / 2;
__device__ __forceinline__ void pair_windows(const u32* T, const AesKeyPair& kk, u64 c00, u32 nc0, u64 c01, u32 nc1,
                                             u64* w0, u64* w1) {
    // wave-uniform (kPairWin is a multiple of 64): readfirstlane keeps the key index scalar
    const u32 h = __builtin_amdgcn_readfirstlane(threadIdx.x) >= kPairWin;
    const u32 j = threadIdx.x - h * kPairWin;
    // the key is loaded through an opaque offset: with a plain kk.k[h] the
    // compiler loads both schedules and selects per use inside the loop
    u32 off = h * (u32)sizeof(AesKey);
    asm volatile("" : "+s"(off));
    const AesKey& k = *reinterpret_cast<const AesKey*>(reinterpret_cast<const char*>(&kk) + off);
    if (j < (h ? nc1 : nc0)) {
        u64 lo, hi;
        aes_ctr_block(T, threadIdx.x & 31, k, (h ? c01 : c00) + j, lo, hi);
        u64* win = h ? w1 : w0;
        win[2 * j] = lo;
        win[2 * j + 1] = hi;
    }
}

// No product: plain getTruncationTuple.
struct SrcNone {
    __device__ u64 operator()(u64) const { return 0; }
};
// GEMM: sum of split-K partial slabs [nsplit][n].
struct SrcSlabs {
    const i64* P;
    u32 nsplit;
    u64 stride;
    __device__ u64 operator()(u64 i) const {
        u64 v = 0;
        for (u32 s = 0; s < nsplit; ++s) v += (u64)P[s * stride + i];
        return v;
    }
};
// GEMM product minus a subtrahend (z = product - R of the truncation pair).
struct SrcSlabsMinus {
    const i64* P;
    u32 nsplit;
    u64 stride;
    const i64* sub;
    __device__ u64 operator()(u64 i) const {
        u64 v = 0;
        for (u32 s = 0; s < nsplit; ++s) v += (u64)P[s * stride + i];
        return v - (u64)sub[i];
    }
};
// Hadamard: A0 B0 + A0 B1 + A1 B0 = A0 (B0 + B1) + A1 B0, mod 2^64.
struct SrcHadamard {
    const i64 *A0, *A1, *B0, *B1;
    __device__ u64 operator()(u64 i) const {
        u64 a0 = (u64)A0[i], a1 = (u64)A1[i], b0 = (u64)B0[i], b1 = (u64)B1[i];
        return a0 * (b0 + b1) + a1 * b0;
    }
};

// Hadamard product minus a subtrahend.
struct SrcHadamardMinus {
    const i64 *A0, *A1, *B0, *B1, *sub;
    __device__ u64 operator()(u64 i) const {
        u64 a0 = (u64)A0[i], a1 = (u64)A1[i], b0 = (u64)B0[i], b1 = (u64)B1[i];
        return a0 * (b0 + b1) + a1 * b0 - (u64)sub[i];
    }
};

// C0[i] = src(i): the share product without a zero-share (used when the
// caller adds randomness itself).
template <class Src>
__global__ void __launch_bounds__(kEpiBlock) k_finish_plain(Src src, u64 n, i64* __restrict__ C0) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x)
        C0[i] = (i64)src(i);
}

// C0[i] = src(i) + getShare(draw_base + i)   (Sh3Evaluator.cpp:101-105)
template <class Src>
__global__ void __launch_bounds__(kEpiBlock, 4) k_finish_zero_share(const u32* __restrict__ T0g, Src src, u64 n,
                                                                    AesKeyPair kk, u64 base, i64* __restrict__ C0) {
    __shared__ u32 lds[kAesLdsWords];  // static: lookups fold the table base into ds_read's offset
    aes_fill_lds(lds, T0g);
    __shared__ u64 wp[2 * kPairWin], wn[2 * kPairWin];
    const u64 c_first = base >> 1, nc = ((base + n - 1) >> 1) - c_first + 1;
    for (u64 w0 = (u64)blockIdx.x * kPairWin; w0 < nc; w0 += (u64)gridDim.x * kPairWin) {
        __syncthreads();
        const u32 m = (u32)min((u64)kPairWin, nc - w0);
        pair_windows(lds, kk, c_first + w0, m, c_first + w0, m, wp, wn);
        __syncthreads();
        const u64 j = 2 * (c_first + w0) + threadIdx.x;
        if (j >= base && j - base < n) {
            const u64 i = j - base;
            C0[i] = (i64)(src(i) + wp[threadIdx.x] - wn[threadIdx.x]);
        }
    }
}

// R = t0 >> 2, RT = (t0 >> (d+2), t1 >> (d+2)); z = src(i) - R when z != null.
// t0 = word (nw0 + i) of the next stream, t1 = word (pw0 + i) of the prev
// stream. No windows: a thread encrypts one counter c of ONE stream and emits
// the elements of its two words 2c, 2c+1 (whatever the stream's parity), so
// threads never exchange words and the grid-stride loop balances to a block.
// Even waves run the next stream (R, RT0, z), odd waves the prev stream
// (RT1): the key is wave-uniform, one schedule in SGPRs.
// The body of k_finish_trunc for workgroup `bid` of `nblocks` (any
// blockDim that is a multiple of 128; lds: kAesLdsWords words).
template <class Src>
__device__ __forceinline__ void trunc_pair_block(u32* lds, const u32* __restrict__ T0g, Src src, const AesKeyPair& kk,
                                                 u64 nw0, u64 pw0, u64 n, u32 d, i64* __restrict__ R,
                                                 i64* __restrict__ RT0, i64* __restrict__ RT1, i64* __restrict__ z,
                                                 u32 bid, u32 nblocks) {
    aes_fill_lds(lds, T0g);
    const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), h = wave & 1, lane = threadIdx.x & 63;
    u32 off = h * (u32)sizeof(AesKey);
    asm volatile("" : "+s"(off));  // opaque: load only the selected schedule
    const AesKey& k = *reinterpret_cast<const AesKey*>(reinterpret_cast<const char*>(&kk) + off);
    const u64 w0 = h ? pw0 : nw0;
    const u64 c_first = w0 >> 1, c_last = (w0 + n - 1) >> 1;
    typedef long long i64x2v __attribute__((ext_vector_type(2)));
    // 16-byte stores: an even stream offset and 16-byte aligned outputs
    const bool vec = (w0 & 1) == 0 && (((uintptr_t)R | (uintptr_t)RT0 | (uintptr_t)RT1 | (uintptr_t)z) & 15) == 0;
    const u64 per = (u64)nblocks * (blockDim.x >> 1);  // threads per stream
    // two counters per step (c, c + per), as k_aes_ctr
    for (u64 c = c_first + ((u64)bid * (blockDim.x >> 7) + (wave >> 1)) * 64 + lane; c <= c_last; c += 2 * per) {
        u64 w[4];
        {
            // interleaved: the two blocks' table reads overlap (latency-bound at small n)
            const AesKey* ks[2] = {&k, &k};
            const u64 ctr[2] = {c, c + per};
            u64 lo[2], hi[2];
            aes_ctr_blocks<2>(lds, threadIdx.x & 31, ks, ctr, lo, hi);
            w[0] = lo[0], w[1] = hi[0], w[2] = lo[1], w[3] = hi[1];
        }
#pragma unroll
        for (int p2 = 0; p2 < 2; ++p2) {
            // the block's two words are elements i, i + 1: one 16-byte store
            // per output when both exist and the stream offset is even
            const u64 j = 2 * (c + p2 * per);
            const u64 i = j - w0;
            if (vec && j >= w0 && i + 1 < n) {
                const i64 t0 = (i64)w[2 * p2], t1 = (i64)w[2 * p2 + 1];
                if (h) {
                    *reinterpret_cast<i64x2v*>(RT1 + i) = i64x2v{t0 >> (d + 2), t1 >> (d + 2)};
                } else {
                    const i64 r0 = t0 >> 2, r1 = t1 >> 2;
                    if (R) *reinterpret_cast<i64x2v*>(R + i) = i64x2v{r0, r1};
                    if (z) *reinterpret_cast<i64x2v*>(z + i) = i64x2v{(i64)(src(i) - (u64)r0), (i64)(src(i + 1) - (u64)r1)};
                    *reinterpret_cast<i64x2v*>(RT0 + i) = i64x2v{t0 >> (d + 2), t1 >> (d + 2)};
                }
                continue;
            }
#pragma unroll
            for (int q = 2 * p2; q < 2 * p2 + 2; ++q) {
                const u64 jq = 2 * (c + (q >> 1) * per) + (q & 1);
                if (jq < w0 || jq - w0 >= n) continue;
                const u64 iq = jq - w0;
                const i64 t = (i64)w[q];
                if (h) {
                    RT1[iq] = t >> (d + 2);
                } else {
                    const i64 r = t >> 2;
                    if (R) R[iq] = r;
                    if (z) z[iq] = (i64)(src(iq) - (u64)r);
                    RT0[iq] = t >> (d + 2);
                }
            }
        }
    }
}

// R = t0 >> 2, RT = (t0 >> (d+2), t1 >> (d+2)); z = src(i) - R when z != null.
// t0 = word (nw0 + i) of the next stream, t1 = word (pw0 + i) of the prev
// stream. No windows: a thread encrypts one counter c of ONE stream and emits
// the elements of its two words 2c, 2c+1 (whatever the stream's parity), so
// threads never exchange words and the grid-stride loop balances to a block.
// Even waves run the next stream (R, RT0, z), odd waves the prev stream
// (RT1): the key is wave-uniform, one schedule in SGPRs.
template <class Src>
__global__ void __launch_bounds__(kEpiBlock) k_finish_trunc(const u32* __restrict__ T0g, Src src, AesKeyPair kk,
                                                            u64 nw0, u64 pw0, u64 n, u32 d, i64* __restrict__ R,
                                                            i64* __restrict__ RT0, i64* __restrict__ RT1,
                                                            i64* __restrict__ z) {
    __shared__ u32 lds[kAesLdsWords];  // static: lookups fold the table base into ds_read's offset
    trunc_pair_block(lds, T0g, src, kk, nw0, pw0, n, d, R, RT0, RT1, z, blockIdx.x, gridDim.x);
}

template <class Src>
void launch_finish_zero_share(Src src, u64 n, const aby3g_zero_share& zs, i64* C0, hipStream_t s) {
    if (!n) return;
    const AesKeyPair kk{{expand_key(zs.k_prev), expand_key(zs.k_next)}};
    u64 counters = ((zs.draw_base + n - 1) >> 1) - (zs.draw_base >> 1) + 1;
    launch(PROBE_EPILOGUE, k_finish_zero_share<Src>, dim3(aes_grid(counters, kPairWin)), dim3(kEpiBlock), 0, s,
           aes_table(), src, n, kk, zs.draw_base, C0);
}

template <class Src>
void launch_finish_plain(Src src, u64 n, i64* C0, hipStream_t s) {
    if (!n) return;
    launch(PROBE_EPILOGUE, k_finish_plain<Src>, dim3(aes_grid(n, kEpiBlock)), dim3(kEpiBlock), 0, s, src, n, C0);
}

template <class Src>
void launch_finish_trunc(Src src, const aby3g_trunc_streams& ts, u64 n, unsigned d, i64* R, i64* RT0, i64* RT1,
                         i64* z, hipStream_t s) {
    ABY3G_REQUIRE(ts.next_off % 8 == 0 && ts.prev_off % 8 == 0, "stream offsets must be multiples of 8");
    ABY3G_REQUIRE(d < 62, "shift too large");
    if (!n) return;
    const AesKeyPair kk{{expand_key(ts.next_seed), expand_key(ts.prev_seed)}};
    // one workgroup per CU at most (half aes_grid's cap): half the 64 KiB
    // table fills, and the pass shares the chip with the co-located parties'
    // share GEMMs (C2 0.2527-0.2547 against 0.2546-0.2557 ms with 512, same
    // box; 128 measured 0.265)
    const u32 grid = std::min<u32>(aes_grid(n / 2 + 1, kEpiBlock / 2), 256);
    launch(PROBE_EPILOGUE, k_finish_trunc<Src>, dim3(grid), dim3(kEpiBlock), 0, s, aes_table(), src, kk,
           ts.next_off / 8, ts.prev_off / 8, n, (u32)d, R, RT0, RT1, z);
}

}  // namespace aby3g
