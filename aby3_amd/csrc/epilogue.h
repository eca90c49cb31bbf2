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
// truncation windows: 510 elements, so that each stream's words span at most
// 256 AES counters -- one block per thread, half the workgroup per stream
constexpr u32 kTruncWin = kEpiBlock - 2;

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
template <class Src>
__global__ void __launch_bounds__(kEpiBlock, 4) k_finish_trunc(const u32* __restrict__ T0g, Src src, AesKeyPair kk,
                                                               u64 nw0, u64 pw0, u64 n, u32 d, i64* __restrict__ R,
                                                            i64* __restrict__ RT0, i64* __restrict__ RT1,
                                                            i64* __restrict__ z) {
    __shared__ u32 lds[kAesLdsWords];  // static: lookups fold the table base into ds_read's offset
    aes_fill_lds(lds, T0g);
    __shared__ u64 wn[kTruncWin + 2], wp[kTruncWin + 2];
    for (u64 e0 = (u64)blockIdx.x * kTruncWin; e0 < n; e0 += (u64)gridDim.x * kTruncWin) {
        const u32 E = (u32)min((u64)kTruncWin, n - e0);
        __syncthreads();
        // kk = (next, prev); each stream's E words span at most kPairWin counters
        const u64 cn = (nw0 + e0) >> 1, cp = (pw0 + e0) >> 1;
        pair_windows(lds, kk, cn, (u32)(((nw0 + e0 + E - 1) >> 1) - cn + 1), cp,
                     (u32)(((pw0 + e0 + E - 1) >> 1) - cp + 1), wn, wp);
        __syncthreads();
        const u32 on = (u32)((nw0 + e0) & 1), op = (u32)((pw0 + e0) & 1);
        for (u32 e = threadIdx.x; e < E; e += blockDim.x) {
            const i64 t0 = (i64)wn[on + e], t1 = (i64)wp[op + e];
            const i64 r = t0 >> 2;
            const u64 i = e0 + e;
            if (R) R[i] = r;
            if (z) z[i] = (i64)(src(i) - (u64)r);
            RT0[i] = t0 >> (d + 2);
            RT1[i] = t1 >> (d + 2);
        }
    }
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
    u32 grid = aes_grid((n + kTruncWin - 1) / kTruncWin, 1);
    launch(PROBE_EPILOGUE, k_finish_trunc<Src>, dim3(grid), dim3(kEpiBlock), 0, s, aes_table(), src, kk,
           ts.next_off / 8, ts.prev_off / 8, n, (u32)d, R, RT0, RT1, z);
}

}  // namespace aby3g
