// Shared definitions of the gfx950 engine: error plumbing, the launch probe
// and the device AES-128 used by every randomness kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdint>
#include <string>
#include <vector>
#include "../../include/aby3gpu.h"

namespace aby3g {

using u8 = uint8_t;
using u32 = uint32_t;
using u64 = uint64_t;
using i64 = int64_t;

// ---------------------------------------------------------------- errors --
void set_error(const std::string& msg);
struct Error {
    int code;
    std::string msg;
};
#define ABY3G_CHECK_HIP(expr)                                                                        \
    do {                                                                                             \
        hipError_t e_ = (expr);                                                                      \
        if (e_ != hipSuccess)                                                                        \
            throw ::aby3g::Error{ABY3G_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)};     \
    } while (0)
#define ABY3G_REQUIRE(cond, msg)                                                                     \
    do {                                                                                             \
        if (!(cond)) throw ::aby3g::Error{ABY3G_EINVAL, std::string(__func__) + ": " + (msg)};       \
    } while (0)

// calling thread's time inside C-ABI calls (host overhead accounting)
extern thread_local double t_api_us;
extern thread_local u64 t_api_calls;
struct ApiClock {
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    ~ApiClock() {
        t_api_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        ++t_api_calls;
    }
};

// diagnostics: the names of the process's recent C-ABI calls (a ring of 32),
// so that an asynchronous device fault that surfaces in a later call can be
// traced to the work enqueued just before it (aby3g_recent_calls)
void note_call(const char* name);

template <class F>
int guarded_at(const char* name, F&& f) {
    note_call(name);
    ApiClock clock;
    try {
        f();
        return ABY3G_OK;
    } catch (const Error& e) {
        set_error(e.msg);
        return e.code;
    } catch (const std::exception& e) {
        set_error(e.what());
        return ABY3G_EINVAL;
    }
}
// every C-ABI entry point reads `return guarded([&] { ... });`: the entry's
// own name goes into the ring
#define guarded(...) guarded_at(__func__, __VA_ARGS__)

// ----------------------------------------------------------------- probe --
enum ProbeFamily { PROBE_GEMM = 0, PROBE_EPILOGUE = 1, PROBE_BINARY = 2, PROBE_AES = 3, PROBE_OTHER = 4, PROBE_DIGITS = 5 };
void probe_begin(int family, hipStream_t s);
void probe_end(int family, hipStream_t s);

// Launch helper: checks the launch and feeds the probe.
template <class K, class... Args>
void launch(int family, K kernel, dim3 grid, dim3 block, size_t lds, hipStream_t s, Args... args) {
    if (grid.x == 0 || grid.y == 0 || grid.z == 0) return;
    probe_begin(family, s);
    hipLaunchKernelGGL(kernel, grid, block, lds, s, args...);
    ABY3G_CHECK_HIP(hipGetLastError());
    probe_end(family, s);
}

// ------------------------------------------------------------------- AES --
// Round keys as little-endian column words (byte 4c+r of round key = byte r
// of word c). Passed to kernels by value (176 B of kernarg).
struct AesKey {
    u32 rk[44];
};
AesKey expand_key(const u8 key[16]);
// Two keys as one kernel argument: a kernel that gives each half of its
// workgroup one of them indexes k[] with a wave-uniform value, and only the
// selected schedule is held in SGPRs.
struct AesKeyPair {
    AesKey k[2];
};
// Device copy of T0[x] = 2S | S<<8 | S<<16 | 3S<<24 for the current device
// (computed on the host from the S-box definition, uploaded once).
const u32* aes_table();

// LDS image of the round tables: T0 and T1 = rotl(T0, 8), each replicated
// 32 times, at byte address x << 8 | t << 7 | c << 2 (table t, entry x,
// copy c). Lane l reads copy (l & 31): ds_read_b32 serves a wave in two
// 32-lane halves over 32 banks, so every lane hits its own bank and the
// random lookups are conflict-free. Because the entry sits in address byte 1
// and (table, copy) in byte 0, one v_perm_b32 of (state word, per-lane
// constant) forms a lookup address -- one VALU op instead of extract + scale
// + add. 64 KiB per workgroup.
constexpr int kAesLdsWords = 256 * 64;

__host__ __device__ __forceinline__ u32 rotl(u32 x, int r) { return __builtin_rotateleft32(x, r); }

// The 64 KiB image is 4096 16-byte chunks (entry x: chunks 16x .. 16x + 15,
// the first 8 holding T0[x] four times each, the last 8 T1[x]); consecutive
// threads write consecutive chunks, so every ds_write_b128 of a wave covers
// 1 KiB of consecutive banks, and every table read is in flight before the
// first store. (Measured in the fused LR kernel, whose one workgroup fills
// the table at the start of every launch: 8.4 us for the first fill of a
// launch -- the launch's cold start, kernel arguments and code, whatever the
// fill does: a table computed in registers instead of loaded took as long --
// and 0.8 us for a second fill right after it.)
__device__ __forceinline__ void aes_fill_lds(u32* lds, const u32* __restrict__ T0g) {
    static_assert(kAesLdsWords == 256 * 64, "layout");
    typedef u32 v4u __attribute__((ext_vector_type(4)));
    constexpr u32 kChunks = kAesLdsWords / 4, kU = 16;  // 16 chunks per thread at 256 threads
    v4u* dst = reinterpret_cast<v4u*>(lds);
    u32 v[kU];
#pragma unroll
    for (u32 i = 0; i < kU; ++i) {
        const u32 q = threadIdx.x + i * blockDim.x;
        v[i] = q < kChunks ? T0g[q >> 4] : 0;
    }
#pragma unroll
    for (u32 i = 0; i < kU; ++i) {
        const u32 q = threadIdx.x + i * blockDim.x;
        if (q < kChunks) {
            const u32 x = (q & 8) ? rotl(v[i], 8) : v[i];
            dst[q] = v4u{x, x, x, x};
        }
    }
    for (u32 q = threadIdx.x + kU * blockDim.x; q < kChunks; q += blockDim.x) {  // blocks under 256 threads
        const u32 x = (q & 8) ? rotl(T0g[q >> 4], 8) : T0g[q >> 4];
        dst[q] = v4u{x, x, x, x};
    }
    __syncthreads();
}

// byte offset of the entry (byte j of s) in the table / copy selected by L's byte 0
__host__ __device__ __forceinline__ u32 aes_addr(u32 s, u32 L, int j) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(s, L, 0x0c0c0000u | ((4u + j) << 8));
#else
    return (((s >> (8 * j)) & 0xffu) << 8) | (L & 0xffu);
#endif
}

// a ^ b ^ k in one VALU op, k wave-uniform (a round-key word, kept in an
// SGPR; the compiler does not form v_bitop3 for xor3 itself)
__host__ __device__ __forceinline__ u32 xor3_uniform(u32 a, u32 b, u32 k) {
#if defined(__HIP_DEVICE_COMPILE__)
    u32 r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(k));
    return r;
#else
    return a ^ b ^ k;
#endif
}

// a ^ b ^ k in one VALU op with k in a VGPR (a key schedule held per lane)
__host__ __device__ __forceinline__ u32 xor3_v(u32 a, u32 b, u32 k) {
#if defined(__HIP_DEVICE_COMPILE__)
    u32 r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(k));
    return r;
#else
    return a ^ b ^ k;
#endif
}

// S-box bytes of four T0 entries, packed little-endian: S[x] = byte 1 of T0[x]
__host__ __device__ __forceinline__ u32 aes_sb4(u32 A, u32 B, u32 C, u32 D) {
#if defined(__HIP_DEVICE_COMPILE__)
    const u32 u = __builtin_amdgcn_perm(B, A, 0x0c0c0501u), v = __builtin_amdgcn_perm(D, C, 0x0c0c0501u);
    return __builtin_amdgcn_perm(v, u, 0x05040100u);
#else
    return ((A >> 8) & 0xffu) | (B & 0xff00u) | (((C >> 8) & 0xffu) << 16) | ((D & 0xff00u) << 16);
#endif
}

// 64 x 64 bit transpose across a wave: lane i holds row i (bit k = column k);
// afterwards lane i holds column i (bit k = bit i of row k). Six butterfly
// stages: at stage j the lanes i and i ^ j swap the off-diagonal j x j
// blocks of their 2j x 2j block. The exchanges stay off the LDS pipe
// (ds_bpermute, twelve per transpose, made the C5 mapped transposes ~40 %
// slower): gfx950's v_permlane32_swap does stage 32 in one instruction (lanes
// below 32 keep their low words and take the partner's, lanes above keep
// their high words), v_permlane16_swap stage 16 on 16-bit pieces packed into
// whole words (E: pieces 0 and 2, O: pieces 1 and 3), and DPP row / quad
// permutations the stages within a row of 16 lanes.
template <int kCtrl>
__device__ __forceinline__ u32 dpp_mov(u32 v) {
    return __builtin_amdgcn_update_dpp(0u, v, kCtrl, 0xf, 0xf, false);
}
template <int kCtrl>
__device__ __forceinline__ u64 dpp_mov64(u64 v) {
    return (u64)dpp_mov<kCtrl>((u32)v) | ((u64)dpp_mov<kCtrl>((u32)(v >> 32)) << 32);
}
__device__ __forceinline__ u64 transpose_stage(u64 x, u64 y, u32 lane, u32 j, u64 m) {
    return (lane & j) ? ((x & ~m) | ((y & ~m) >> j)) : ((x & m) | ((y & m) << j));
}
__device__ __forceinline__ u64 transpose64(u64 x, u32 lane) {
    u32 lo = (u32)x, hi = (u32)(x >> 32);
    {  // j = 32
        const auto r = __builtin_amdgcn_permlane32_swap(lo, hi, false, false);
        lo = r[0];
        hi = r[1];
    }
    {  // j = 16
        const u32 e = (lo & 0xffffu) | (hi << 16), o = (lo >> 16) | (hi & 0xffff0000u);
        const auto r = __builtin_amdgcn_permlane16_swap(e, o, false, false);
        lo = (r[0] & 0xffffu) | (r[1] << 16);
        hi = (r[0] >> 16) | (r[1] & 0xffff0000u);
    }
    x = (u64)lo | ((u64)hi << 32);
    x = transpose_stage(x, dpp_mov64<0x128>(x), lane, 8, 0x00FF00FF00FF00FFull);                     // row_ror:8 = i ^ 8
    x = transpose_stage(x, dpp_mov64<0x141>(dpp_mov64<0x1B>(x)), lane, 4, 0x0F0F0F0F0F0F0F0Full);   // (i ^ 3) ^ 7
    x = transpose_stage(x, dpp_mov64<0x4E>(x), lane, 2, 0x3333333333333333ull);                     // quad_perm 2,3,0,1
    x = transpose_stage(x, dpp_mov64<0xB1>(x), lane, 1, 0x5555555555555555ull);                     // quad_perm 1,0,3,2
    return x;
}

// Round-key sources of aes_ctr_blocks. Keys in SGPRs: schedules that are
// kernel arguments (a kernel with one or two keys keeps them resident).
struct AesRkSgpr {
    const AesKey* const* k;
    __host__ __device__ __forceinline__ void round(int b, int r, u32 (&o)[4]) const {
        o[0] = k[b]->rk[4 * r + 0];
        o[1] = k[b]->rk[4 * r + 1];
        o[2] = k[b]->rk[4 * r + 2];
        o[3] = k[b]->rk[4 * r + 3];
    }
    static __host__ __device__ __forceinline__ u32 x3(u32 a, u32 b, u32 k) { return xor3_uniform(a, b, k); }
};
// Keys in LDS (44-word schedules at 16-byte aligned offsets), one broadcast
// ds_read_b128 per round and block: a kernel with many keys would otherwise
// spill them from SGPRs into VGPR lanes, loading the whole kernel-argument
// block up front one dependent 64-byte scalar load at a time.
struct AesRkLds {
    const u32* const* k;
    __device__ __forceinline__ void round(int b, int r, u32 (&o)[4]) const {
        typedef u32 v4u __attribute__((ext_vector_type(4)));
        const v4u v = *reinterpret_cast<const v4u*>(k[b] + 4 * r);
        o[0] = v.x, o[1] = v.y, o[2] = v.z, o[3] = v.w;
    }
    static __device__ __forceinline__ u32 x3(u32 a, u32 b, u32 k) { return xor3_v(a, b, k); }
};

// AES-128 of the counter block LE64(ctr) || 0^8 under key b of `R`, T-table
// form. Column c of the state is the LE word of bytes 4c..4c+3; after
// ShiftRows, row r of column c comes from column c+r, and MixColumns row
// weights of input row r are T0 rotated left by 8r bits, so a column is
//   xor3(T0[a], T1[b], rk) ^ rotl(T0[c] ^ T1[d], 16).
// NB blocks (keys / counters of their own) are interleaved so each round
// issues 16 * NB independent table reads.
template <int NB, class RK>
__host__ __device__ __forceinline__ void aes_ctr_blocks_rk(const u32* __restrict__ T, u32 lane32, const RK& R,
                                                           const u64* ctr, u64* lo, u64* hi) {
    const u8* Tb = reinterpret_cast<const u8*>(T);
    const u32 L0 = lane32 << 2, L1 = L0 | 0x80u;
#define ABY3G_TL(s, L, j) (*reinterpret_cast<const u32*>(Tb + aes_addr((s), (L), (j))))
    u32 s0[NB], s1[NB], s2[NB], s3[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        u32 k[4];
        R.round(b, 0, k);
        s0[b] = (u32)ctr[b] ^ k[0];
        s1[b] = (u32)(ctr[b] >> 32) ^ k[1];
        s2[b] = k[2];
        s3[b] = k[3];
    }
#pragma unroll
    for (int r = 1; r < 10; ++r) {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            u32 k[4];
            R.round(b, r, k);
            const u32 t0 = RK::x3(ABY3G_TL(s0[b], L0, 0), ABY3G_TL(s1[b], L1, 1), k[0]) ^
                           rotl(ABY3G_TL(s2[b], L0, 2) ^ ABY3G_TL(s3[b], L1, 3), 16);
            const u32 t1 = RK::x3(ABY3G_TL(s1[b], L0, 0), ABY3G_TL(s2[b], L1, 1), k[1]) ^
                           rotl(ABY3G_TL(s3[b], L0, 2) ^ ABY3G_TL(s0[b], L1, 3), 16);
            const u32 t2 = RK::x3(ABY3G_TL(s2[b], L0, 0), ABY3G_TL(s3[b], L1, 1), k[2]) ^
                           rotl(ABY3G_TL(s0[b], L0, 2) ^ ABY3G_TL(s1[b], L1, 3), 16);
            const u32 t3 = RK::x3(ABY3G_TL(s3[b], L0, 0), ABY3G_TL(s0[b], L1, 1), k[3]) ^
                           rotl(ABY3G_TL(s1[b], L0, 2) ^ ABY3G_TL(s2[b], L1, 3), 16);
            s0[b] = t0;
            s1[b] = t1;
            s2[b] = t2;
            s3[b] = t3;
        }
    }
    // last round: SubBytes + ShiftRows
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        u32 k[4];
        R.round(b, 10, k);
        const u32 o0 = aes_sb4(ABY3G_TL(s0[b], L0, 0), ABY3G_TL(s1[b], L0, 1), ABY3G_TL(s2[b], L0, 2),
                               ABY3G_TL(s3[b], L0, 3)) ^ k[0];
        const u32 o1 = aes_sb4(ABY3G_TL(s1[b], L0, 0), ABY3G_TL(s2[b], L0, 1), ABY3G_TL(s3[b], L0, 2),
                               ABY3G_TL(s0[b], L0, 3)) ^ k[1];
        const u32 o2 = aes_sb4(ABY3G_TL(s2[b], L0, 0), ABY3G_TL(s3[b], L0, 1), ABY3G_TL(s0[b], L0, 2),
                               ABY3G_TL(s1[b], L0, 3)) ^ k[2];
        const u32 o3 = aes_sb4(ABY3G_TL(s3[b], L0, 0), ABY3G_TL(s0[b], L0, 1), ABY3G_TL(s1[b], L0, 2),
                               ABY3G_TL(s2[b], L0, 3)) ^ k[3];
        lo[b] = (u64)o0 | ((u64)o1 << 32);
        hi[b] = (u64)o2 | ((u64)o3 << 32);
    }
#undef ABY3G_TL
}

template <int NB>
__host__ __device__ __forceinline__ void aes_ctr_blocks(const u32* __restrict__ T, u32 lane32, const AesKey* const* k,
                                                        const u64* ctr, u64* lo, u64* hi) {
    aes_ctr_blocks_rk<NB>(T, lane32, AesRkSgpr{k}, ctr, lo, hi);
}

// A key schedule copied into VGPRs (44 per lane): a kernel that needs two
// schedules in one wave keeps the second here instead of spilling SGPRs.
struct AesKeyV {
    u32 rk[44];
};
__device__ __forceinline__ AesKeyV key_to_vgprs(const AesKey& k) {
    AesKeyV v;
#pragma unroll
    for (int i = 0; i < 44; ++i) asm volatile("v_mov_b32 %0, %1" : "=v"(v.rk[i]) : "s"(k.rk[i]));
    return v;
}

// AES-128 CTR block as aes_ctr_blocks<1>, round keys from VGPRs
__device__ __forceinline__ void aes_ctr_block_v(const u32* __restrict__ T, u32 lane32, const AesKeyV& k, u64 ctr,
                                                u64& lo, u64& hi) {
    const u8* Tb = reinterpret_cast<const u8*>(T);
    const u32 L0 = lane32 << 2, L1 = L0 | 0x80u;
#define ABY3G_TL(s, L, j) (*reinterpret_cast<const u32*>(Tb + aes_addr((s), (L), (j))))
    u32 s0 = (u32)ctr ^ k.rk[0], s1 = (u32)(ctr >> 32) ^ k.rk[1], s2 = k.rk[2], s3 = k.rk[3];
#pragma unroll
    for (int r = 1; r < 10; ++r) {
        const u32 t0 = xor3_v(ABY3G_TL(s0, L0, 0), ABY3G_TL(s1, L1, 1), k.rk[4 * r + 0]) ^
                       rotl(ABY3G_TL(s2, L0, 2) ^ ABY3G_TL(s3, L1, 3), 16);
        const u32 t1 = xor3_v(ABY3G_TL(s1, L0, 0), ABY3G_TL(s2, L1, 1), k.rk[4 * r + 1]) ^
                       rotl(ABY3G_TL(s3, L0, 2) ^ ABY3G_TL(s0, L1, 3), 16);
        const u32 t2 = xor3_v(ABY3G_TL(s2, L0, 0), ABY3G_TL(s3, L1, 1), k.rk[4 * r + 2]) ^
                       rotl(ABY3G_TL(s0, L0, 2) ^ ABY3G_TL(s1, L1, 3), 16);
        const u32 t3 = xor3_v(ABY3G_TL(s3, L0, 0), ABY3G_TL(s0, L1, 1), k.rk[4 * r + 3]) ^
                       rotl(ABY3G_TL(s1, L0, 2) ^ ABY3G_TL(s2, L1, 3), 16);
        s0 = t0, s1 = t1, s2 = t2, s3 = t3;
    }
    const u32 o0 = aes_sb4(ABY3G_TL(s0, L0, 0), ABY3G_TL(s1, L0, 1), ABY3G_TL(s2, L0, 2), ABY3G_TL(s3, L0, 3)) ^ k.rk[40];
    const u32 o1 = aes_sb4(ABY3G_TL(s1, L0, 0), ABY3G_TL(s2, L0, 1), ABY3G_TL(s3, L0, 2), ABY3G_TL(s0, L0, 3)) ^ k.rk[41];
    const u32 o2 = aes_sb4(ABY3G_TL(s2, L0, 0), ABY3G_TL(s3, L0, 1), ABY3G_TL(s0, L0, 2), ABY3G_TL(s1, L0, 3)) ^ k.rk[42];
    const u32 o3 = aes_sb4(ABY3G_TL(s3, L0, 0), ABY3G_TL(s0, L0, 1), ABY3G_TL(s1, L0, 2), ABY3G_TL(s2, L0, 3)) ^ k.rk[43];
#undef ABY3G_TL
    lo = (u64)o0 | ((u64)o1 << 32);
    hi = (u64)o2 | ((u64)o3 << 32);
}

__host__ __device__ __forceinline__ void aes_ctr_block(const u32* __restrict__ T, u32 lane32, const AesKey& k, u64 ctr,
                                              u64& lo, u64& hi) {
    const AesKey* kp = &k;
    aes_ctr_blocks<1>(T, lane32, &kp, &ctr, &lo, &hi);
}

// two independent blocks (e.g. the prev / next keys of a draw). Issued one
// after the other: with 16 waves per CU the interleaved form measured no
// faster and doubled the live registers.
__host__ __device__ __forceinline__ void aes_ctr_block2(const u32* __restrict__ T, u32 lane32, const AesKey& k1,
                                                        u64 c1, const AesKey& k2, u64 c2, u64& lo1, u64& hi1,
                                                        u64& lo2, u64& hi2) {
    aes_ctr_block(T, lane32, k1, c1, lo1, hi1);
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_sched_barrier(0);
#endif
    aes_ctr_block(T, lane32, k2, c2, lo2, hi2);
}

// Grid sizing for grid-stride AES kernels: every workgroup pays a 64 KiB LDS
// table fill and two fit a CU, so stop at 2 workgroups per CU (512) and let
// each one loop over several windows; never more workgroups than the work.
inline u32 aes_grid(u64 items, u32 block) {
    u64 g = (items + block - 1) / block;
    if (g > 512) g = 512;
    return (u32)(g ? g : 1);
}

inline hipStream_t S(aby3g_stream s) { return reinterpret_cast<hipStream_t>(s); }

// ------------------------------------------------------------ gate formulas --
// One gate of the bit-sliced engine on one 64-row word of both shares
// (Sh3BinaryEvaluator.cpp:700-1065). AND-type gates (AND, OR, NOR, na_And)
// produce only share 0, x0y0 ^ x0y1 ^ x1y0 (on the inverted inputs for NOR /
// na_And) ^ z; share 1 arrives from the previous party next round.
__device__ __forceinline__ bool gate_is_and(u32 t) {
    return t == ABY3G_GATE_AND || t == ABY3G_GATE_OR || t == ABY3G_GATE_NOR || t == ABY3G_GATE_NA_AND;
}
// share 0 of an AND-type gate before its mask (T: u64, or a vector of words)
template <class T>
__device__ __forceinline__ T gate_and_share(u32 type, T x0, T x1, T y0, T y1) {
    if (type == ABY3G_GATE_AND) return (x0 & y0) ^ (x0 & y1) ^ (x1 & y0);
    if (type == ABY3G_GATE_OR) return (x0 & y0) ^ (x0 & y1) ^ (x1 & y0) ^ x0 ^ y0;
    if (type == ABY3G_GATE_NOR) return (~x0 & ~y0) ^ (~x0 & ~y1) ^ (~x1 & ~y0);
    return (~x0 & y0) ^ (~x0 & y1) ^ (~x1 & y0);  // NA_AND
}
// both shares of a local gate (COPY, INV, XOR, NXOR)
template <class T>
__device__ __forceinline__ void gate_local(u32 type, T x0, T x1, T y0, T y1, T& o0, T& o1) {
    switch (type) {
        case ABY3G_GATE_COPY: o0 = x0; o1 = x1; break;
        case ABY3G_GATE_INV: o0 = ~x0; o1 = ~x1; break;
        case ABY3G_GATE_XOR: o0 = x0 ^ y0; o1 = x1 ^ y1; break;
        default: o0 = ~(x0 ^ y0); o1 = ~(x1 ^ y1); break;  // NXOR
    }
}

// ------------------------------------------------------ in-kernel hand-off --
// A message between co-located parties handed over inside the kernels
// (aby3g_handoff): the producer stores the payload write-through (sc1) --
// hs_store / hs_store2 -- and, once every storing wave has drained its
// stores, one lane stores flags[chunk] = seq (sc1); a consumer workgroup polls
// the flags of the chunks it reads (one lane, relaxed sc1 loads, s_sleep)
// and then reads the payload with sc1 loads (hs_load / hs_load2), which
// bypass its CU's L1 -- the R1 form of the guides' inter-workgroup recipe,
// no release or acquire fence. A wait gives up after kHandoffTimeoutTicks of
// the 100 MHz wall clock (a peer stream that cannot progress, e.g. two
// streams sharing a hardware queue), adds 1 to the device's timeout counter
// (pinned host memory, a system-scope atomic) and lets every wait enqueued
// before the host saw that count give up at once (each wait carries the
// count at its enqueue, `status0`): the results are then wrong, never hung,
// and the host raises an error (aby3g_handoff_status: callers compare the
// count before and after their run, so concurrent callers on one device
// cannot clear each other's timeout).
typedef __attribute__((address_space(1))) u64 gu64;
typedef __attribute__((address_space(1))) u32 gu32;
typedef u32 v4u32 __attribute__((ext_vector_type(4)));
constexpr u64 kHandoffTimeoutTicks = 500000000ull;  // 5 s (default; aby3g_set_handoff_timeout_us)
constexpr u64 kHandoffRows = ABY3G_HANDOFF_ROWS;

// the current device's hand-off timeout counter (pinned host memory, mapped)
u32* handoff_status_word();
// the wait limit kernels launched now use, in wall-clock ticks
u64 handoff_timeout_ticks();

// What a waiting kernel needs to give up: the counter, its value when the
// wait was enqueued, and the limit.
struct HsStatus {
    u32* word;
    u32 base;
    u64 limit;
};
inline HsStatus hs_status() {
    u32* w = handoff_status_word();
    return HsStatus{w, *(volatile u32*)w, handoff_timeout_ticks()};
}
// true once any wait on the device has timed out since this wait was enqueued
__device__ __forceinline__ bool hs_failed(const HsStatus& s) {
    return __hip_atomic_load(s.word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != s.base;
}
__device__ __forceinline__ void hs_fail(const HsStatus& s) {
    __hip_atomic_fetch_add(s.word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct HsWait {
    const u64* flags;  // null: nothing to wait for
    u64 seq;
    u64* ticks;        // optional: wall-clock ticks the first workgroup waited
    HsStatus status;
};
struct HsPost {
    u64* flags;  // null: nothing to publish
    u64 seq;
};
inline HsWait hs_wait_arg(const aby3g_handoff* h) {
    if (!h || !h->flags) return HsWait{nullptr, 0, nullptr, HsStatus{nullptr, 0, 0}};
    return HsWait{h->flags, h->seq, h->wait_ticks, hs_status()};
}
inline HsPost hs_post_arg(const aby3g_handoff* h) {
    if (!h || !h->flags) return HsPost{nullptr, 0};
    return HsPost{h->flags, h->seq};
}

// One lane waits until flags[c] >= seq for c in [c0, c1); the workgroup
// leaves together. Returns false after a timeout (here or elsewhere).
__device__ __forceinline__ bool hs_wait(const HsWait& w, u64 c0, u64 c1) {
    if (!w.flags) return true;
    __shared__ u32 ok;
    if (threadIdx.x == 0) {
        const u64 t0 = wall_clock64();
        u32 good = 1;
        for (u64 c = c0; c < c1 && good; ++c) {
            for (u32 spins = 0; __hip_atomic_load((const gu64*)w.flags + c, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT) < w.seq;) {
                __builtin_amdgcn_s_sleep(1);
                if ((++spins & 63) == 0) {
                    if (hs_failed(w.status)) {
                        good = 0;
                        break;
                    }
                    if (wall_clock64() - t0 > w.status.limit) {
                        hs_fail(w.status);
                        good = 0;
                        break;
                    }
                }
            }
        }
        if (w.ticks && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0)
            __hip_atomic_fetch_add((gu64*)w.ticks, wall_clock64() - t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = good;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the payload loads below the poll
    __syncthreads();
    return ok != 0;
}

// Every storing wave drains its write-through stores, then one lane
// publishes flags[c] = seq for c in [c0, c1). Call from every thread.
__device__ __forceinline__ void hs_post(const HsPost& p, u64 c0, u64 c1) {
    if (!p.flags) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        for (u64 c = c0; c < c1; ++c)
            __hip_atomic_store((gu64*)p.flags + c, p.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// write-through payload stores / L1-bypassing payload loads (8 and 16 bytes)
__device__ __forceinline__ void hs_store(u64* p, u64 v) {
    __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 hs_load(const u64* p) {
    return __hip_atomic_load((const gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16 B at byte offset `off` (< 4 GiB) of `base` (wave-uniform), sc1
__device__ __forceinline__ void hs_store2(void* base, u32 off, u64 a, u64 b) {
    const auto r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0xffffffffu, 0x00020000);
    const v4u32 v = {(u32)a, (u32)(a >> 32), (u32)b, (u32)(b >> 32)};
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}
__device__ __forceinline__ void hs_load2(const void* base, u32 off, u64& a, u64& b) {
    const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0xffffffffu, 0x00020000);
    const v4u32 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
    a = (u64)v.x | ((u64)v.y << 32);
    b = (u64)v.z | ((u64)v.w << 32);
}

// The calling thread's current device as last set through aby3g_set_device
// (queried from HIP once per thread otherwise). Threads that drive the
// library switch devices only through aby3g_set_device.
extern thread_local int t_device;
int current_device();

// device-to-device copy on the current device (runtime.hip)
void launch_copy(void* dst, const void* src, size_t bytes, hipStream_t s);

}  // namespace aby3g
