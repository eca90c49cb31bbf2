// Shared definitions of the gfx950 engine: error plumbing, the launch probe
// and the device AES-128 used by every randomness kernel.
#pragma once
#include <hip/hip_runtime.h>
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

template <class F>
int guarded(F&& f) {
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
// Device copy of T0[x] = 2S | S<<8 | S<<16 | 3S<<24 for the current device
// (computed on the host from the S-box definition, uploaded once).
const u32* aes_table();

// The LDS copy of T0 is replicated 32 times with entry x of copy c at word
// 32*x + c, and lane l reads copy (l & 31): ds_read_b32 serves a wave in two
// 32-lane halves over 32 banks, so every lane hits its own bank and the
// random S-box lookups are conflict-free. 32 KiB per workgroup.
constexpr int kAesLdsWords = 256 * 32;

__device__ __forceinline__ void aes_fill_lds(u32* lds, const u32* __restrict__ T0g) {
    for (int i = threadIdx.x; i < kAesLdsWords; i += blockDim.x) lds[i] = T0g[i >> 5];
    __syncthreads();
}

__host__ __device__ __forceinline__ u32 rotl(u32 x, int r) { return __builtin_rotateleft32(x, r); }

struct AesState {
    u32 s0, s1, s2, s3;
};

// AES-128 of the counter block LE64(ctr) || 0^8 under `k`, T-table form.
// Column c of the state is the LE word of bytes 4c..4c+3; after ShiftRows,
// row r of column c comes from column c+r, and MixColumns row weights of
// input row r are T0 rotated left by 8r bits.
__host__ __device__ __forceinline__ void aes_ctr_block(const u32* __restrict__ T, u32 lane32, const AesKey& k, u64 ctr,
                                              u64& lo, u64& hi) {
    u32 s0 = (u32)ctr ^ k.rk[0];
    u32 s1 = (u32)(ctr >> 32) ^ k.rk[1];
    u32 s2 = k.rk[2];
    u32 s3 = k.rk[3];
#define T0L(x) T[((x) << 5) | lane32]
#pragma unroll
    for (int r = 1; r < 10; ++r) {
        u32 t0 = T0L(s0 & 0xff) ^ rotl(T0L((s1 >> 8) & 0xff), 8) ^ rotl(T0L((s2 >> 16) & 0xff), 16) ^
                 rotl(T0L(s3 >> 24), 24) ^ k.rk[4 * r + 0];
        u32 t1 = T0L(s1 & 0xff) ^ rotl(T0L((s2 >> 8) & 0xff), 8) ^ rotl(T0L((s3 >> 16) & 0xff), 16) ^
                 rotl(T0L(s0 >> 24), 24) ^ k.rk[4 * r + 1];
        u32 t2 = T0L(s2 & 0xff) ^ rotl(T0L((s3 >> 8) & 0xff), 8) ^ rotl(T0L((s0 >> 16) & 0xff), 16) ^
                 rotl(T0L(s1 >> 24), 24) ^ k.rk[4 * r + 2];
        u32 t3 = T0L(s3 & 0xff) ^ rotl(T0L((s0 >> 8) & 0xff), 8) ^ rotl(T0L((s1 >> 16) & 0xff), 16) ^
                 rotl(T0L(s2 >> 24), 24) ^ k.rk[4 * r + 3];
        s0 = t0;
        s1 = t1;
        s2 = t2;
        s3 = t3;
    }
    // last round: SubBytes + ShiftRows; S[x] = byte 1 of T0[x]
#define SB(x) ((T0L(x) >> 8) & 0xff)
    u32 o0 = (SB(s0 & 0xff) | (SB((s1 >> 8) & 0xff) << 8) | (SB((s2 >> 16) & 0xff) << 16) | (SB(s3 >> 24) << 24)) ^
             k.rk[40];
    u32 o1 = (SB(s1 & 0xff) | (SB((s2 >> 8) & 0xff) << 8) | (SB((s3 >> 16) & 0xff) << 16) | (SB(s0 >> 24) << 24)) ^
             k.rk[41];
    u32 o2 = (SB(s2 & 0xff) | (SB((s3 >> 8) & 0xff) << 8) | (SB((s0 >> 16) & 0xff) << 16) | (SB(s1 >> 24) << 24)) ^
             k.rk[42];
    u32 o3 = (SB(s3 & 0xff) | (SB((s0 >> 8) & 0xff) << 8) | (SB((s1 >> 16) & 0xff) << 16) | (SB(s2 >> 24) << 24)) ^
             k.rk[43];
#undef SB
#undef T0L
    lo = (u64)o0 | ((u64)o1 << 32);
    hi = (u64)o2 | ((u64)o3 << 32);
}

// Grid sizing for grid-stride AES kernels: every workgroup pays a 32 KiB LDS
// table fill, so stop at 4 workgroups per CU and let each one loop over
// several windows; never more workgroups than the work.
inline u32 aes_grid(u64 items, u32 block) {
    u64 g = (items + block - 1) / block;
    if (g > 1024) g = 1024;
    return (u32)(g ? g : 1);
}

inline hipStream_t S(aby3g_stream s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace aby3g
