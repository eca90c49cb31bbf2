// Element-wise helpers of the protocols around the hot kernels: share sums
// and differences, fixed-point constants, the trunc finalize, bitwise ops on
// binary shares and the gather/scatter of the merge network.
#include "common.h"

namespace aby3g {

namespace {

constexpr u32 kB = 256;

inline u32 ew_grid(u64 n) {
    u64 g = (n + kB - 1) / kB;
    if (g > 8192) g = 8192;
    return (u32)(g ? g : 1);
}

#define GRID_STRIDE(i, n) for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += (u64)gridDim.x * blockDim.x)

__global__ void k_lincomb(u64 n, u64 ca, const i64* __restrict__ a, u64 cb, const i64* __restrict__ b, u64 c,
                          i64* __restrict__ out) {
    GRID_STRIDE(i, n) {
        u64 v = ca * (u64)a[i] + c;
        if (b) v += cb * (u64)b[i];
        out[i] = (i64)v;
    }
}

// Sh3Evaluator.cpp:712-718: C[party] += (za + zb + zo) >> d. Two elements a
// thread (16-byte accesses) when every pointer is 16-byte aligned.
__global__ void k_trunc_finalize(u64 n, const i64* __restrict__ za, const i64* __restrict__ zb,
                                 const i64* __restrict__ zo, u32 d, i64* __restrict__ c) {
    GRID_STRIDE(i, n) {
        const i64 s = (i64)((u64)za[i] + (u64)zb[i] + (u64)zo[i]);
        c[i] = (i64)((u64)c[i] + (u64)(s >> d));
    }
}
typedef i64 i64x2 __attribute__((ext_vector_type(2)));
__global__ void k_trunc_finalize2(u64 n2, const i64x2* __restrict__ za, const i64x2* __restrict__ zb,
                                  const i64x2* __restrict__ zo, u32 d, i64x2* __restrict__ c) {
    GRID_STRIDE(i, n2) {
        const i64x2 a = za[i], b = zb[i], o = zo[i];
        i64x2 v = c[i];
        const i64 s0 = (i64)((u64)a.x + (u64)b.x + (u64)o.x), s1 = (i64)((u64)a.y + (u64)b.y + (u64)o.y);
        v.x = (i64)((u64)v.x + (u64)(s0 >> d));
        v.y = (i64)((u64)v.y + (u64)(s1 >> d));
        c[i] = v;
    }
}

__global__ void k_bitop(int op, u64 n, const u64* __restrict__ a, const u64* __restrict__ b, u64* __restrict__ out) {
    GRID_STRIDE(i, n) {
        u64 v;
        switch (op) {
            case 0: v = a[i] ^ b[i]; break;
            case 1: v = a[i] & b[i]; break;
            case 2: v = ~a[i]; break;
            case 3: v = 0 - (a[i] & 1); break;
            default: v = a[i]; break;
        }
        out[i] = v;
    }
}

// one row per (y, x-chunk); both shares
__global__ void k_gather_rows(const i64* __restrict__ src, u64 rows, u64 cols, const u32* __restrict__ idx, u64 n,
                              i64* __restrict__ dst) {
    const u64 total = 2 * n * cols;
    GRID_STRIDE(t, total) {
        const u64 s = t / (n * cols), rem = t % (n * cols), i = rem / cols, c = rem % cols;
        dst[t] = src[s * rows * cols + (u64)idx[i] * cols + c];
    }
}

// out[i][w] = a[g][w] ^ b[g][w] ^ c[g][w] ^ mask[w], g = idx ? idx[i] : i
// (every operand optional)
__global__ void k_xor_gather_units(u64 units, u64 unit, const u32* __restrict__ idx, const u64* __restrict__ a,
                                   const u64* __restrict__ b, const u64* __restrict__ c, const u64* __restrict__ mask,
                                   u64* __restrict__ out) {
    GRID_STRIDE(t, units * unit) {
        const u64 i = t / unit, w = t % unit;
        const u64 g = (idx ? (u64)idx[i] : i) * unit + w;
        u64 v = mask ? mask[w] : 0;
        if (a) v ^= a[g];
        if (b) v ^= b[g];
        if (c) v ^= c[g];
        out[t] = v;
    }
}

// 64 x 64 tile transpose through LDS (padded rows: conflict-free)
__global__ void __launch_bounds__(256) k_transpose(const i64* __restrict__ src, u64 rows, u64 cols,
                                                   i64* __restrict__ dst) {
    __shared__ i64 tile[64][65];
    const u64 s = blockIdx.z;
    const u64 r0 = (u64)blockIdx.y * 64, c0 = (u64)blockIdx.x * 64;
    const i64* S = src + s * rows * cols;
    i64* Dd = dst + s * rows * cols;
    for (u32 k = threadIdx.x; k < 64 * 64; k += blockDim.x) {
        const u32 r = k / 64, c = k % 64;
        if (r0 + r < rows && c0 + c < cols) tile[r][c] = S[(r0 + r) * cols + c0 + c];
    }
    __syncthreads();
    for (u32 k = threadIdx.x; k < 64 * 64; k += blockDim.x) {
        const u32 c = k / 64, r = k % 64;  // output row = input column
        if (r0 + r < rows && c0 + c < cols) Dd[(c0 + c) * rows + r0 + r] = tile[r][c];
    }
}

__global__ void k_gather(u64 n, const u32* __restrict__ idx, const u64* __restrict__ src, u64* __restrict__ dst) {
    GRID_STRIDE(i, n) dst[i] = src[idx[i]];
}
__global__ void k_scatter(u64 n, const u32* __restrict__ idx, const u64* __restrict__ src, u64* __restrict__ dst) {
    GRID_STRIDE(i, n) dst[idx[i]] = src[i];
}

}  // namespace

}  // namespace aby3g

using namespace aby3g;

extern "C" {

int aby3g_i64_lincomb(uint64_t n, int64_t ca, const int64_t* a, int64_t cb, const int64_t* b, int64_t c, int64_t* out,
                      aby3g_stream stream) {
    return guarded([&] {
        if (!n) return;
        launch(PROBE_OTHER, k_lincomb, dim3(ew_grid(n)), dim3(kB), 0, S(stream), n, (u64)ca, a, (u64)cb, b, (u64)c,
               out);
    });
}

int aby3g_trunc_finalize(int party, const int64_t* z_a, const int64_t* z_b, const int64_t* z_own, unsigned d,
                         int64_t* C, uint64_t n, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(party >= 0 && party <= 2, "party out of range");
        ABY3G_REQUIRE(d < 64, "shift too large");
        if (party == 2 || !n) return;  // only P0 and P1 finalize (Sh3Evaluator.cpp:692)
        i64* c = C + (u64)party * n;
        auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
        if (n % 2 == 0 && a16(z_a) && a16(z_b) && a16(z_own) && a16(c))
            launch(PROBE_EPILOGUE, k_trunc_finalize2, dim3(ew_grid(n / 2)), dim3(kB), 0, S(stream), n / 2,
                   (const i64x2*)z_a, (const i64x2*)z_b, (const i64x2*)z_own, (u32)d, (i64x2*)c);
        else
            launch(PROBE_EPILOGUE, k_trunc_finalize, dim3(ew_grid(n)), dim3(kB), 0, S(stream), n, z_a, z_b, z_own,
                   (u32)d, c);
    });
}

int aby3g_u64_bitop(int op, uint64_t n, const uint64_t* a, const uint64_t* b, uint64_t* out, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(op >= 0 && op <= 4, "bad op");
        ABY3G_REQUIRE(op >= 2 || b != nullptr, "binary op needs b");
        if (!n) return;
        launch(PROBE_OTHER, k_bitop, dim3(ew_grid(n)), dim3(kB), 0, S(stream), op, n, a, b, out);
    });
}

int aby3g_i64_gather_rows(const int64_t* src, uint64_t rows, uint64_t cols, const uint32_t* idx, uint64_t n,
                          int64_t* dst, aby3g_stream stream) {
    return guarded([&] {
        if (!n || !cols) return;
        launch(PROBE_OTHER, k_gather_rows, dim3(ew_grid(2 * n * cols)), dim3(kB), 0, S(stream), src, rows, cols, idx,
               n, dst);
    });
}

int aby3g_u64_xor_gather_units(uint64_t units, uint64_t unit, const uint32_t* idx, const uint64_t* a,
                               const uint64_t* b, const uint64_t* c, const uint64_t* mask, uint64_t* out,
                               aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(out != nullptr, "null output");
        ABY3G_REQUIRE(!idx || (out != a && out != b && out != c), "a gathering step cannot run in place");
        if (!units || !unit) return;
        launch(PROBE_OTHER, k_xor_gather_units, dim3(ew_grid(units * unit)), dim3(kB), 0, S(stream), units, unit, idx,
               a, b, c, mask, out);
    });
}

int aby3g_i64_transpose(const int64_t* src, uint64_t rows, uint64_t cols, int64_t* dst, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(src != dst, "in-place transpose is not supported");
        if (!rows || !cols) return;
        dim3 grid((u32)((cols + 63) / 64), (u32)((rows + 63) / 64), 2);
        launch(PROBE_OTHER, k_transpose, grid, dim3(256), 0, S(stream), src, rows, cols, dst);
    });
}

int aby3g_u64_gather(uint64_t n, const uint32_t* idx, const uint64_t* src, uint64_t* dst, aby3g_stream stream) {
    return guarded([&] {
        if (!n) return;
        launch(PROBE_OTHER, k_gather, dim3(ew_grid(n)), dim3(kB), 0, S(stream), n, idx, src, dst);
    });
}

int aby3g_u64_scatter(uint64_t n, const uint32_t* idx, const uint64_t* src, uint64_t* dst, aby3g_stream stream) {
    return guarded([&] {
        if (!n) return;
        launch(PROBE_OTHER, k_scatter, dim3(ew_grid(n)), dim3(kB), 0, S(stream), n, idx, src, dst);
    });
}

}  // extern "C"
