// Microbenchmark: in-kernel hand-off latency between two workgroups of one
// launch -- the floor under the fused LR iteration's per-level round trip.
// Workgroups a = 0 and b (b = 1: next XCD under round-robin dispatch; b = 8:
// same XCD as 0) bounce a counter through agent-scope relaxed 64-bit stores
// and polling loads (hs_store / hs_load of common.h), N round trips; the
// time per round trip is printed for polls with and without s_sleep.
// Build: hipcc --offload-arch=gfx950 -O3 ingrid_pingpong.hip -o ingrid_pingpong
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned long long u64;
typedef unsigned int u32;
typedef __attribute__((address_space(1))) u64 gu64;

__device__ __forceinline__ void st(u64* p, u64 v) {
    __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 ld(const u64* p) {
    return __hip_atomic_load((const gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool kSleep>
__global__ void k_pingpong(u64* box, u32 b, u32 n, u64* out) {
    const u32 me = blockIdx.x;
    if ((me != 0 && me != b) || threadIdx.x != 0) return;
    u64* mine = box + (me == 0 ? 0 : 16);
    const u64* other = box + (me == 0 ? 16 : 0);
    const u64 t0 = wall_clock64();
    for (u64 i = 1; i <= n; ++i) {
        if (me == 0) {
            st(mine, i);
            for (u32 s = 0; ld(other) < i; ++s) {
                if (kSleep) __builtin_amdgcn_s_sleep(1);
                if (s > (1u << 26)) return;  // bounded
            }
        } else {
            for (u32 s = 0; ld(other) < i; ++s) {
                if (kSleep) __builtin_amdgcn_s_sleep(1);
                if (s > (1u << 26)) return;
            }
            st(mine, i);
        }
    }
    if (me == 0) out[0] = wall_clock64() - t0;
}

int main() {
    u64 *box, *out;
    if (hipMalloc(&box, 4096) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    const u32 n = 20000;
    for (int sleep = 0; sleep < 2; ++sleep)
        for (u32 b : {1u, 8u, 2u, 16u}) {
            for (int rep = 0; rep < 2; ++rep) {
                hipMemset(box, 0, 4096);
                hipMemset(out, 0, 64);
                if (sleep)
                    hipLaunchKernelGGL(k_pingpong<true>, dim3(b + 1), dim3(64), 0, 0, box, b, n, out);
                else
                    hipLaunchKernelGGL(k_pingpong<false>, dim3(b + 1), dim3(64), 0, 0, box, b, n, out);
                if (hipDeviceSynchronize() != hipSuccess) return 2;
                u64 t = 0;
                hipMemcpy(&t, out, 8, hipMemcpyDeviceToHost);
                if (rep) std::printf("partner block %2u, %s: %.3f us per round trip\n", b, sleep ? "s_sleep 1" : "busy poll",
                                     t * 0.01 / n);
            }
        }
    return 0;
}
