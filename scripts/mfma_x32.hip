// Microbenchmark: cycles per v_mfma_i32_16x16x32_i8 against
// v_mfma_i32_16x16x64_i8 (back-to-back, independent accumulators, one
// workgroup of 4 waves per CU): whether the share GEMM's four half-used
// 16x16x64 MFMAs per block and stage would cost less as 16x16x32.
// Build: hipcc --offload-arch=gfx950 -O3 mfma_x32.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256, 1) k64(int steps, int seed, int* out) {
    v4i a = v4i{seed, seed + 1, seed + 2, (int)threadIdx.x}, b = a + 7;
    v4i acc[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) acc[s] = v4i{0};
    for (int it = 0; it < steps; ++it)
#pragma unroll
        for (int s = 0; s < 8; ++s) acc[s] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[s], 0, 0, 0);
    int r = 0;
#pragma unroll
    for (int s = 0; s < 8; ++s) r += acc[s][0] + acc[s][1] + acc[s][2] + acc[s][3];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

__global__ void __launch_bounds__(256, 1) k32(int steps, int seed, int* out) {
    long a = ((long)seed << 32) | threadIdx.x, b = a * 3 + 1;
    v4i acc[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) acc[s] = v4i{0};
    for (int it = 0; it < steps; ++it)
#pragma unroll
        for (int s = 0; s < 8; ++s) acc[s] = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, acc[s], 0, 0, 0);
    int r = 0;
#pragma unroll
    for (int s = 0; s < 8; ++s) r += acc[s][0] + acc[s][1] + acc[s][2] + acc[s][3];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main() {
    const int blocks = 256, steps = 20000;
    int* out;
    hipMalloc(&out, blocks * 256 * sizeof(int));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep)
        for (int form = 0; form < 2; ++form) {
            hipEventRecord(e0);
            if (form == 0)
                k64<<<blocks, 256>>>(steps, rep + 3, out);
            else
                k32<<<blocks, 256>>>(steps, rep + 3, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            // one wave per SIMD: MFMAs per SIMD = steps * 8
            const double ns_per = ms * 1e6 / (steps * 8.0);
            printf("%s: %.3f ms, %.2f ns per MFMA per SIMD (%.1f cycles at 2.4 GHz)\n",
                   form == 0 ? "16x16x64_i8" : "16x16x32_i8", ms, ns_per, ns_per * 2.4);
        }
    hipFree(out);
    return 0;
}
