// Microbenchmark: sustained v_mfma_i32_32x32x32_i8 rate on random vs zero
// operands (fragments in registers, 36 MFMAs per step into 8 accumulator
// planes exactly like k_share_gemm's inner loop). Gives the chip's int8 MFMA
// ceiling under its power/clock behaviour, the reference for the share GEMM's
// roofline fraction.  Build: hipcc --offload-arch=gfx950 -O3 mfma_peak.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void __launch_bounds__(512, 1) k_peak(const v4i* frag, int steps, int* out) {
    const int lane = threadIdx.x;
    v4i a[8], b[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) {
        a[p] = frag[(blockIdx.x * 16 + p) * 512 + lane];
        b[p] = frag[(blockIdx.x * 16 + 8 + p) * 512 + lane];
    }
    v16i acc[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) acc[s] = v16i{0};
    for (int it = 0; it < steps; ++it) {
#pragma unroll
        for (int p = 0; p < 8; ++p)
#pragma unroll
            for (int q = 0; q + p < 8; ++q)
                acc[p + q] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[p], b[q], acc[p + q], 0, 0, 0);
    }
    int r = 0;
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int j = 0; j < 16; ++j) r += acc[s][j];
    out[blockIdx.x * 512 + lane] = r;
}

// the same work in v_mfma_i32_16x16x64_i8 form: a 32x32 wave tile as 2x2
// 16x16 tiles, 4 x 36 MFMAs per step
__global__ void __launch_bounds__(512, 1) k_peak16(const v4i* frag, int steps, int* out) {
    const int lane = threadIdx.x;
    v4i a[8], b[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) {
        a[p] = frag[(blockIdx.x * 16 + p) * 512 + lane];
        b[p] = frag[(blockIdx.x * 16 + 8 + p) * 512 + lane];
    }
    v4i acc[8][4];
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[s][t] = v4i{0};
    for (int it = 0; it < steps; ++it) {
#pragma unroll
        for (int p = 0; p < 8; ++p)
#pragma unroll
            for (int q = 0; q + p < 8; ++q)
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    acc[p + q][t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[p], b[q], acc[p + q][t], 0, 0, 0);
    }
    int r = 0;
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int j = 0; j < 4; ++j) r += acc[s][t][j];
    out[blockIdx.x * 512 + lane] = r;
}

int main() {
    const int blocks = 256 * 4, steps = 2000;
    const size_t nfrag = (size_t)blocks * 16 * 512;
    std::vector<v4i> h(nfrag);
    for (int mode = 0; mode < 2; ++mode) {
        srand(1);
        for (auto& x : h)
            for (int j = 0; j < 4; ++j) x[j] = mode ? rand() : 0;
        v4i* d;
        int* o;
        hipMalloc(&d, nfrag * sizeof(v4i));
        hipMalloc(&o, blocks * 512 * sizeof(int));
        hipMemcpy(d, h.data(), nfrag * sizeof(v4i), hipMemcpyHostToDevice);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        for (int form = 0; form < 2; ++form) {
            auto run = [&] {
                if (form) k_peak16<<<blocks, 512>>>(d, steps, o);
                else k_peak<<<blocks, 512>>>(d, steps, o);
            };
            for (int w = 0; w < 3; ++w) run();
            hipEventRecord(e0);
            const int reps = 5;
            for (int w = 0; w < reps; ++w) run();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double ops = (double)reps * blocks * 8 * steps * 36 * 32.0 * 32 * 32 * 2;
            printf("%s %s operands: %.0f int8 TOP/s (%.1f %% of 5033)\n", form ? "16x16x64" : "32x32x32",
                   mode ? "random" : "zero", ops / (ms * 1e-3) / 1e12, 100 * ops / (ms * 1e-3) / 1e12 / 5033.0);
        }
        hipFree(d);
        hipFree(o);
    }
    return 0;
}
