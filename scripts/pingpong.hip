// Microbenchmark: cross-stream hand-off latency on one GPU, the per-level /
// per-round cost of the co-located parties' protocol messages. Two streams
// alternate tiny kernels, each waiting for the other's previous kernel:
//   (a) hipEventRecord + hipStreamWaitEvent   (what Channel uses)
//   (b) hipStreamWriteValue64 + hipStreamWaitValue64 on a device word
//   (c) the same chain on ONE stream (no hand-off) for reference
// Build: hipcc --offload-arch=gfx950 -O3 pingpong.hip -o pingpong
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

__global__ void k_tick(unsigned long long* p) {
    if (threadIdx.x == 0) *p += 1;
}

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            printf("%s: %s\n", #x, hipGetErrorString(e));                      \
            return 1;                                                          \
        }                                                                      \
    } while (0)

int main(int argc, char** argv) {
    const int only = argc > 1 ? atoi(argv[1]) : -1;
    hipStream_t s[2];
    for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    unsigned long long *d, *sig;
    CK(hipMalloc(&d, 64));
    CK(hipMemset(d, 0, 64));
    CK(hipExtMallocWithFlags((void**)&sig, 8, hipMallocSignalMemory));
    CK(hipMemset(sig, 0, 8));
    const int N = 2000;
    hipEvent_t ev[2];
    for (auto& evx : ev) CK(hipEventCreateWithFlags(&evx, hipEventDisableTiming));
    for (int mode = 0; mode < 4; ++mode) {
        if (only >= 0 && mode != only) continue;
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipDeviceSynchronize());
            auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < N; ++i) {
                const int a = i & 1, b = a ^ 1;
                if (mode == 2) {
                    k_tick<<<1, 64, 0, s[0]>>>(d);
                    continue;
                }
                if (mode == 3) {
                    if (i) CK(hipStreamWaitValue64(s[a], sig, (uint64_t)i, hipStreamWaitValueGte, ~0ull));
                    k_tick<<<1, 64, 0, s[a]>>>(d);
                    CK(hipStreamWriteValue64(s[a], sig, (uint64_t)(i + 1), 0));
                    continue;
                }
                if (mode == 0) {
                    if (i) CK(hipStreamWaitEvent(s[a], ev[b], 0));
                    k_tick<<<1, 64, 0, s[a]>>>(d);
                    CK(hipEventRecord(ev[a], s[a]));
                } else {
                    if (i) CK(hipStreamWaitValue64(s[a], d + 1, (uint64_t)i, hipStreamWaitValueGte, ~0ull));
                    k_tick<<<1, 64, 0, s[a]>>>(d);
                    CK(hipStreamWriteValue64(s[a], d + 1, (uint64_t)(i + 1), 0));
                }
            }
            CK(hipDeviceSynchronize());
            auto t1 = std::chrono::steady_clock::now();
            if (rep)
                printf("%s: %.2f us per hand-off\n",
                       mode == 0   ? "event record/wait"
                       : mode == 1 ? "write/wait value (device word)"
                       : mode == 2 ? "one stream, no hand-off"
                                   : "write/wait value (signal memory)",
                       std::chrono::duration<double, std::micro>(t1 - t0).count() / N);
            CK(hipMemset(d, 0, 64));
            CK(hipMemset(sig, 0, 8));
        }
    }
    return 0;
}
