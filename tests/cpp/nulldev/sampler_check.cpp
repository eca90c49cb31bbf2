// DeviceBatchSampler (aby3ML.h) against BatchSampler, on the null device
// (device memory is host memory there, so the batches the device pointers
// name can be read directly): the same mini-batches, in the same order,
// across reshuffles and batches that straddle them, with the reshuffle on the
// sampler's host thread. Built with -fsanitize=address / thread by
// tests/test_host_asan.py.
#include <cstdio>
#include <vector>
#include "aby3ML.h"

using namespace aby3;

static bool same(u64 n, u64 B, u64 iters) {
    Gpu g(0);
    g.bind();
    DeviceBatchSampler dev(g, n, B);
    BatchSampler host(n);
    std::vector<u64> b(B);
    for (u64 t = 0; t < iters; ++t) {
        const u32* p = dev.next();
        host.next(b);
        for (u64 i = 0; i < B; ++i)
            if (p[i] != (u32)b[i]) {
                std::printf("FAIL n %llu B %llu: iteration %llu row %llu: %u != %llu\n", (unsigned long long)n,
                            (unsigned long long)B, (unsigned long long)t, (unsigned long long)i, p[i],
                            (unsigned long long)b[i]);
                return false;
            }
    }
    const u64 want = (iters * B + n - 1) / n + (iters * B % n == 0 ? 1 : 0);  // the first getSubset reshuffles too
    if (dev.reshuffles() != want) {
        std::printf("FAIL n %llu B %llu: %llu reshuffles, expected %llu\n", (unsigned long long)n,
                    (unsigned long long)B, (unsigned long long)dev.reshuffles(), (unsigned long long)want);
        return false;
    }
    return true;
}

int main() {
    // batches inside one pool, straddling reshuffles, B dividing n, B == n
    const u64 cases[][3] = {{1000, 64, 100}, {1000, 7, 500}, {1024, 256, 20}, {50, 50, 6}, {50, 49, 7}, {1, 1, 5}};
    for (const auto& c : cases)
        if (!same(c[0], c[1], c[2])) return 1;
    std::printf("sampler_check: ok\n");
    return 0;
}
