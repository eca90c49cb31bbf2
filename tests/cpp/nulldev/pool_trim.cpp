// The stream-ordered pool gives its cache back (with the
// out-of-memory retry gone, nothing trimmed the cache). On the null device:
// (1) a Gpu's pool filled with blocks of many size classes is emptied by
// trim() and allocates again; (2) a session whose parties' caches pass
// ABY3_POOL_TRIM_MB (0 here) trims them between runs -- after the run, so
// the run itself still makes no device-wide wait -- and keeps running.
// Built with -fsanitize=address by tests/test_host_asan.py.
#include <aby3.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "Device.h"

extern "C" unsigned long nulldev_blocking_calls();

int main() {
    {
        aby3::Gpu g(0);
        {
            std::vector<aby3::DeviceBuffer> bufs;
            for (size_t b : {17ul, 4096ul, 100000ul, 1ul << 20, 3ul << 20, 5000ul, 1ul << 22})
                for (int k = 0; k < 3; ++k) bufs.emplace_back(g, b + k);
        }
        if (!g.cachedBytes()) {
            std::printf("FAIL nothing cached after the buffers were released\n");
            return 1;
        }
        const unsigned long b0 = nulldev_blocking_calls();
        g.trim();
        if (g.cachedBytes() || nulldev_blocking_calls() == b0) {
            std::printf("FAIL trim left %zu bytes cached\n", g.cachedBytes());
            return 1;
        }
        aby3::DeviceBuffer again(g, 3ul << 20);
        if (!again.data()) {
            std::printf("FAIL no allocation after trim\n");
            return 1;
        }
    }
    setenv("ABY3_POOL_TRIM_MB", "0", 1);
    const int dev[3] = {0, 0, 0};
    const uint64_t p[] = {64, 48, 80, 16, 1};
    aby3h_session* s = aby3h_session_create(ABY3H_JOB_MUL_TRUNC, p, 5, dev, 0);
    if (!s) {
        std::printf("FAIL create: %s\n", aby3h_last_error());
        return 1;
    }
    unsigned long trims = 0;
    for (int r = 0; r < 3; ++r) {
        const unsigned long b0 = nulldev_blocking_calls();
        if (aby3h_session_run(s, 2)) {
            std::printf("FAIL run %d: %s\n", r, aby3h_last_error());
            return 1;
        }
        trims += nulldev_blocking_calls() - b0;
    }
    if (aby3h_session_check(s) == 2) {
        std::printf("FAIL check: %s\n", aby3h_last_error());
        return 1;
    }
    aby3h_session_destroy(s);
    if (!trims) {
        std::printf("FAIL the session never trimmed its pools\n");
        return 1;
    }
    std::printf("pool_trim: ok (%lu frees between runs)\n", trims);
    return 0;
}
