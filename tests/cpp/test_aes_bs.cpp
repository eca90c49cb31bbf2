// The bitsliced AES (aby3_amd/csrc/aes_bs.h, host compile of the device
// code) against the oracle's textbook AES: 32-block counter batches for
// several keys and counter bases, and the 32 x 32 bit transpose. CPU only.
#include <cstdio>
#include <cstring>
#include <random>
#include "../../aby3_amd/csrc/aes_bs.h"
#include "orc_aes.h"

using namespace aby3g::bs;

static int failures = 0;
#define CHECK(c, ...)                     \
    do {                                  \
        if (!(c)) {                       \
            std::printf("FAIL " __VA_ARGS__); \
            std::printf("\n");            \
            ++failures;                   \
        }                                 \
    } while (0)

int main() {
    std::mt19937_64 rng(7);
    // transpose32: bit t of a[j] <- bit j of a[t]
    {
        u32 a[32], b[32];
        for (auto& v : a) v = (u32)rng();
        std::memcpy(b, a, sizeof(a));
        transpose32(b);
        bool ok = true;
        for (int t = 0; t < 32; ++t)
            for (int j = 0; j < 32; ++j) ok = ok && (((b[j] >> t) & 1) == ((a[t] >> j) & 1));
        CHECK(ok, "transpose32");
    }
    const uint64_t bases[] = {0, 2048, 1ull << 40, 0xFFFFFFFFFFFFF800ull};
    for (int kk = 0; kk < 4; ++kk) {
        uint8_t key[16];
        for (auto& b : key) b = (uint8_t)rng();
        if (kk == 0) std::memset(key, 0, 16);
        orc::AesRef ref;
        ref.setKey(key);
        u32 rk[44];
        for (int r = 0; r < 11; ++r)
            for (int c = 0; c < 4; ++c) std::memcpy(&rk[4 * r + c], &ref.rk[r][4 * c], 4);
        for (uint64_t base : bases)
            for (u32 lane : {0u, 1u, 37u, 63u}) {
                u32 st[128];
                load_counters(st, base, lane);
                encrypt(st, rk);
                planes_to_blocks(st);
                for (int j = 0; j < 32; ++j) {
                    const uint64_t ctr = base + lane + 64ull * j;
                    orc::Block e = ref.encrypt(orc::Block{ctr, 0});
                    uint64_t lo = (uint64_t)st[4 * j] | ((uint64_t)st[4 * j + 1] << 32);
                    uint64_t hi = (uint64_t)st[4 * j + 2] | ((uint64_t)st[4 * j + 3] << 32);
                    CHECK(lo == e.lo && hi == e.hi, "key %d base %llx lane %u block %d", kk,
                          (unsigned long long)base, lane, j);
                }
            }
    }
    if (failures)
        std::printf("FAIL aes_bs (%d)\n", failures);
    else
        std::printf("PASS aes_bs\n");
    return failures ? 1 : 0;
}
