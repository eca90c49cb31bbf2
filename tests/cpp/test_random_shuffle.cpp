// CPU-only: the reference draws its mini-batches (getSubset, Regression.h:24-40)
// and the shuffle's permutations (get_permutation, BoolBasic.cpp:925-934) with
// std::random_shuffle(first, last, prng). The product (aby3::BatchSampler,
// aby3::get_permutation) and the oracle (orc::BatchSampler,
// orc::shufflePermutation) restate that call as an explicit loop. Here the
// loop is checked against the standard library's own std::random_shuffle
// (libstdc++, the reference's toolchain), driven by the same PRNG stream
// through a functor with cryptoTools' PRNG::operator()(R mod) semantics:
// get<make_unsigned<R>>() % mod. (cryptoTools is not vendored in the
// reference; that functor's semantics is the one piece this cannot pin.)
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>
#include "Shuffle.h"
#include "aby3ML.h"
#include "orc_core.h"

#pragma GCC diagnostic ignored "-Wdeprecated-declarations"

using namespace aby3;

static int failures = 0;
static void check(bool c, const std::string& what) {
    if (!c) throw std::runtime_error("check failed: " + what);
}
static void test(const char* name, void (*f)()) {
    try {
        f();
        std::printf("PASS %s\n", name);
    } catch (const std::exception& e) {
        ++failures;
        std::printf("FAIL %s: %s\n", name, e.what());
    }
}

// the PRNG as a random_shuffle generator, cryptoTools-style
struct PrngFunctor {
    HostPrng* p;
    template <class R>
    R operator()(R mod) {
        return (R)(p->get<typename std::make_unsigned<R>::type>() % (typename std::make_unsigned<R>::type)mod);
    }
};

// getSubset with the library call, as the reference writes it
static void getSubsetStd(std::vector<u64>& dest, std::vector<u64>& pool, std::vector<u64>::iterator& it,
                         PrngFunctor& prng) {
    auto d = dest.begin();
    while (d != dest.end()) {
        auto step = std::min<u64>(pool.end() - it, dest.end() - d);
        std::copy(it, it + step, d);
        it += step;
        d += step;
        if (it == pool.end()) {
            std::random_shuffle(pool.begin(), pool.end(), prng);
            it = pool.begin();
        }
    }
}

static void batches_match_std() {
    // pool sizes with and without a batch boundary on the pool's end, several
    // reshuffles each
    const u64 cases[][2] = {{1000, 256}, {777, 256}, {64, 64}, {5, 3}, {2, 1}};
    for (const auto& c : cases) {
        const u64 n = c[0], B = c[1];
        std::vector<u64> pool(n);
        std::iota(pool.begin(), pool.end(), 0);
        auto it = pool.end();  // the first call reshuffles (main-logistic's iterator starts at end)
        HostPrng hp(toBlock(234543234));
        PrngFunctor f{&hp};
        BatchSampler prod(n);
        orc::BatchSampler orcS(n);
        for (int b = 0; b < 12; ++b) {
            std::vector<u64> a(B), p(B), o(B);
            getSubsetStd(a, pool, it, f);
            prod.next(p);
            orcS.next(o);
            check(a == p, "product batch " + std::to_string(b) + " of n=" + std::to_string(n));
            check(a == o, "oracle batch " + std::to_string(b) + " of n=" + std::to_string(n));
        }
    }
}

static void permutations_match_std() {
    for (u64 len : {1ull, 2ull, 3ull, 17ull, 1000ull, 4096ull}) {
        for (u64 s = 0; s < 3; ++s) {
            const block seed = toBlock(s * 7919 + len);
            std::vector<size_t> a(len);
            std::iota(a.begin(), a.end(), size_t(0));
            HostPrng hp(seed);
            PrngFunctor f{&hp};
            std::random_shuffle(a.begin(), a.end(), f);
            std::vector<size_t> p;
            get_permutation(len, p, seed);
            check(a == p, "product permutation of length " + std::to_string(len));
            u8 sb[16];
            std::memcpy(sb, &seed, 16);
            const std::vector<u64> o = orc::shufflePermutation(len, sb);
            check(std::equal(a.begin(), a.end(), o.begin(), o.end()),
                  "oracle permutation of length " + std::to_string(len));
        }
    }
}

int main() {
    test("getSubset: product and oracle samplers = std::random_shuffle", batches_match_std);
    test("get_permutation: product and oracle = std::random_shuffle", permutations_match_std);
    return failures ? 1 : 0;
}
