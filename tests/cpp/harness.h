// Test harness for protocol-level parity: three parties as three host threads
// in one process (each with its own Sh3Runtime, stream and channels), the way
// the reference's unit tests run them (Sh3EvaluatorTests.cpp:23-131), on GPU
// `device`. Results are compared share-by-share against the CPU oracle.
#pragma once
#include "Sh3Encryptor.h"
#include "Sh3Evaluator.h"
#include "orc_core.h"
#include <cstdio>
#include <exception>
#include <functional>
#include <thread>

namespace harness {

using namespace aby3;

struct Party {
    int idx;
    Sh3Runtime rt;
    Sh3Encryptor enc;
    Sh3Evaluator eval;
};

// Runs f on the three parties concurrently; rethrows the first exception.
inline void run3(const std::function<void(Party&)>& f, int device = 0) {
    auto comms = makeLocalRing();
    std::exception_ptr err[3];
    std::thread th[3];
    for (int i = 0; i < 3; ++i)
        th[i] = std::thread([&, i] {
            try {
                Party p;
                p.idx = i;
                p.rt.init(i, comms[i], device);
                // seeds of the reference tests: enc toBlock(0, i), eval toBlock(1, i)
                p.enc.init(i, toBlock(0, i), toBlock(0, (i + 1) % 3));
                p.eval.init(i, toBlock(1, i), toBlock(1, (i + 1) % 3));
                f(p);
                p.rt.gpu().sync();
            } catch (...) {
                err[i] = std::current_exception();
            }
        });
    for (auto& t : th) t.join();
    for (auto& e : err)
        if (e) std::rethrow_exception(e);
}

inline int g_failures = 0;
inline void check(bool c, const std::string& what) {
    if (!c) throw std::runtime_error("check failed: " + what);
}
inline void test(const char* name, const std::function<void()>& f) {
    try {
        f();
        std::printf("PASS %s\n", name);
    } catch (const std::exception& e) {
        ++g_failures;
        std::printf("FAIL %s: %s\n", name, e.what());
    }
    std::fflush(stdout);
}

inline orc::Mat toOrc(const i64Matrix& m) {
    orc::Mat r(m.rows(), m.cols());
    std::copy(m.mData.begin(), m.mData.end(), r.v.begin());
    return r;
}

// compares every party's two shares with the oracle's
struct ShareSink {
    std::vector<i64> s[3][2];
    void put(int p, const SharedMat& m) {
        s[p][0] = m.shareToHost(0);
        s[p][1] = m.shareToHost(1);
    }
    void expectEq(const orc::Shared& o, const std::string& what) const {
        for (int p = 0; p < 3; ++p)
            for (int k = 0; k < 2; ++k)
                if (s[p][k] != o[p].s[k].v)
                    throw std::runtime_error(what + ": party " + std::to_string(p) + " share " + std::to_string(k) +
                                             " differs from the oracle");
    }
};

inline i64Matrix randMat(u64 r, u64 c, u64 seed, i64 lo = INT64_MIN, i64 hi = INT64_MAX) {
    i64Matrix m(r, c);
    u64 x = seed * 0x9E3779B97F4A7C15ull + 1;
    for (auto& v : m.mData) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        if (lo == INT64_MIN && hi == INT64_MAX)
            v = (i64)x;
        else
            v = lo + (i64)(x % (u64)(hi - lo + 1));
    }
    return m;
}

}  // namespace harness
