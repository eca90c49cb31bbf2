// Plaintext semantics of the circuit library (CPU only): every circuit
// evaluated on random and edge-case 64-bit inputs against C++ integer
// arithmetic, plus the levelization invariants the engine relies on.
// Anchors: CircuitTests.cpp:16-81 (piecewise helper, 200 tries),
// Sh3BinaryEvaluatorTests.cpp:333-424 (add / msb), BoolTest.cpp (lt = [A<B]).
#include "Circuit.h"
#include <cstdio>
#include <sstream>
#include <functional>
#include <limits>
#include <random>
#include <set>

using namespace aby3;

static int failures = 0;
static void check(bool c, const std::string& w) {
    if (!c) throw std::runtime_error(w);
}
static void test(const char* name, const std::function<void()>& f) {
    try {
        f();
        std::printf("PASS %s\n", name);
    } catch (const std::exception& e) {
        ++failures;
        std::printf("FAIL %s: %s\n", name, e.what());
    }
}

static std::vector<u64> samples(size_t n, u64 seed) {
    std::mt19937_64 r(seed);
    std::vector<u64> v = {0, 1, ~0ull, 1ull << 63, (1ull << 63) - 1, 2, ~1ull, 0x8000000000000001ull};
    while (v.size() < n) {
        u64 x = r();
        switch (v.size() % 4) {
            case 0: x >>= r() % 64; break;
            case 1: x = ~(x >> (r() % 64)); break;
            default: break;
        }
        v.push_back(x);
    }
    return v;
}

static void binaryCircuit(BetaCircuit* c, const std::function<u64(u64, u64)>& f, size_t out = 0) {
    auto a = samples(4096, 1), b = samples(4096, 2);
    // include all pairs of the edge values
    for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 8; ++j) {
            a.push_back(a[i]);
            b.push_back(b[j]);
        }
    a.push_back(5);
    b.push_back(5);
    auto o = c->evalPlain({a, b});
    for (size_t i = 0; i < a.size(); ++i) {
        u64 e = f(a[i], b[i]);
        if (c->mOutputs[out].size() < 64) e &= (1ull << c->mOutputs[out].size()) - 1;
        if (o[out][i] != e)
            throw std::runtime_error("mismatch at a=" + std::to_string(a[i]) + " b=" + std::to_string(b[i]));
    }
}

static void levelInvariants(BetaCircuit* c) {
    // AND-type outputs are never consumed in their own level; batches are independent
    check(c->levelized(), "not levelized");
    std::vector<int> lvlOf(c->mWireCount, -1);
    size_t gi = 0;
    for (size_t L = 0; L < c->mLevelCounts.size(); ++L) {
        std::set<u32> andOut;
        for (u32 k = 0; k < c->mLevelCounts[L]; ++k, ++gi) {
            const auto& g = c->mLevelGates[gi];
            check(!andOut.count(g.in0) && !andOut.count(g.in1), "AND output used in its own level");
            if (isAndType(g.type)) andOut.insert(g.out);
        }
        for (const auto& b : c->mLevelBatches[L]) {
            std::set<u32> outs;
            for (u32 k = 0; k < b.count; ++k) outs.insert(c->mBatchGates[b.begin + k].out);
            for (u32 k = 0; k < b.count; ++k) {
                const auto& g = c->mBatchGates[b.begin + k];
                check(!outs.count(g.in0) && !outs.count(g.in1), "dependency inside a batch");
            }
        }
    }
    check(gi == c->mGates.size(), "level counts");
}

int main() {
    CircuitLibrary lib;
    test("int_comp_helper_64 = MSB(a+b)", [&] {
        auto* c = lib.int_comp_helper(64);
        levelInvariants(c);
        binaryCircuit(c, [](u64 a, u64 b) { return (a + b) >> 63; });
        std::printf("  msb(64): %zu gates, %u AND, %zu levels\n", c->mGates.size(), c->mAndCount, c->mLevelCounts.size());
    });
    test("int_int_lt_64 = [a < b] signed", [&] {
        auto* c = lib.int_int_lt(64);
        levelInvariants(c);
        binaryCircuit(c, [](u64 a, u64 b) { return (u64)((i64)a < (i64)b); });
        std::printf("  lt(64): %zu gates, %u AND, %zu levels\n", c->mGates.size(), c->mAndCount, c->mLevelCounts.size());
    });
    test("int_int_lt_8", [&] {
        auto* c = lib.int_int_lt(8);
        auto a = samples(300, 3), b = samples(300, 4);
        for (auto& x : a) x &= 0xff;
        for (auto& x : b) x &= 0xff;
        auto o = c->evalPlain({a, b});
        for (size_t i = 0; i < a.size(); ++i) check(o[0][i] == (u64)((int8_t)a[i] < (int8_t)b[i]), "lt8");
    });
    test("int_eq_64", [&] {
        auto* c = lib.int_eq(64);
        levelInvariants(c);
        binaryCircuit(c, [](u64 a, u64 b) { return (u64)(a == b); });
    });
    test("int_int_add_64", [&] {
        auto* c = lib.int_int_add(64);
        levelInvariants(c);
        binaryCircuit(c, [](u64 a, u64 b) { return a + b; });
    });
    test("int_int_sub_64", [&] {
        auto* c = lib.int_int_sub(64);
        levelInvariants(c);
        binaryCircuit(c, [](u64 a, u64 b) { return a - b; });
    });
    test("int_int_add_8 (Sh3_BinaryEngine_add_test width)", [&] {
        auto* c = lib.int_int_add(8);
        binaryCircuit(c, [](u64 a, u64 b) { return (a + b) & 0xff; });
    });
    test("bitwise and/or/nor", [&] {
        binaryCircuit(lib.int_int_bitwiseAnd(64), [](u64 a, u64 b) { return a & b; });
        binaryCircuit(lib.int_int_bitwiseOr(64), [](u64 a, u64 b) { return a | b; });
        binaryCircuit(lib.bits_nor_helper(64), [](u64 a, u64 b) { return ~(a | b); });
    });
    test("cmp_swap_64 = (min, max)", [&] {
        auto* c = lib.cmp_swap(64);
        levelInvariants(c);
        binaryCircuit(c, [](u64 a, u64 b) { return (u64)std::min((i64)a, (i64)b); }, 0);
        binaryCircuit(c, [](u64 a, u64 b) { return (u64)std::max((i64)a, (i64)b); }, 1);
    });
    test("int_Sh3Piecewise_helper (CircuitTests.cpp:16-81)", [&] {
        // thresholds t0 < t1; inputs aa_t = x - t_t (as x0 + x2 - t split with b = x1), b
        auto* c = lib.int_Sh3Piecewise_helper(64, 2);
        levelInvariants(c);
        std::mt19937_64 r(7);
        const i64 t0 = -(1 << 15), t1 = 1 << 15;
        for (int tries = 0; tries < 200; ++tries) {
            std::vector<u64> x(64), x1(64), a0(64), a1(64);
            for (int i = 0; i < 64; ++i) {
                x[i] = (u64)((i64)(r() % (1 << 18)) - (1 << 17));
                x1[i] = r();
                a0[i] = x[i] - x1[i] - (u64)t0;
                a1[i] = x[i] - x1[i] - (u64)t1;
            }
            auto o = c->evalPlain({a0, a1, x1});
            for (int i = 0; i < 64; ++i) {
                i64 v = (i64)x[i];
                check(o[0][i] == (u64)(v < t0), "region 0");
                check(o[1][i] == (u64)(v >= t0 && v < t1), "region 1");
                check(o[2][i] == (u64)(v >= t1), "region 2");
            }
        }
    });
    test("BetaCircuit writeBin / readBin round trip (DBServer.cpp:48-54)", [&] {
        const char* names[] = {"int_comp_helper", "int_int_lt", "int_eq", "int_int_add", "int_int_sub",
                               "cmp_swap", "bits_nor_helper", "int_Sh3Piecewise_helper"};
        for (const char* n : names) {
            BetaCircuit* c = lib.byName(n, 64, 2);
            std::stringstream f;
            c->writeBin(f);
            const std::string bytes = f.str();
            BetaCircuit d;
            d.readBin(f);
            check(d.mWireCount == c->mWireCount && d.mGates.size() == c->mGates.size(), std::string(n) + " shape");
            for (size_t i = 0; i < c->mGates.size(); ++i) {
                const auto &g = c->mGates[i], &h = d.mGates[i];
                check(g.in0 == h.in0 && g.in1 == h.in1 && g.out == h.out && g.type == h.type, std::string(n) + " gate");
            }
            check(d.mInputs == c->mInputs && d.mOutputs == c->mOutputs, std::string(n) + " bundles");
            d.levelByAndDepth();
            levelInvariants(&d);
            check(d.mAndCount == c->mAndCount && d.mLevelCounts == c->mLevelCounts, std::string(n) + " levels");
            check(d.serial() != c->serial(), "a loaded circuit gets its own serial");
            std::vector<std::vector<u64>> in;
            for (size_t b = 0; b < c->mInputs.size(); ++b) in.push_back(samples(64, 100 + b));
            check(d.evalPlain(in) == c->evalPlain(in), std::string(n) + " evaluation");
            std::stringstream f2;
            d.writeBin(f2);
            check(f2.str() == bytes, std::string(n) + " re-written bytes");
            // u64 wires, u64 nonXor, bundles, u64 gates, 16 B per gate
            u64 expect = 8 * 5;
            for (auto* bs : {&c->mInputs, &c->mOutputs})
                for (auto& b : *bs) expect += 8 + 4 * b.size();
            check(bytes.size() == expect + 16 * c->mGates.size(), std::string(n) + " layout size");
        }
    });
    test("BetaCircuit readBin rejects malformed files", [&] {
        std::stringstream f;
        lib.int_int_add(8)->writeBin(f);
        const std::string good = f.str();
        auto rejects = [&](std::string b, const char* what) {
            std::stringstream in(b);
            BetaCircuit d;
            bool threw = false;
            try {
                d.readBin(in);
            } catch (const std::runtime_error&) {
                threw = true;
            }
            check(threw, what);
        };
        rejects(good.substr(0, good.size() - 3), "truncated");
        std::string t = good;
        t[t.size() - 4] = 7;  // last gate: Nand (unsupported)
        rejects(t, "gate type");
        t = good;
        t[0] = 2;  // wire count 2: indices out of range
        rejects(t, "wire range");
        t = good;
        t[8] ^= 1;  // non-XOR count off by one
        rejects(t, "and count");
    });
    return failures ? 1 : 0;
}
