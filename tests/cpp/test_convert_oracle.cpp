// CPU-only: the oracle's share conversions (orc::toBinaryMatrix,
// orc::bitInjection, orc::toPackedBin / fromPackedBin) against the revealed
// semantics the reference's tests check (Sh3ConverterTests.cpp:170-435), on
// the engine's adder circuit (Sh3Converter::buildArithToBinCircuit).
#include <cstdio>
#include <stdexcept>
#include <string>
#include "Sh3Converter.h"
#include "orc_core.h"

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

static orc::Mat randMat(u64 r, u64 c, u64 seed, u64 bits) {
    orc::Mat m(r, c);
    u64 x = seed * 0x9E3779B97F4A7C15ull + 7;
    for (u64 i = 0; i < r; ++i)
        for (u64 j = 0; j < c; ++j) {
            x ^= x << 13, x ^= x >> 7, x ^= x << 17;
            const u64 lo = 64 * j;
            u64 v = x;
            if (lo >= bits) v = 0;
            else if (bits - lo < 64) v &= (1ull << (bits - lo)) - 1;
            m(i, j) = (i64)v;
        }
    return m;
}

static orc::Circuit adder(u64 bits) {
    BetaCircuit c;
    Sh3Converter::buildArithToBinCircuit(c, 64, bits);
    c.levelByAndDepth();
    orc::Circuit o;
    o.wireCount = c.mWireCount;
    for (auto& g : c.mLevelGates) o.gates.push_back(orc::Gate{g.in0, g.in1, g.out, (u32)g.type});
    o.levelCounts = c.mLevelCounts;
    o.inputs = c.mInputs;
    o.outputs = c.mOutputs;
    return o;
}

static std::array<orc::Party, 3> gens() {
    std::array<orc::Party, 3> g;
    for (int i = 0; i < 3; ++i)
        g[i].initEncryptor(i, orc::toBlock(0, (u64)i + 1), orc::toBlock(0, (u64)(i + 1) % 3 + 1));
    return g;
}

static void a2b() {
    for (u64 bits : {64ull, 91ull, 128ull}) {
        const u64 cols = (bits + 63) / 64;
        orc::Mat x = randMat(43, cols, bits, bits);
        auto enc = orc::makeEncryptors(0);
        auto g = gens();
        orc::converterInit(g);
        orc::Shared y = orc::toBinaryMatrix(g, adder(bits), orc::shareInt(enc, 0, x), bits);
        check(orc::consistent(y), "replicated shares");
        check(orc::revealBin(y).v == x.v, "revealed == x, bits " + std::to_string(bits));
    }
}

static void bitinj() {
    for (bool two : {false, true}) {
        orc::Mat x = randMat(43, 1, 17 + two, 17);
        auto enc = orc::makeEncryptors(0);
        auto g = gens();
        auto cv = orc::converterInit(g);
        orc::Shared y = orc::bitInjection(g, cv, orc::shareBin(enc, 0, x), 17, two);
        check(orc::consistent(y), "replicated shares");
        orc::Mat r = orc::revealInt(y);
        for (u64 i = 0; i < 43; ++i)
            for (u64 j = 0; j < 17; ++j) check(r(i, j) == (i64)(((u64)x(i, 0) >> j) & 1), "revealed bit");
    }
}

static void packed() {
    orc::Mat x = randMat(100, 2, 5, 91);
    auto enc = orc::makeEncryptors(0);
    orc::Shared X = orc::shareBin(enc, 0, x);
    for (int p = 0; p < 3; ++p) {
        orc::SMat P = orc::toPackedBin(X[p], 91);
        check(P.rows() == 91 && P.cols() == 2, "packed shape");
        for (u64 i = 0; i < 100; ++i)
            for (u64 j = 0; j < 91; ++j)
                for (int s = 0; s < 2; ++s)
                    check((((u64)P.s[s](j, i / 64) >> (i % 64)) & 1) == (((u64)X[p].s[s](i, j / 64) >> (j % 64)) & 1),
                          "bit (i, j) -> (j, i)");
        orc::SMat back = orc::fromPackedBin(P, 100, 91);
        for (int s = 0; s < 2; ++s)
            for (u64 i = 0; i < 100; ++i) {
                check(back.s[s](i, 0) == X[p].s[s](i, 0), "round trip word 0");
                check(back.s[s](i, 1) == (i64)((u64)X[p].s[s](i, 1) & ((1ull << 27) - 1)), "round trip trimmed");
            }
    }
}

int main() {
    test("oracle_a2b_revealed (Sh3_convert_arithToBinaryMatrix_test)", a2b);
    test("oracle_bitinj_revealed (Sh3_convert_BitInjection_test)", bitinj);
    test("oracle_packed_transpose (Sh3_convert_sb64_sPackedBin_test)", packed);
    return failures ? 1 : 0;
}
