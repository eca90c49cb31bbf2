// The square-root ORAM and its position map (aby3-Basic/SqrtOram.h) on the GPU
// engine, three parties, checked at the revealed level exactly as the
// reference's own tests check them: pos_map_test (aby3_tests/Test.cpp:771-906:
// the linear map at 16 entries, the recursive map at 64 entries with a stash
// miss and a stash hit) and sqrt_oram_test (:908-981), here for every access
// instead of access 0 only, plus a deeper recursive map.
#include "SqrtOram.h"
#include "harness.h"

using namespace aby3;
using harness::check;
using harness::run3;
using harness::test;

// units [n][rows] holding value(i, j), shared by party 0 one unit at a time
static std::vector<sbMatrix> shareUnits(harness::Party& p, u64 n, u64 rows, u64 bits,
                                        const std::function<i64(u64, u64)>& value) {
    std::vector<sbMatrix> enc(n);
    for (u64 i = 0; i < n; ++i) {
        i64Matrix x(rows, 1);
        for (u64 j = 0; j < rows; ++j) x(j, 0) = value(i, j);
        enc[i].resize(rows, bits);
        if (p.idx == 0)
            p.enc.localBinMatrix(p.rt, x, enc[i]).get();
        else
            p.enc.remoteBinMatrix(p.rt, enc[i]).get();
    }
    return enc;
}

static i64 reveal1(harness::Party& p, const sbMatrix& m) {
    i64Matrix r;
    p.enc.revealAll(p.rt, m, r).get();
    return r(0, 0);
}

// the position map over a shuffled vector of units i (Test.cpp:790-905)
static void posMapTest(u64 n, u64 pack, u64 S, const std::vector<i64>& queries, bool expectLinear) {
    std::vector<i64> got(queries.size(), -1);
    run3([&](harness::Party& p) {
        auto enc = shareUnits(p, n, 1, 1, [](u64 i, u64) { return (i64)i; });
        std::vector<si64> pi;
        efficient_shuffle_with_random_permutation(enc, p.idx, enc, pi, p.enc, p.eval, p.rt);
        std::vector<boolIndex> perm(n);
        for (u64 i = 0; i < n; ++i) perm[i] = boolIndex(pi[i].mData[0], pi[i].mData[1]);
        ABY3PosMap map(n, pack, S, perm, p.idx, p.enc, p.eval, p.rt);
        check(map.linear() == expectLinear, "linear / recursive branch");
        const boolShare fake(false, p.idx);
        for (size_t q = 0; q < queries.size(); ++q) {
            const i64 phy = map.access(boolIndex(queries[q], p.idx), fake);
            check(phy >= 0 && (u64)phy < n, "physical index in range");
            const i64 v = reveal1(p, enc[(u64)phy]);
            if (p.idx == 0) got[q] = v;
        }
    });
    for (size_t q = 0; q < queries.size(); ++q)
        check(got[q] == queries[q], "posMap(" + std::to_string(queries[q]) + ") -> " + std::to_string(got[q]));
}

static void oramTest(u64 n, u64 S, u64 pack, u64 block, u64 bits) {
    std::vector<std::vector<i64>> got(n);
    auto value = [](u64 i, u64 j) { return (i64)(i * 1000003 + j); };
    run3([&](harness::Party& p) {
        auto enc = shareUnits(p, n, block, bits, value);
        ABY3SqrtOram oram((int)n, (int)S, (int)pack, p.idx, p.enc, p.eval, p.rt);
        oram.initiate(enc);
        // every index once, in the reference test's order (last first)
        for (i64 i = (i64)n - 1; i >= 0; --i) {
            sbMatrix r = oram.access(boolIndex(i, p.idx));
            i64Matrix v;
            p.enc.revealAll(p.rt, r, v).get();
            if (p.idx == 0) got[(u64)i] = v.mData;
        }
    });
    for (u64 i = 0; i < n; ++i)
        for (u64 j = 0; j < block; ++j) check(got[i][j] == value(i, j), "ORAM access " + std::to_string(i));
}

int main() {
    test("pos_map linear: 16 entries, pack 2, S 32 (Test.cpp:790-835)",
         [] { posMapTest(16, 2, 32, {16 / 3}, true); });
    // the reference labels this case "recursive", but map_len = 64 / 8 = 8 < S
    // = 16 selects the linear map there too (oram.h:106-111)
    test("pos_map 'recursive' case: 64 entries, pack 8, S 16, indices 1, 5, 1 (Test.cpp:838-905)",
         [] { posMapTest(64, 8, 16, {1, 5, 1}, true); });
    test("pos_map recursive: 64 entries, pack 8, S 4, stash miss + hit",
         [] { posMapTest(64, 8, 4, {1, 5, 1, 63, 9}, false); });
    test("pos_map two recursion levels: 256 entries, pack 4, S 8",
         [] { posMapTest(256, 4, 8, {7, 200, 7, 3}, false); });
    test("sqrt_oram: 32 blocks of 4 rows, pack 4, S 32 (Test.cpp:908-981), every access",
         [] { oramTest(32, 32, 4, 4, 1); });
    test("sqrt_oram: 64 blocks of 2 x 64 bits, pack 2, S 8 (recursive position map)",
         [] { oramTest(64, 8, 2, 2, 64); });
    return harness::g_failures ? 1 : 0;
}
