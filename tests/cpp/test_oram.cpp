// The square-root ORAM and its position map (aby3-Basic/SqrtOram.h) on the GPU
// engine, three parties, checked two ways:
//  * at the revealed level exactly as the reference's own tests check them:
//    pos_map_test (aby3_tests/Test.cpp:771-906: the linear map at 16 entries,
//    the recursive map at 64 entries with a stash miss and a stash hit) and
//    sqrt_oram_test (:908-981), here for every access instead of access 0
//    only, plus a deeper recursive map;
//  * share by share against the oracle's restatement (oracle/src/orc_oram.cpp):
//    after every access, every party's whole position-map state at every
//    recursion level (usage map, permutation, packed map, stash, the shares of
//    the physical index before it is opened), and every party's shares of the
//    ORAM memory after the shuffle and of each access result.
#include "Basic.h"
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

static orc::Circuit toOrc(BetaCircuit* c) {
    if (!c->levelized()) c->levelByAndDepth();
    orc::Circuit o;
    o.wireCount = c->mWireCount;
    for (auto& g : c->mLevelGates) o.gates.push_back(orc::Gate{g.in0, g.in1, g.out, (u32)g.type});
    o.levelCounts = c->mLevelCounts;
    o.inputs = c->mInputs;
    o.outputs = c->mOutputs;
    return o;
}

// the circuits the product's BoolBasic helpers evaluate (Basic.cpp)
static orc::OramCircuits oramCircuits() {
    CircuitLibrary& lib = basicLibrary();
    return orc::OramCircuits{toOrc(lib.int_eq(64)), toOrc(lib.int_int_bitwiseAnd(64)), toOrc(lib.int_int_bitwiseOr(1))};
}

// party view of the position map, in the order orc::PosMap3::dump uses
static std::vector<i64> dump(const ABY3PosMap& m) {
    std::vector<i64> d{(i64)m.linear(), (i64)m.t, m.last_physical_index.indexShares[0],
                       m.last_physical_index.indexShares[1]};
    for (auto& u : m.usage_map) d.insert(d.end(), {(i64)u.bshares[0], (i64)u.bshares[1]});
    for (auto& x : m.permutation) d.insert(d.end(), {x.indexShares[0], x.indexShares[1]});
    for (auto* v : {&m.packed_index, &m.stash})
        for (auto& q : *v) {
            d.insert(d.end(), {q.logicalIndex.indexShares[0], q.logicalIndex.indexShares[1]});
            for (auto& x : q.packedIndices) d.insert(d.end(), {x.indexShares[0], x.indexShares[1]});
        }
    if (m.subPosMap) {
        const std::vector<i64> s = dump(*m.subPosMap);
        d.insert(d.end(), s.begin(), s.end());
    }
    return d;
}

static std::vector<i64> words(const sbMatrix& m) {
    std::vector<i64> a = m.shareToHost(0), b = m.shareToHost(1);
    a.insert(a.end(), b.begin(), b.end());
    return a;
}
static std::vector<i64> words(const orc::SMat& m) {
    std::vector<i64> a = m.s[0].v;
    a.insert(a.end(), m.s[1].v.begin(), m.s[1].v.end());
    return a;
}

// the oracle's units, shared by party 0 one unit at a time as shareUnits does
static std::vector<orc::Shared> orcUnits(std::array<orc::Party, 3>& enc, u64 n, u64 rows,
                                         const std::function<i64(u64, u64)>& value) {
    std::vector<orc::Shared> u;
    for (u64 i = 0; i < n; ++i) {
        orc::Mat x(rows, 1);
        for (u64 j = 0; j < rows; ++j) x(j, 0) = value(i, j);
        u.push_back(orc::shareBin(enc, 0, x));
    }
    return u;
}

static i64 reveal1(harness::Party& p, const sbMatrix& m) {
    i64Matrix r;
    p.enc.revealAll(p.rt, m, r).get();
    return r(0, 0);
}

// the position map over a shuffled vector of units i (Test.cpp:790-905)
static void posMapTest(u64 n, u64 pack, u64 S, const std::vector<i64>& queries, bool expectLinear) {
    std::vector<i64> got(queries.size(), -1);
    std::vector<std::vector<i64>> state[3];  // [party][query]
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
            state[p.idx].push_back(dump(map));
            const i64 v = reveal1(p, enc[(u64)phy]);
            if (p.idx == 0) got[q] = v;
        }
    });
    for (size_t q = 0; q < queries.size(); ++q)
        check(got[q] == queries[q], "posMap(" + std::to_string(queries[q]) + ") -> " + std::to_string(got[q]));
    // the oracle: same seeds (enc toBlock(0, i), eval toBlock(1, i)), same calls
    auto oenc = orc::makeEncryptors(0);
    auto oev = orc::makeEvaluators(1);
    const orc::OramCircuits cir = oramCircuits();
    orc::OramOps ops{&oev, &cir};
    auto units = orcUnits(oenc, n, 1, [](u64 i, u64) { return (i64)i; });
    orc::Shared T, Pi;
    for (int q = 0; q < 3; ++q) {
        T[q] = orc::SMat(n, 1);
        for (u64 i = 0; i < n; ++i)
            for (int s = 0; s < 2; ++s) T[q].s[s].v[i] = units[i][q].s[s].v[0];
    }
    orc::shuffleWithPermutation(oenc, T, Pi);
    std::vector<orc::Index3> perm(n);
    for (u64 i = 0; i < n; ++i)
        for (int q = 0; q < 3; ++q) perm[i].s[q] = {Pi[q].s[0].v[i], Pi[q].s[1].v[i]};
    orc::PosMap3 omap(oenc, ops, n, pack, S, perm);
    for (size_t q = 0; q < queries.size(); ++q) {
        const i64 phy = omap.access(orc::Index3::pub(queries[q]), orc::Bool3::pub(false));
        (void)phy;
        for (int pp = 0; pp < 3; ++pp)
            check(state[pp][q] == omap.dump(pp), "position-map state of party " + std::to_string(pp) +
                                                     " after access " + std::to_string(q) + " vs the oracle");
    }
}

static void oramTest(u64 n, u64 S, u64 pack, u64 block, u64 bits) {
    std::vector<std::vector<i64>> got(n);
    std::vector<std::vector<i64>> mem[3], res[3];  // [party][unit or access]
    auto value = [](u64 i, u64 j) { return (i64)(i * 1000003 + j); };
    std::vector<i64> order;
    for (i64 i = (i64)n - 1; i >= 0; --i) order.push_back(i);  // the reference test's order (last first)
    run3([&](harness::Party& p) {
        auto enc = shareUnits(p, n, block, bits, value);
        ABY3SqrtOram oram((int)n, (int)S, (int)pack, p.idx, p.enc, p.eval, p.rt);
        oram.initiate(enc);
        for (auto& m : oram.shuffle_mem) mem[p.idx].push_back(words(m));
        for (i64 i : order) {
            sbMatrix r = oram.access(boolIndex(i, p.idx));
            res[p.idx].push_back(words(r));
            i64Matrix v;
            p.enc.revealAll(p.rt, r, v).get();
            if (p.idx == 0) got[(u64)i] = v.mData;
        }
    });
    for (u64 i = 0; i < n; ++i)
        for (u64 j = 0; j < block; ++j) check(got[i][j] == value(i, j), "ORAM access " + std::to_string(i));
    auto oenc = orc::makeEncryptors(0);
    auto oev = orc::makeEvaluators(1);
    const orc::OramCircuits cir = oramCircuits();
    orc::OramOps ops{&oev, &cir};
    orc::SqrtOram3 oram(oenc, ops, n, S, pack);
    oram.initiate(orcUnits(oenc, n, block, value));
    for (int pp = 0; pp < 3; ++pp)
        for (u64 i = 0; i < n; ++i)
            check(mem[pp][i] == words(oram.shuffle_mem[i][pp]), "ORAM memory unit " + std::to_string(i) + " of party " +
                                                                    std::to_string(pp) + " vs the oracle");
    for (size_t k = 0; k < order.size(); ++k) {
        const orc::Shared r = oram.access(orc::Index3::pub(order[k]));
        for (int pp = 0; pp < 3; ++pp)
            check(res[pp][k] == words(r[pp]), "ORAM access " + std::to_string(order[k]) + " shares of party " +
                                                  std::to_string(pp) + " vs the oracle");
    }
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
