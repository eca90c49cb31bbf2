// Protocol-level parity of the binary engine and everything built on it:
// every library circuit evaluated by three GPU parties, compared share by
// share with the CPU oracle evaluating the same levelized gate list, and at
// the revealed level against plaintext semantics (Sh3BinaryEvaluatorTests.cpp
// :333-424, BoolTest.cpp:21-300, Test.cpp:74-191, SortTest.cpp:354-487,
// Sh3PiecewiseTests.cpp:13-83).
#include <algorithm>
#include "Basic.h"
#include "Sh3Piecewise.h"
#include "harness.h"

using namespace aby3;
using namespace harness;

static orc::Circuit toOrc(const BetaCircuit& c) {
    orc::Circuit o;
    o.wireCount = c.mWireCount;
    for (auto& g : c.mLevelGates) o.gates.push_back(orc::Gate{g.in0, g.in1, g.out, (u32)g.type});
    o.levelCounts = c.mLevelCounts;
    o.inputs = c.mInputs;
    o.outputs = c.mOutputs;
    return o;
}

static i64Matrix mask(const i64Matrix& m, u64 bits) {
    i64Matrix r = m;
    if (bits < 64)
        for (auto& v : r.mData) v &= (i64)((1ull << bits) - 1);
    return r;
}

// Evaluates `cir` (2 inputs of `bits`) on rows x 2 random inputs on the GPU and in the oracle.
static void circuitParity(const char* name, BetaCircuit* (CircuitLibrary::*make)(u64), u64 bits, u64 rows,
                          const std::function<u64(u64, u64)>& f) {
    CircuitLibrary lib;
    BetaCircuit* cir = (lib.*make)(bits);
    i64Matrix a = mask(randMat(rows, 1, rows + 11), bits), b = mask(randMat(rows, 1, rows + 12), bits);
    const size_t nOut = cir->mOutputs.size();
    std::vector<ShareSink> got(nOut);
    std::vector<std::vector<i64>> revealed(nOut);
    run3([&](harness::Party& p) {
        sbMatrix A(rows, bits), B(rows, bits);
        if (p.idx == 0) {
            p.enc.localBinMatrix(p.rt, a, A).get();
            p.enc.localBinMatrix(p.rt, b, B).get();
        } else {
            p.enc.remoteBinMatrix(p.rt, A).get();
            p.enc.remoteBinMatrix(p.rt, B).get();
        }
        std::vector<sbMatrix> outs(nOut);
        std::vector<sbMatrix*> op;
        for (auto& o : outs) op.push_back(&o);
        CircuitLibrary local;
        evalCircuit((local.*make)(bits), {&A, &B}, op, p.eval, p.rt);
        for (size_t o = 0; o < nOut; ++o) {
            got[o].put(p.idx, outs[o]);
            i64Matrix r(rows, outs[o].i64Cols());
            p.enc.revealAll(p.rt, outs[o], r).get();
            if (p.idx == 0) revealed[o] = r.mData;
        }
    });
    auto enc = orc::makeEncryptors(0);
    auto ev = orc::makeEvaluators(1);
    orc::Shared A = orc::shareBin(enc, 0, toOrc(a)), B = orc::shareBin(enc, 0, toOrc(b));
    orc::Circuit oc = toOrc(*cir);
    auto outs = orc::evalCircuit(ev, oc, {&A, &B});
    for (size_t o = 0; o < nOut; ++o) got[o].expectEq(outs[o], std::string(name) + " output " + std::to_string(o));
    for (u64 i = 0; i < rows; ++i) {
        u64 e = f((u64)a(i, 0), (u64)b(i, 0));
        check((u64)revealed[0][i] == e, std::string(name) + " revealed value");
    }
}

static void boolBasic16() {
    // BoolTest.cpp:21-300 values: x = i, y = 16 - i
    const int T = 16;
    i64Matrix x(T, 1), y(T, 1);
    for (int i = 0; i < T; ++i) {
        x(i, 0) = i;
        y(i, 0) = T - i;
    }
    std::vector<i64> gt, eq, add, orr, andd, nt;
    run3([&](harness::Party& p) {
        sbMatrix X(T, 64), Y(T, 64);
        if (p.idx == 0) {
            p.enc.localBinMatrix(p.rt, x, X).get();
            p.enc.localBinMatrix(p.rt, y, Y).get();
        } else {
            p.enc.remoteBinMatrix(p.rt, X).get();
            p.enc.remoteBinMatrix(p.rt, Y).get();
        }
        auto rev = [&](sbMatrix& m, std::vector<i64>& dst) {
            i64Matrix r;
            p.enc.revealAll(p.rt, m, r).get();
            if (p.idx == 0) dst = r.mData;
        };
        sbMatrix r1, r2, r3, r4, r5, r6;
        bool_cipher_lt(p.idx, Y, X, r1, p.eval, p.rt);  // BoolTest.cpp:122: lt(Y, X) = [x > y]
        rev(r1, gt);
        bool_cipher_eq(p.idx, Y, X, r2, p.eval, p.rt);
        rev(r2, eq);
        bool_cipher_add(p.idx, X, Y, r3, p.eval, p.rt);
        rev(r3, add);
        bool_cipher_or(p.idx, X, Y, r4, p.eval, p.rt);
        rev(r4, orr);
        bool_cipher_and(p.idx, X, Y, r5, p.eval, p.rt);
        rev(r5, andd);
        bool_cipher_not(p.idx, X, r6);
        rev(r6, nt);
    });
    for (int i = 0; i < T; ++i) {
        check(gt[i] == (i > T - i), "gt");
        check(eq[i] == (i == T - i), "eq");
        check(add[i] == T, "add");
        check(orr[i] == (i | (T - i)), "or");
        check(andd[i] == (i & (T - i)), "and");
        check(nt[i] == ~(i64)i, "not");
    }
}

static void arithCompare16() {
    // Test.cpp:74-191: gt / ge / eq through fetch_msb and the eq circuit,
    // mul_ab (shared x shared bit) on x = i, y = 16 - i
    const int T = 16;
    i64Matrix x(T, 1), y(T, 1);
    for (int i = 0; i < T; ++i) {
        x(i, 0) = i;
        y(i, 0) = T - i;
    }
    std::vector<i64> gt, ge, eq, mulab;
    run3([&](harness::Party& p) {
        si64Matrix X(T, 1), Y(T, 1), AB;
        if (p.idx == 0) {
            p.enc.localIntMatrix(p.rt, x, X).get();
            p.enc.localIntMatrix(p.rt, y, Y).get();
        } else {
            p.enc.remoteIntMatrix(p.rt, X).get();
            p.enc.remoteIntMatrix(p.rt, Y).get();
        }
        sbMatrix g, gq, e;
        cipher_gt(p.idx, X, Y, g, p.eval, p.rt);
        cipher_ge(p.idx, X, Y, gq, p.eval, p.rt);
        circuit_cipher_eq(p.idx, X, Y, e, p.eval, p.rt);
        cipher_mul(p.idx, X, g, AB, p.eval, p.rt);
        i64Matrix r;
        p.enc.revealAll(p.rt, g, r).get();
        if (p.idx == 0) gt = r.mData;
        p.enc.revealAll(p.rt, gq, r).get();
        if (p.idx == 0) ge = r.mData;
        p.enc.revealAll(p.rt, e, r).get();
        if (p.idx == 0) eq = r.mData;
        p.enc.revealAll(p.rt, AB, r).get();
        if (p.idx == 0) mulab = r.mData;
    });
    for (int i = 0; i < T; ++i) {
        check((gt[i] & 1) == (i > T - i), "gt");
        check((ge[i] & 1) == (i >= T - i), "ge");
        check((eq[i] & 1) == (i == T - i), "eq");
        check(mulab[i] == (i > T - i ? i : 0), "mul_ab");
    }
}

static void fetchMsbParity(u64 n) {
    i64Matrix a = randMat(n, 1, 31), b = randMat(n, 1, 32);
    ShareSink got;
    run3([&](harness::Party& p) {
        si64Matrix A(n, 1), B(n, 1);
        if (p.idx == 0) {
            p.enc.localIntMatrix(p.rt, a, A).get();
            p.enc.localIntMatrix(p.rt, b, B).get();
        } else {
            p.enc.remoteIntMatrix(p.rt, A).get();
            p.enc.remoteIntMatrix(p.rt, B).get();
        }
        sbMatrix g;
        cipher_gt(p.idx, A, B, g, p.eval, p.rt);
        got.put(p.idx, g);
    });
    auto enc = orc::makeEncryptors(0);
    auto ev = orc::makeEvaluators(1);
    orc::Shared A = orc::shareInt(enc, 0, toOrc(a)), B = orc::shareInt(enc, 0, toOrc(b));
    orc::Shared diff = A;
    for (int p = 0; p < 3; ++p)
        for (int s = 0; s < 2; ++s)
            for (u64 k = 0; k < n; ++k) diff[p].s[s].v[k] = (i64)((u64)B[p].s[s].v[k] - (u64)A[p].s[s].v[k]);
    CircuitLibrary lib;
    got.expectEq(orc::fetchMsb(ev, toOrc(*lib.int_comp_helper(64)), diff), "cipher_gt");
    auto r = orc::revealBin(orc::fetchMsb(ev, toOrc(*lib.int_comp_helper(64)), diff));
    (void)r;
}

static void piecewiseParity(u64 n, u64 D) {
    // the reference's sigmoid (aby3ML.h:121-139): thresholds +-0.5, f = 0 | 0.5 + x | 1
    i64Matrix x(n, 1);
    for (u64 i = 0; i < n; ++i) x(i, 0) = (i64)(((double)i / n * 4.0 - 2.0) * (double)(1ull << D));
    ShareSink got;
    std::vector<i64> revealed;
    run3([&](harness::Party& p) {
        si64Matrix X(n, 1), Y;
        if (p.idx == 0)
            p.enc.localIntMatrix(p.rt, x, X).get();
        else
            p.enc.remoteIntMatrix(p.rt, X).get();
        Sh3Piecewise pw;
        pw.mThresholds = {Sh3Piecewise::Coef(-0.5), Sh3Piecewise::Coef(0.5)};
        pw.mCoefficients.resize(3);
        pw.mCoefficients[1] = {Sh3Piecewise::Coef(0.5), Sh3Piecewise::Coef(1)};
        pw.mCoefficients[2] = {Sh3Piecewise::Coef(1)};
        pw.eval(p.rt, X, Y, D, p.eval).get();
        got.put(p.idx, Y);
        i64Matrix r;
        p.enc.revealAll(p.rt, Y, r).get();
        if (p.idx == 0) revealed = r.mData;
    });
    auto enc = orc::makeEncryptors(0);
    auto ev = orc::makeEvaluators(1);
    orc::Shared X = orc::shareInt(enc, 0, toOrc(x));
    orc::Piecewise pw;
    pw.thresholds = {orc::Coef{false, 0, -0.5}, orc::Coef{false, 0, 0.5}};
    pw.coefs = {{}, {orc::Coef{false, 0, 0.5}, orc::Coef{true, 1, 0}}, {orc::Coef{true, 1, 0}}};
    CircuitLibrary lib;
    orc::Shared Y = orc::piecewiseEval(ev, pw, toOrc(*lib.int_Sh3Piecewise_helper(64, 2)), X, D);
    got.expectEq(Y, "piecewise");
    // plaintext sigmoid approximation within 2^-16 (Sh3PiecewiseTests.cpp:13-83)
    for (u64 i = 0; i < n; ++i) {
        double v = (double)x(i, 0) / (double)(1ull << D);
        double e = v < -0.5 ? 0 : (v < 0.5 ? 0.5 + v : 1.0);
        double gotv = (double)revealed[i] / (double)(1ull << D);
        check(std::abs(gotv - e) <= 1.0 / (1ull << D), "sigmoid value");
    }
}

static void mergeTest(std::vector<u64> lens, u64 seed) {
    // SortTest.cpp:354-487: merge sorted arrays, compare with std::sort
    std::vector<i64Matrix> arrs;
    std::vector<i64> all;
    u64 x = seed;
    for (u64 L : lens) {
        std::vector<i64> v(L);
        for (auto& e : v) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            e = (i64)(x >> 24);  // < 2^40, non-negative
        }
        std::sort(v.begin(), v.end());
        i64Matrix m(L, 1);
        m.mData = v;
        arrs.push_back(m);
        all.insert(all.end(), v.begin(), v.end());
    }
    std::sort(all.begin(), all.end());
    std::vector<i64> revealed;
    run3([&](harness::Party& p) {
        std::vector<sbMatrix> data(lens.size());
        for (size_t k = 0; k < lens.size(); ++k) {
            data[k].resize(lens[k], 64);
            if (p.idx == 0)
                p.enc.localBinMatrix(p.rt, arrs[k], data[k]).get();
            else
                p.enc.remoteBinMatrix(p.rt, data[k]).get();
        }
        sbMatrix sorted;
        odd_even_multi_merge(data, sorted, p.idx, p.eval, p.rt);
        i64Matrix r;
        p.enc.revealAll(p.rt, sorted, r).get();
        if (p.idx == 0) revealed = r.mData;
    });
    check(revealed == all, "merged order");
}

static void replicatedInput() {
    // setReplicatedInput (Sh3BinaryEvaluator.cpp:105-138): a one-row shared
    // constant broadcast to every row; a & c over 300 rows
    const u64 rows = 300;
    i64Matrix a = randMat(rows, 1, 41), c(1, 1);
    c(0, 0) = (i64)0xF0F0F0F00FF00FF0ull;
    std::vector<i64> revealed;
    run3([&](harness::Party& p) {
        sbMatrix A(rows, 64), C(1, 64), out;
        if (p.idx == 0) {
            p.enc.localBinMatrix(p.rt, a, A).get();
            p.enc.localBinMatrix(p.rt, c, C).get();
        } else {
            p.enc.remoteBinMatrix(p.rt, A).get();
            p.enc.remoteBinMatrix(p.rt, C).get();
        }
        CircuitLibrary lib;
        Sh3BinaryEvaluator eng;
        eng.setCir(lib.int_int_bitwiseAnd(64), rows, p.eval.mShareGen);
        eng.setInput(0, A);
        eng.setReplicatedInput(1, C);
        eng.asyncEvaluate(p.rt.noDependencies()).then([&](Sh3Task&) { eng.getOutput(0, out); }).get();
        i64Matrix r;
        p.enc.revealAll(p.rt, out, r).get();
        if (p.idx == 0) revealed = r.mData;
    });
    for (u64 i = 0; i < rows; ++i) check(revealed[i] == (a(i, 0) & c(0, 0)), "a & replicated c");
}

// Several evaluators of one party alive at once: three setCir calls before
// any evaluation (the third finds both buffers of the Gpu's mask ring held and
// draws into its own), evaluated in order, the first one evaluated twice on
// its masks. Every party's output shares must equal those of the same calls
// made one evaluator at a time (same keys, same messages, only the
// scheduling and the mask buffers differ).
static void interleavedEvaluators() {
    const u64 rows = 5000;
    i64Matrix a = randMat(rows, 1, 91), b = randMat(rows, 1, 92);
    using Make = BetaCircuit* (CircuitLibrary::*)(u64);
    const Make makes[3] = {&CircuitLibrary::int_int_add, &CircuitLibrary::int_comp_helper, &CircuitLibrary::int_eq};
    // [pattern][party][call] -> both shares of output 0
    std::vector<std::vector<i64>> got[2][3];
    for (int pattern = 0; pattern < 2; ++pattern)
        run3([&](harness::Party& p) {
            sbMatrix A(rows, 64), B(rows, 64);
            if (p.idx == 0) {
                p.enc.localBinMatrix(p.rt, a, A).get();
                p.enc.localBinMatrix(p.rt, b, B).get();
            } else {
                p.enc.remoteBinMatrix(p.rt, A).get();
                p.enc.remoteBinMatrix(p.rt, B).get();
            }
            CircuitLibrary lib;
            Sh3BinaryEvaluator eng[3];
            sbMatrix out[4];
            auto run = [&](int k, sbMatrix& o) {
                eng[k].setInput(0, A);
                eng[k].setInput(1, B);
                eng[k].asyncEvaluate(p.rt.noDependencies()).then([&](Sh3Task&) { eng[k].getOutput(0, o); }).get();
            };
            if (pattern == 0) {
                for (int k = 0; k < 3; ++k) {
                    eng[k].setCir((lib.*makes[k])(64), rows, p.eval.mShareGen);
                    run(k, out[k]);
                    if (k == 0) run(0, out[3]);
                }
            } else {
                for (int k = 0; k < 3; ++k) eng[k].setCir((lib.*makes[k])(64), rows, p.eval.mShareGen);
                run(0, out[0]);
                run(0, out[3]);
                run(1, out[1]);
                run(2, out[2]);
            }
            for (auto& o : out) {
                got[pattern][p.idx].push_back(o.shareToHost(0));
                got[pattern][p.idx].push_back(o.shareToHost(1));
            }
        });
    for (int i = 0; i < 3; ++i) {
        check(got[0][i].size() == 8 && got[1][i].size() == 8, "interleaved: outputs collected");
        for (size_t k = 0; k < got[0][i].size(); ++k)
            check(got[0][i][k] == got[1][i][k], "interleaved evaluators: shares equal to one-at-a-time evaluation");
    }
}

int main() {
    auto msb = [](u64 a, u64 b) { return (a + b) >> 63; };
    test("bin_msb_64_rows256 (Sh3_BinaryEngine_add_msb_test)",
         [&] { circuitParity("msb", &CircuitLibrary::int_comp_helper, 64, 256, msb); });
    test("bin_msb_64_rows1", [&] { circuitParity("msb", &CircuitLibrary::int_comp_helper, 64, 1, msb); });
    test("bin_msb_64_rows5000", [&] { circuitParity("msb", &CircuitLibrary::int_comp_helper, 64, 5000, msb); });
    test("bin_lt_64", [&] {
        circuitParity("lt", &CircuitLibrary::int_int_lt, 64, 3000,
                      [](u64 a, u64 b) { return (u64)((i64)a < (i64)b); });
    });
    test("bin_add_8 (Sh3_BinaryEngine_add_test)", [&] {
        circuitParity("add8", &CircuitLibrary::int_int_add, 8, 256, [](u64 a, u64 b) { return (a + b) & 0xff; });
    });
    test("bin_and_8 (Sh3_BinaryEngine_and_test)", [&] {
        circuitParity("and8", &CircuitLibrary::int_int_bitwiseAnd, 8, 256, [](u64 a, u64 b) { return a & b; });
    });
    test("bin_add_64", [&] {
        circuitParity("add", &CircuitLibrary::int_int_add, 64, 1000, [](u64 a, u64 b) { return a + b; });
    });
    test("bin_eq_64", [&] {
        circuitParity("eq", &CircuitLibrary::int_eq, 64, 700, [](u64 a, u64 b) { return (u64)(a == b); });
    });
    test("bin_nor_64", [&] {
        circuitParity("nor", &CircuitLibrary::bits_nor_helper, 64, 300, [](u64 a, u64 b) { return ~(a | b); });
    });
    test("bin_cmp_swap_64", [&] {
        circuitParity("cmp_swap", &CircuitLibrary::cmp_swap, 64, 2049,
                      [](u64 a, u64 b) { return (u64)std::min((i64)a, (i64)b); });
    });
    test("bool_basic_16 (BoolTest.cpp)", boolBasic16);
    test("arith_compare_16 (Test.cpp gt/ge/eq/mul_ab)", arithCompare16);
    test("cipher_gt_parity_1000", [] { fetchMsbParity(1000); });
    test("interleaved_evaluators (mask ring, re-evaluation)", interleavedEvaluators);
    test("piecewise_sigmoid_256_D16", [] { piecewiseParity(256, 16); });
    test("setReplicatedInput_and_300", replicatedInput);
    test("odd_even_merge_2x8 (SortTest.cpp)", [] { mergeTest({8, 8}, 1); });
    test("odd_even_multi_merge_4 (SortTest.cpp)", [] { mergeTest({5, 7, 8, 3}, 2); });
    test("odd_even_multi_merge_8x64", [] { mergeTest({64, 64, 64, 64, 64, 64, 64, 64}, 3); });
    return g_failures ? 1 : 0;
}
