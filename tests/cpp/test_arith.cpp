// Protocol-level parity of the arithmetic evaluator: input sharing,
// asyncMul (Hadamard and GEMM, with and without truncation), the OT bit
// multiplications and reveal -- every party's shares bit-exact against the
// CPU oracle on the reference tests' seeds (Sh3EvaluatorTests.cpp:594-690,
// :350-410, :780-1032; Test.cpp:74-191).
#include "Basic.h"
#include "harness.h"

using namespace aby3;
using namespace harness;

// alias: 0 C separate, 1 C is A, 2 C is B (the product overwrites an operand)
static void mulTest(MulMode mode, u64 M, u64 K, u64 N, bool trunc, u64 d, u64 seed, int alias = 0) {
    const u64 bRows = mode == MulMode::Gemm ? K : M;
    const u64 bCols = mode == MulMode::Gemm ? N : K;
    i64Matrix a = randMat(M, K, seed), b = randMat(bRows, bCols, seed + 1);
    if (trunc) {  // fixed-point operands: |x| < 2^20 keeps |sum a*b| far below 2^62 (truncation valid)
        a = randMat(M, K, seed, -(1ll << 20), 1ll << 20);
        b = randMat(bRows, bCols, seed + 1, -(1ll << 20), 1ll << 20);
    }
    ShareSink got;
    std::vector<i64> revealed;
    run3([&](harness::Party& p) {
        si64Matrix A(M, K), B(bRows, bCols), C;
        if (p.idx == 0) {
            p.enc.localIntMatrix(p.rt, a, A).get();
            p.enc.localIntMatrix(p.rt, b, B).get();
        } else {
            p.enc.remoteIntMatrix(p.rt, A).get();
            p.enc.remoteIntMatrix(p.rt, B).get();
        }
        si64Matrix& out = alias == 1 ? A : alias == 2 ? B : C;
        if (trunc)
            p.eval.asyncMul(p.rt, A, B, out, d, mode).get();
        else
            p.eval.asyncMul(p.rt, A, B, out, mode).get();
        got.put(p.idx, out);
        i64Matrix r;
        p.enc.revealAll(p.rt, out, r).get();
        if (p.idx == 0) revealed = r.mData;
    });
    auto enc = orc::makeEncryptors(0);
    auto ev = orc::makeEvaluators(1);
    orc::Shared A = orc::shareInt(enc, 0, toOrc(a)), B = orc::shareInt(enc, 0, toOrc(b));
    orc::MulMode om = mode == MulMode::Gemm ? orc::MUL_GEMM : orc::MUL_HADAMARD;
    orc::Shared C = trunc ? orc::mulTrunc(ev, om, A, B, d) : orc::mul(ev, om, A, B);
    got.expectEq(C, "asyncMul");
    check(revealed == orc::revealInt(C).v, "revealAll");
    // plaintext: exact product, and within 1 of the floor for truncation (:396-407)
    orc::SMat As, Bs;
    orc::Mat plain;
    As.s[0] = toOrc(a);
    As.s[1] = orc::Mat(M, K);
    Bs.s[0] = toOrc(b);
    Bs.s[1] = orc::Mat(bRows, bCols);
    // (a0, 0) x (b0, 0) with A1 = B1 = 0 gives the plain product
    orc::localProduct(om, As, Bs, plain);
    for (u64 i = 0; i < plain.size(); ++i) {
        if (!trunc) {
            check(revealed[i] == plain.v[i], "plain product");
        } else {
            // three floored pair shares plus the floored reveal: the result lies in
            // (floor(xy/2^d) - 4, floor(xy/2^d) + 1] (Sh3EvaluatorTests.cpp:396-407 bounds it by 4)
            i64 e = plain.v[i] >> d;
            check(revealed[i] - e <= 1 && e - revealed[i] < 4, "truncation error out of (-4, 1]");
        }
    }
}

// Sh3_Evaluator_asyncMul_test (Sh3EvaluatorTests.cpp:20-135): per trial, ten
// dependent multiplications chained through Sh3Task::then,
//   task = asyncMul(task, A, B, C); task = task.then(A = C + A);
// with one .get() at the end; every party's shares of C and A are compared
// with the oracle's after the chain, and the revealed C with the plaintext
// recurrence c = a * b; a = c + a (mod 2^64).
static void chainedMulTest(MulMode mode, u64 dim, u64 trials, u64 seed) {
    const orc::MulMode om = mode == MulMode::Gemm ? orc::MUL_GEMM : orc::MUL_HADAMARD;
    for (u64 t = 0; t < trials; ++t) {
        i64Matrix a = randMat(dim, dim, seed + 2 * t), b = randMat(dim, dim, seed + 2 * t + 1);
        ShareSink gotC, gotA;
        std::vector<i64> revealed;
        run3([&](harness::Party& p) {
            si64Matrix A(dim, dim), B(dim, dim), C(dim, dim);
            if (p.idx == 0) {
                p.enc.localIntMatrix(p.rt, a, A).get();
                p.enc.localIntMatrix(p.rt, b, B).get();
            } else {
                p.enc.remoteIntMatrix(p.rt, A).get();
                p.enc.remoteIntMatrix(p.rt, B).get();
            }
            Sh3Task task = p.rt.noDependencies();
            for (u64 j = 0; j < dim; ++j) {
                task = p.eval.asyncMul(task, A, B, C, mode);
                task = task.then([&](CommPkg&, Sh3Task& self) {
                    // A = C + A, both shares (sMatrix operator+)
                    GPU_CALL(aby3g_i64_lincomb(2 * A.size(), 1, C.data(), 1, A.data(), 0, A.data(),
                                               self.getRuntime().gpu().stream()));
                });
            }
            task.get();
            gotC.put(p.idx, C);
            gotA.put(p.idx, A);
            i64Matrix r;
            p.enc.revealAll(p.rt, C, r).get();
            if (p.idx == 0) revealed = r.mData;
        });
        auto enc = orc::makeEncryptors(0);
        auto ev = orc::makeEvaluators(1);
        orc::Shared A = orc::shareInt(enc, 0, toOrc(a)), B = orc::shareInt(enc, 0, toOrc(b)), C;
        for (u64 j = 0; j < dim; ++j) {
            C = orc::mul(ev, om, A, B);
            for (int p = 0; p < 3; ++p)
                for (int k = 0; k < 2; ++k)
                    for (u64 i = 0; i < A[p].s[k].v.size(); ++i)
                        A[p].s[k].v[i] = (i64)((u64)C[p].s[k].v[i] + (u64)A[p].s[k].v[i]);
        }
        gotC.expectEq(C, "chained asyncMul: C");
        gotA.expectEq(A, "chained asyncMul: A = C + A");
        // plaintext recurrence
        orc::SMat As, Bs;
        As.s[0] = toOrc(a);
        As.s[1] = orc::Mat(dim, dim);
        Bs.s[0] = toOrc(b);
        Bs.s[1] = orc::Mat(dim, dim);
        orc::Mat c;
        for (u64 j = 0; j < dim; ++j) {
            orc::localProduct(om, As, Bs, c);
            for (u64 i = 0; i < c.size(); ++i) As.s[0].v[i] = (i64)((u64)c.v[i] + (u64)As.s[0].v[i]);
        }
        check(revealed == c.v, "chained asyncMul: revealed C differs from the plaintext recurrence");
    }
}

static void bitMulTest(bool pub, u64 n, u64 seed) {
    i64Matrix a = randMat(n, 1, seed), bits = randMat(n, 1, seed + 7, 0, 1);
    const i64 apub = 0x123456789abcdefll;
    ShareSink got;
    std::vector<i64> revealed;
    run3([&](harness::Party& p) {
        si64Matrix A(n, 1), C;
        sbMatrix B(n, 1);
        if (p.idx == 0) {
            p.enc.localBinMatrix(p.rt, bits, B).get();
            if (!pub) p.enc.localIntMatrix(p.rt, a, A).get();
        } else {
            p.enc.remoteBinMatrix(p.rt, B).get();
            if (!pub) p.enc.remoteIntMatrix(p.rt, A).get();
        }
        if (pub)
            p.eval.asyncMul(p.rt, apub, B, C).get();
        else
            p.eval.asyncMul(p.rt, A, B, C).get();
        got.put(p.idx, C);
        i64Matrix r;
        p.enc.revealAll(p.rt, C, r).get();
        if (p.idx == 0) revealed = r.mData;
    });
    auto enc = orc::makeEncryptors(0);
    auto ev = orc::makeEvaluators(1);
    orc::Shared B = orc::shareBin(enc, 0, toOrc(bits));
    orc::Shared C;
    if (pub) {
        C = orc::mulPubBit(ev, apub, B);
    } else {
        orc::Shared A = orc::shareInt(enc, 0, toOrc(a));
        C = orc::mulBit(ev, A, B);
    }
    got.expectEq(C, pub ? "asyncMul(i64, sb)" : "asyncMul(si64, sb)");
    for (u64 i = 0; i < n; ++i) check(revealed[i] == (bits(i, 0) ? (pub ? apub : a(i, 0)) : 0), "bit product");
}

static void arithBasic16() {
    // Test.cpp:74-191: x = i, y = 16 - i; mul (Hadamard, the fork's cipher_mul)
    const int T = 16;
    i64Matrix x(T, 1), y(T, 1);
    for (int i = 0; i < T; ++i) {
        x(i, 0) = i;
        y(i, 0) = T - i;
    }
    std::vector<i64> revealed;
    run3([&](harness::Party& p) {
        si64Matrix X(T, 1), Y(T, 1), Z;
        if (p.idx == 0) {
            p.enc.localIntMatrix(p.rt, x, X).get();
            p.enc.localIntMatrix(p.rt, y, Y).get();
        } else {
            p.enc.remoteIntMatrix(p.rt, X).get();
            p.enc.remoteIntMatrix(p.rt, Y).get();
        }
        p.eval.asyncMul(p.rt, X, Y, Z, MulMode::Hadamard).get();
        i64Matrix r;
        p.enc.revealAll(p.rt, Z, r).get();
        if (p.idx == 0) revealed = r.mData;
    });
    for (int i = 0; i < T; ++i) check(revealed[i] == i * (T - i), "mul 16");
}

// large_data_sending / large_data_receiving (aby3-Basic/Basic.cpp:3-62):
// host and device columns in chunks, both directions, ragged last chunk
static void largeData(u64 len, u64 chunk) {
    i64Matrix col(len, 1);
    for (u64 i = 0; i < len; ++i) col(i, 0) = (i64)(i * 0x9E3779B97F4A7C15ull);
    i64Matrix gotHost, gotDev, gotBack;
    run3([&](harness::Party& p) {
        Gpu& g = p.rt.gpu();
        if (p.idx == 0) {
            large_data_sending(0, col, p.rt, true, chunk);  // host -> P1
            DeviceBuffer d(g, 8 * len);
            toDevice(d.data(), col.mData.data(), 8 * len, g);
            large_data_sending(0, d.as<i64>(), len, p.rt, true, chunk);  // device -> P1
            g.sync();
        } else if (p.idx == 1) {
            i64Matrix h(len, 1);
            large_data_receiving(1, h, p.rt, true, chunk);
            gotHost = h;
            DeviceBuffer d(g, 8 * len);
            large_data_receiving(1, d.as<i64>(), len, p.rt, true, chunk);
            i64Matrix back(len, 1);
            toHost(back.mData.data(), d.data(), 8 * len, g);
            gotDev = back;
            large_data_sending(1, d.as<i64>(), len, p.rt, false, chunk);  // device -> P0, P1's prev
            g.sync();
        }
        if (p.idx == 0) {
            i64Matrix h(len, 1);
            DeviceBuffer d(g, 8 * len);
            large_data_receiving(0, d.as<i64>(), len, p.rt, false, chunk);  // from next (P1)
            toHost(h.mData.data(), d.data(), 8 * len, g);
            gotBack = h;
        }
    });
    check(gotHost.mData == col.mData, "host column");
    check(gotDev.mData == col.mData, "device column");
    check(gotBack.mData == col.mData, "device column back to prev");
}

int main() {
    test("large_data_sending_receiving_10007_in_chunks_of_1000", [] { largeData(10007, 1000); });
    test("large_data_sending_receiving_4096_one_chunk", [] { largeData(4096, MAX_SENDING_SIZE); });
    test("share_reveal_and_hadamard_16 (Test.cpp arith_basic_test mul)", arithBasic16);
    test("asyncMul_hadamard_128x128", [] { mulTest(MulMode::Hadamard, 128, 128, 128, false, 0, 1); });
    test("asyncMul_gemm_10x10 (Sh3_Evaluator_mul_test)", [] { mulTest(MulMode::Gemm, 10, 10, 10, false, 0, 2); });
    test("asyncMul_gemm_33x17x65", [] { mulTest(MulMode::Gemm, 33, 17, 65, false, 0, 3); });
    test("asyncMul_gemm_256x128x1 (LR xw)", [] { mulTest(MulMode::Gemm, 256, 128, 1, false, 0, 4); });
    test("asyncMul_trunc_hadamard_4x4_D8", [] { mulTest(MulMode::Hadamard, 4, 4, 4, true, 8, 5); });
    test("asyncMul_trunc_gemm_4x4_D8 (matrixFixed_test)", [] { mulTest(MulMode::Gemm, 4, 4, 4, true, 8, 6); });
    test("asyncMul_trunc_gemm_128x256x1_D27 (LR update)", [] { mulTest(MulMode::Gemm, 128, 256, 1, true, 27, 7); });
    test("asyncMul_trunc_gemm_256x256x256_D16", [] { mulTest(MulMode::Gemm, 256, 256, 256, true, 16, 8); });
    // C aliasing an operand (C = A * B with C == A or B): the reference forms the
    // product in an Eigen temporary before assigning
    test("asyncMul_gemm_alias_C_is_A_64", [] { mulTest(MulMode::Gemm, 64, 64, 64, false, 0, 12, 1); });
    test("asyncMul_trunc_gemm_alias_C_is_A_512_D16", [] { mulTest(MulMode::Gemm, 512, 512, 512, true, 16, 13, 1); });
    test("asyncMul_trunc_gemm_alias_C_is_B_300x300x40", [] { mulTest(MulMode::Gemm, 300, 300, 40, true, 16, 14, 2); });
    test("asyncMul_trunc_hadamard_alias_C_is_B_100x7_D8", [] { mulTest(MulMode::Hadamard, 100, 7, 7, true, 8, 15, 2); });
    // Sh3_Evaluator_asyncMul_test: 10 trials of 10 dependent 10x10 products (the
    // reference expects the upstream GEMM; the fork's Hadamard form as well)
    test("asyncMul_chained_then_gemm_10x10 (Sh3_Evaluator_asyncMul_test)",
         [] { chainedMulTest(MulMode::Gemm, 10, 10, 100); });
    test("asyncMul_chained_then_hadamard_10x10", [] { chainedMulTest(MulMode::Hadamard, 10, 10, 200); });
    test("asyncMul_si64_x_sb (sh3_asyncArithBinMul_test)", [] { bitMulTest(false, 100, 9); });
    test("asyncMul_i64_x_sb (sh3_asyncPubArithBinMul_test)", [] { bitMulTest(true, 100, 10); });
    test("asyncMul_si64_x_sb_1000", [] { bitMulTest(false, 1000, 11); });
    return g_failures ? 1 : 0;
}
