// Protocol-level parity of the share conversions (aby3/sh3/Sh3Converter.cpp):
// three GPU parties against the CPU oracle share by share, and at the revealed
// level the reference's own checks (Sh3ConverterTests.cpp:170-282 packed
// transposes, :285-353 arithmetic -> binary, :355-435 bit injection), with the
// reference tests' converter seeds (gens[i].init(toBlock(i+1), toBlock(next+1)),
// :314-316, :385-387).
#include "Basic.h"
#include "Sh3Converter.h"
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

static block convPrevSeed(int i) { return toBlock(0, (u64)i + 1); }
static block convNextSeed(int i) { return toBlock(0, (u64)(i + 1) % 3 + 1); }

static std::array<orc::Party, 3> orcConvGens() {
    std::array<orc::Party, 3> g;
    for (int i = 0; i < 3; ++i)
        g[i].initEncryptor(i, orc::toBlock(0, (u64)i + 1), orc::toBlock(0, (u64)(i + 1) % 3 + 1));
    return g;
}

// x masked to `bits` per row (aby3::details::trim)
static i64Matrix trimmed(i64Matrix x, u64 bits) {
    const u64 cols = x.cols();
    for (u64 i = 0; i < x.rows(); ++i)
        for (u64 j = 0; j < cols; ++j) {
            const u64 lo = j * 64;
            if (lo >= bits)
                x(i, j) = 0;
            else if (bits - lo < 64)
                x(i, j) &= (i64)((1ull << (bits - lo)) - 1);
        }
    return x;
}

// toPackedBin / toBinaryMatrix(sPackedBin): local transposes, both directions
static void packedParity(u64 rows, u64 bits) {
    const u64 cols = (bits + 63) / 64;
    i64Matrix x = trimmed(randMat(rows, cols, rows * 7 + bits), bits);
    ShareSink packed, back;
    run3([&](harness::Party& p) {
        sbMatrix X(rows, bits);
        if (p.idx == 0)
            p.enc.localBinMatrix(p.rt, x, X).get();
        else
            p.enc.remoteBinMatrix(p.rt, X).get();
        Sh3Converter conv;
        sPackedBin P;
        sbMatrix Y;
        conv.toPackedBin(X, P);
        conv.toBinaryMatrix(P, Y);
        packed.put(p.idx, P);
        back.put(p.idx, Y);
        check(P.bitCount() == bits && P.shareCount() == rows && P.simdWidth() == (rows + 63) / 64, "packed shape");
    });
    auto enc = orc::makeEncryptors(0);
    orc::Shared X = orc::shareBin(enc, 0, toOrc(x)), P, Y;
    for (int p = 0; p < 3; ++p) {
        P[p] = orc::toPackedBin(X[p], bits);
        Y[p] = orc::fromPackedBin(P[p], rows, bits);
    }
    packed.expectEq(P, "toPackedBin");
    back.expectEq(Y, "toBinaryMatrix(sPackedBin)");
    // round trip = the input with every share trimmed to `bits` (mtx.trim(),
    // Sh3ConverterTests.cpp:188,220)
    for (int p = 0; p < 3; ++p)
        for (int k = 0; k < 2; ++k) {
            i64Matrix m(rows, cols);
            m.mData = X[p].s[k].v;
            X[p].s[k].v = trimmed(m, bits).mData;
        }
    back.expectEq(X, "round trip");
}

// toBinaryMatrix(si64Matrix -> sbMatrix). presetBits = 0: dest empty (resized
// to 64 * cols bits, as Sh3ConverterTests.cpp:323-336).
static void arithToBin(u64 rows, u64 cols, u64 trimBits, u64 presetBits) {
    i64Matrix x = trimmed(randMat(rows, cols, rows + 3 * cols + trimBits), trimBits);
    const u64 bits = presetBits ? presetBits : 64 * cols;
    ShareSink got;
    std::vector<i64> revealed;
    BetaCircuit cir;
    Sh3Converter::buildArithToBinCircuit(cir, 64, bits);
    cir.levelByAndDepth();
    run3([&](harness::Party& p) {
        si64Matrix X(rows, cols);
        if (p.idx == 0)
            p.enc.localIntMatrix(p.rt, x, X).get();
        else
            p.enc.remoteIntMatrix(p.rt, X).get();
        Sh3ShareGen gen;
        gen.init(convPrevSeed(p.idx), convNextSeed(p.idx));
        Sh3Converter conv;
        conv.init(p.rt, gen);
        sbMatrix Y;
        if (presetBits) Y.resize(rows, presetBits);
        conv.toBinaryMatrix(p.rt.noDependencies(), X, Y).get();
        check(Y.rows() == rows && Y.bitCount() == bits, "dest shape");
        got.put(p.idx, Y);
        i64Matrix r;
        p.enc.revealAll(p.rt, Y, r).get();
        if (p.idx == 0) revealed = r.mData;
    });
    auto enc = orc::makeEncryptors(0);
    auto gens = orcConvGens();
    orc::Shared X = orc::shareInt(enc, 0, toOrc(x));
    orc::converterInit(gens);
    orc::Shared Y = orc::toBinaryMatrix(gens, toOrc(cir), X, bits);
    got.expectEq(Y, "toBinaryMatrix shares");
    // revealed: each 64-bit word is x mod 2^(bits in that word)
    const i64Matrix want = trimmed(x, bits);
    check(revealed == want.mData, "toBinaryMatrix revealed value");
}

static void bitInjection(u64 rows, u64 bits, bool twoRounds) {
    const u64 cols = (bits + 63) / 64;
    i64Matrix x = trimmed(randMat(rows, cols, rows * 5 + bits + twoRounds), bits);
    ShareSink got;
    std::vector<i64> revealed;
    run3([&](harness::Party& p) {
        sbMatrix X(rows, bits);
        if (p.idx == 0)
            p.enc.localBinMatrix(p.rt, x, X).get();
        else
            p.enc.remoteBinMatrix(p.rt, X).get();
        Sh3ShareGen gen;
        gen.init(convPrevSeed(p.idx), convNextSeed(p.idx));
        Sh3Converter conv;
        conv.init(p.rt, gen);
        si64Matrix Y;
        conv.bitInjection(p.rt.noDependencies(), X, Y, twoRounds).get();
        // a second call continues both OT counters and both streams
        si64Matrix Y2;
        conv.bitInjection(p.rt.noDependencies(), X, Y2, twoRounds).get();
        check(Y.rows() == rows && Y.cols() == bits, "dest shape");
        got.put(p.idx, Y2);
        i64Matrix r;
        p.enc.revealAll(p.rt, Y, r).get();
        if (p.idx == 0) revealed = r.mData;
    });
    auto enc = orc::makeEncryptors(0);
    auto gens = orcConvGens();
    orc::Shared X = orc::shareBin(enc, 0, toOrc(x));
    auto cv = orc::converterInit(gens);
    orc::Shared Y1 = orc::bitInjection(gens, cv, X, bits, twoRounds);
    orc::Shared Y2 = orc::bitInjection(gens, cv, X, bits, twoRounds);
    got.expectEq(Y2, "bitInjection shares (second call)");
    check(orc::revealInt(Y1).v == orc::revealInt(Y2).v, "oracle calls agree");
    for (u64 i = 0; i < rows; ++i)
        for (u64 j = 0; j < bits; ++j)
            check((u64)revealed[i * bits + j] == (((u64)x(i, j / 64) >> (j % 64)) & 1), "bitInjection revealed bit");
}

// toBinaryMatrix of an odd number of words advances only P0's prev / P2's
// next stream, so the bitInjection that follows sees the two streams at
// offsets of different parity (the sender kernel's straddling path).
static void a2bThenBitInjection(u64 rows, u64 bits) {
    i64Matrix x = randMat(rows, 1, 4242 + rows);
    i64Matrix xb = trimmed(randMat(rows, 1, 4343 + rows), bits);
    ShareSink gotB, gotI;
    BetaCircuit cir;
    Sh3Converter::buildArithToBinCircuit(cir, 64, 64);
    cir.levelByAndDepth();
    run3([&](harness::Party& p) {
        si64Matrix X(rows, 1);
        sbMatrix XB(rows, bits);
        if (p.idx == 0) {
            p.enc.localIntMatrix(p.rt, x, X).get();
            p.enc.localBinMatrix(p.rt, xb, XB).get();
        } else {
            p.enc.remoteIntMatrix(p.rt, X).get();
            p.enc.remoteBinMatrix(p.rt, XB).get();
        }
        Sh3ShareGen gen;
        gen.init(convPrevSeed(p.idx), convNextSeed(p.idx));
        Sh3Converter conv;
        conv.init(p.rt, gen);
        sbMatrix Y;
        conv.toBinaryMatrix(p.rt.noDependencies(), X, Y).get();
        si64Matrix Z;
        conv.bitInjection(p.rt.noDependencies(), XB, Z).get();
        gotB.put(p.idx, Y);
        gotI.put(p.idx, Z);
    });
    auto enc = orc::makeEncryptors(0);
    auto gens = orcConvGens();
    orc::Shared X = orc::shareInt(enc, 0, toOrc(x)), XB = orc::shareBin(enc, 0, toOrc(xb));
    auto cv = orc::converterInit(gens);
    gotB.expectEq(orc::toBinaryMatrix(gens, toOrc(cir), X, 64), "toBinaryMatrix shares");
    gotI.expectEq(orc::bitInjection(gens, cv, XB, bits, false), "bitInjection shares after it");
}

// bool2arith (BoolBasic.cpp:517-593): one bit through pi_cb_mul (shares
// against the oracle's public-bit product with the Encryptor's zero shares),
// 64 bits through the add / open-to-P2 path (revealed; P2's t is private
// randomness, as the reference's rand(), so its shares are not reproducible).
static void bool2arithTest(u64 rows, u64 bits) {
    i64Matrix x = trimmed(randMat(rows, 1, rows * 3 + bits), bits);
    ShareSink got;
    std::vector<i64> revealed;
    run3([&](harness::Party& p) {
        sbMatrix X(rows, bits);
        if (p.idx == 0)
            p.enc.localBinMatrix(p.rt, x, X).get();
        else
            p.enc.remoteBinMatrix(p.rt, X).get();
        si64Matrix Y;
        bool2arith(p.idx, X, Y, p.enc, p.eval, p.rt);
        check(Y.rows() == rows && Y.cols() == 1, "dest shape");
        got.put(p.idx, Y);
        i64Matrix r;
        p.enc.revealAll(p.rt, Y, r).get();
        if (p.idx == 0) revealed = r.mData;
    });
    check(revealed == x.mData, "bool2arith revealed value");
    if (bits == 1) {
        auto enc = orc::makeEncryptors(0);
        auto ev = orc::makeEvaluators(1);
        orc::Shared X = orc::shareBin(enc, 0, toOrc(x));
        auto hyb = ev;
        for (int p = 0; p < 3; ++p) hyb[p].gen = enc[p].gen;
        got.expectEq(orc::mulPubBit(hyb, 1, X), "bool2arith (1 bit) shares");
    } else {
        // replicated consistency: party i's share 1 == party i-1's share 0
        for (int p = 0; p < 3; ++p) check(got.s[p][1] == got.s[(p + 2) % 3][0], "bool2arith replicated shares");
    }
}

int main() {
    test("packed_43x91 (Sh3_convert_sb64_sPackedBin_test)", [] { packedParity(43, 91); });
    test("packed_1x1", [] { packedParity(1, 1); });
    test("packed_1000x64", [] { packedParity(1000, 64); });
    test("packed_4100x130", [] { packedParity(4100, 130); });
    test("a2b_43x2_trim91 (Sh3_convert_arithToBinaryMatrix_test)", [] { arithToBin(43, 2, 91, 0); });
    test("a2b_43x2_dest91", [] { arithToBin(43, 2, 128, 91); });
    test("a2b_5000x1", [] { arithToBin(5000, 1, 64, 0); });
    test("a2b_300x1_dest17", [] { arithToBin(300, 1, 64, 17); });
    test("a2b_0x1", [] { arithToBin(0, 1, 64, 0); });
    test("bitinj_43x17 (Sh3_convert_BitInjection_test)", [] { bitInjection(43, 17, false); });
    test("bitinj_43x17_twoRounds", [] { bitInjection(43, 17, true); });
    test("bitinj_1000x64", [] { bitInjection(1000, 64, false); });
    test("bitinj_77x130_twoRounds", [] { bitInjection(77, 130, true); });
    test("a2b_333_then_bitinj_21x7 (stream parities differ)", [] { a2bThenBitInjection(333, 7); });
    test("a2b_334_then_bitinj_21x7", [] { a2bThenBitInjection(334, 7); });
    test("bool2arith_1000x64", [] { bool2arithTest(1000, 64); });
    test("bool2arith_300x1 (pi_cb_mul)", [] { bool2arithTest(300, 1); });
    test("bool2arith_5x64", [] { bool2arithTest(5, 64); });
    return g_failures ? 1 : 0;
}
