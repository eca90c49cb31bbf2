#include "Sh3Piecewise.h"

namespace aby3 {

namespace {
// fixed-point product, bits [D, D+64) of the 128-bit product (Sh3Piecewise.cpp:14-36)
i64 fxmul(i64 a, i64 b, u64 D) { return (i64)(((__int128)a * (__int128)b) >> D); }
}  // namespace

void Sh3Piecewise::eval(const std::vector<double>& inD, std::vector<double>& outD) const {
    const u64 D = 16;
    const size_t T = mThresholds.size();
    if (!T || mCoefficients.size() != T + 1) throw std::runtime_error(LOCATION);
    outD.assign(inD.size(), 0);
    for (size_t i = 0; i < inD.size(); ++i) {
        const i64 in = (i64)(inD[i] * (double)(1ull << D));
        std::vector<u8> thr(T), region(T + 1);
        for (size_t t = 0; t < T; ++t) thr[t] = in < mThresholds[t].getFixedPoint(D);
        region[0] = thr[0];
        for (size_t t = 1; t < T; ++t) region[t] = (1 ^ thr[t - 1]) & thr[t];
        region[T] = 1 ^ thr[T - 1];
        i64 out = 0;
        for (size_t t = 0; t <= T; ++t) {
            i64 ft = 0, inPower = (i64)(1ll << D);
            for (const auto& c : mCoefficients[t]) {
                ft += fxmul(c.getFixedPoint(D), inPower, D);
                inPower = fxmul(in, inPower, D);
            }
            out += region[t] * ft;
        }
        outD[i] = (double)out / (double)(1ull << D);
    }
}

void Sh3Piecewise::getInputRegions(const si64Matrix& inputs, u64 D, Sh3Runtime& rt, Sh3ShareGen& gen) {
    // Sh3Piecewise.cpp:381-516. P0 reshares x0 + x2 as the binary sharing
    // (x0 + x2, 0, 0); P1/P2 expose x1 as (0, x1, 0). Per threshold the
    // circuit computes MSB((x0 + x2 - t) + x1) = [x < t]. The T shifted
    // copies and x1 go straight into the circuit's input wires in one launch
    // (setTwoInputSharing), with the one message P0 -> P1.
    const u64 n = inputs.size();
    const u64 T = mThresholds.size();
    BetaCircuit* cir = lib.int_Sh3Piecewise_helper(64, T);
    binEng.setCir(cir, n, gen);
    std::vector<u64> in0(T);
    std::vector<i64> off(T);
    for (u64 t = 0; t < T; ++t) {
        in0[t] = t;
        off[t] = (i64)(0 - (u64)mThresholds[t].getFixedPoint(D));
    }
    setTwoInputSharing(binEng, (int)rt.mPartyIdx, {{&inputs, 1}}, 1, in0, off, T, rt.mComm, rt.gpu());
    mInputRegions.resize(T + 1);
    binEng.asyncEvaluate(rt.noDependencies())
        .then([&, T](Sh3Task&) {
            for (u64 t = 0; t <= T; ++t) binEng.getOutput(t, mInputRegions[t]);
        })
        .get();
}

void Sh3Piecewise::getFunctionValues(const si64Matrix& inputs, Sh3Runtime& rt, u64 D) {
    // Sh3Piecewise.cpp:518-567: degree <= 1 with an integer slope
    Gpu& g = rt.gpu();
    const u64 n = inputs.size();
    const u64 p = rt.mPartyIdx;
    for (const auto& c : mCoefficients)
        if (c.size() > 2) throw std::runtime_error("not implemented " LOCATION);
    functionOutputs.resize(mCoefficients.size());
    for (u64 c = 0; c < mCoefficients.size(); ++c) {
        if (mCoefficients[c].size() <= 1) continue;
        auto& f = functionOutputs[c];
        f.resize(inputs.rows(), inputs.cols());
        const i64 cst = mCoefficients[c][0].getFixedPoint(D);
        if (!mCoefficients[c][1].mIsInteger) throw std::runtime_error("not implemented " LOCATION);
        const i64 a = mCoefficients[c][1].getInteger();
        for (int s = 0; s < 2; ++s)
            GPU_CALL(aby3g_i64_lincomb(n, a, inputs.share(s), 0, nullptr, (p < 2 && (u64)s == p) ? cst : 0,
                                       f.share(s), g.stream()));
    }
}

Sh3Task Sh3Piecewise::eval(Sh3Task dep, const si64Matrix& inputs, si64Matrix& outputs, u64 D,
                           Sh3Evaluator& evaluator) {
    if (inputs.cols() != 1) throw std::runtime_error(LOCATION);
    if (mThresholds.empty()) throw std::runtime_error(LOCATION);
    if (mCoefficients.size() != mThresholds.size() + 1) throw std::runtime_error(LOCATION);
    Sh3Runtime& rt = dep.getRuntime();
    Gpu& g = rt.gpu();
    const u64 n = inputs.size();
    getInputRegions(inputs, D, rt, evaluator.mShareGen);
    getFunctionValues(inputs, rt, D);
    outputs.resize(inputs.rows(), inputs.cols());
    outputs.setZero();
    for (u64 c = 0; c < mCoefficients.size(); ++c) {
        const auto& co = mCoefficients[c];
        if (co.empty()) continue;
        auto& f = functionOutputs[c];
        if (co.size() > 1)
            evaluator.asyncMul(dep, f, mInputRegions[c], f).get();  // private value x region bit
        else
            evaluator.asyncMul(dep, co[0].getFixedPoint(D), mInputRegions[c], f).get();  // public constant
        GPU_CALL(aby3g_i64_lincomb(2 * n, 1, outputs.data(), 1, f.data(), 0, outputs.data(), g.stream()));
    }
    return dep;
}

}  // namespace aby3
