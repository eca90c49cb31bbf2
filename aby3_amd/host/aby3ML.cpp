#include "aby3ML.h"

namespace aby3 {

void aby3ML::mul(const si64Matrix& left, const si64Matrix& right, si64Matrix& dest) {
    mEval.asyncMul(mRt.noDependencies(), left, right, dest, mD, MulMode::Gemm).get();
}

void aby3ML::mulTruncate(const si64Matrix& left, const si64Matrix& right, si64Matrix& dest, u64 shift) {
    mEval.asyncMul(mRt.noDependencies(), left, right, dest, mD + shift, MulMode::Gemm).get();
}

void aby3ML::logisticFunc(const si64Matrix& Y, si64Matrix& out) {
    if (mLogistic.mThresholds.empty()) {
        mLogistic.mThresholds = {Sh3Piecewise::Coef(-0.5), Sh3Piecewise::Coef(0.5)};
        mLogistic.mCoefficients.resize(3);
        mLogistic.mCoefficients[1] = {Sh3Piecewise::Coef(0.5), Sh3Piecewise::Coef(1)};
        mLogistic.mCoefficients[2] = {Sh3Piecewise::Coef(1)};
    }
    mLogistic.eval(mRt.noDependencies(), Y, out, mD, mEval).get();
}

void sgdLogisticStep(aby3ML& ml, const si64Matrix& X, const si64Matrix& Y, si64Matrix& w, const u32* batchIdx,
                     u64 B, u64 aB, SgdState& st) {
    Gpu& g = ml.mRt.gpu();
    const u64 d = X.cols();
    // extractBatch (Regression.h:42-58)
    st.XX.resize(B, d);
    st.YY.resize(B, 1);
    GPU_CALL(aby3g_i64_gather_rows(X.data(), X.rows(), d, batchIdx, B, st.XX.data(), g.stream()));
    GPU_CALL(aby3g_i64_gather_rows(Y.data(), Y.rows(), 1, batchIdx, B, st.YY.data(), g.stream()));
    ml.mul(st.XX, w, st.xw);                 // xw = XX * w
    ml.logisticFunc(st.xw, st.fxw);          // f(xw)
    st.err.resize(B, 1);                     // error = f - YY
    GPU_CALL(aby3g_i64_lincomb(2 * B, 1, st.fxw.data(), -1, st.YY.data(), 0, st.err.data(), g.stream()));
    st.XXt.resize(d, B);                     // XX^T
    GPU_CALL(aby3g_i64_transpose(st.XX.data(), B, d, st.XXt.data(), g.stream()));
    ml.mulTruncate(st.XXt, st.err, st.update, aB);  // update = XX^T err / 2^(D + aB)
    GPU_CALL(aby3g_i64_lincomb(2 * d, 1, w.data(), -1, st.update.data(), 0, w.data(), g.stream()));
}

void sgdLogisticStep(aby3ML& ml, const si64Matrix& X, const si64Matrix& Y, si64Matrix& w,
                     const std::vector<u32>& batchIdx, u64 aB, SgdState& st) {
    Gpu& g = ml.mRt.gpu();
    const u64 B = batchIdx.size();
    if (st.idx.bytes() < B * 4) st.idx.reset(g, B * 4);
    toDevice(st.idx.data(), batchIdx.data(), B * 4, g);
    sgdLogisticStep(ml, X, Y, w, st.idx.as<u32>(), B, aB, st);
}

}  // namespace aby3
