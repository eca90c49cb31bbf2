#include "aby3ML.h"
#include <algorithm>
#include <random>

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

void HostPrng::get(void* dst, u64 nbytes) {
    constexpr u64 kBlocks = 256;
    u8* out = static_cast<u8*>(dst);
    while (nbytes) {
        const u64 b = mOff / 16;
        if (mBufBlock == ~0ull || b < mBufBlock || b >= mBufBlock + kBlocks) {
            mBuf.resize(16 * kBlocks);
            GPU_CALL(aby3g_aes_ctr_host(mSeed.data(), b, kBlocks, mBuf.data()));
            mBufBlock = b;
        }
        const u64 at = mOff - 16 * mBufBlock, take = std::min<u64>(nbytes, 16 * kBlocks - at);
        std::memcpy(out, mBuf.data() + at, take);
        out += take;
        mOff += take;
        nbytes -= take;
    }
}

std::vector<double> logisticModel(u64 dim) {
    HostPrng prng(toBlock(1));
    std::vector<double> model(dim, 0.0);
    for (u64 i = 0; i < std::min<u64>(dim, 10); ++i) model[i] = prng.get<int>() % 10;
    return model;
}

void logisticModelGen(const std::vector<double>& model, u64 n, u64 D, i64Matrix& X, i64Matrix& Y) {
    const u64 dim = model.size();
    std::default_random_engine generator(234345);
    std::normal_distribution<double> distribution(1.0, 1.0);
    X.resize(n, dim);
    Y.resize(n, 1);
    const double scale = (double)(1ull << D);
    std::vector<double> row(dim);
    for (u64 i = 0; i < n; ++i) {
        for (u64 j = 0; j < dim; ++j) row[j] = distribution(generator);
        const double noise = distribution(generator);
        double y = 0;
        for (u64 j = 0; j < dim; ++j) y += row[j] * model[j];
        y += noise;
        for (u64 j = 0; j < dim; ++j) X(i, j) = (i64)(row[j] * scale);
        Y(i, 0) = (i64)((y > 0 ? 1.0 : 0.0) * scale);
    }
}

BatchSampler::BatchSampler(u64 n) : mPool(n), mIter(n), mPrng(toBlock(234543234)) {
    for (u64 i = 0; i < n; ++i) mPool[i] = i;
}

void BatchSampler::next(std::vector<u64>& dest) {
    u64 d = 0;
    while (d != dest.size()) {
        const u64 step = std::min<u64>(mPool.size() - mIter, dest.size() - d);
        std::copy(mPool.begin() + mIter, mPool.begin() + mIter + step, dest.begin() + d);
        mIter += step;
        d += step;
        if (mIter == mPool.size()) {
            for (u64 i = 1; i < mPool.size(); ++i) {
                const u64 j = mPrng.get<u64>() % (i + 1);
                if (i != j) std::swap(mPool[i], mPool[j]);
            }
            mIter = 0;
        }
    }
}

MlSeeds mlSeeds(int pIdx) {
    block enc[3], ev[3];
    for (u64 i = 0; i < 3; ++i) {
        HostPrng prng(toBlock(i));
        enc[i] = prng.get<block>();
        ev[i] = prng.get<block>();
    }
    const int prev = (pIdx + 2) % 3;
    return MlSeeds{enc[prev], enc[pIdx], ev[prev], ev[pIdx]};
}

}  // namespace aby3
