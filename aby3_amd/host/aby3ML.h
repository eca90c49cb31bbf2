// The aby3-ML engine wrapper (aby3-ML/aby3ML.h:103-139) and one iteration of
// SGD_Logistic (aby3-ML/Regression.h:218-295) on device shares.
#pragma once
#include "Sh3Encryptor.h"
#include "Sh3Evaluator.h"
#include "Sh3Piecewise.h"

namespace aby3 {

class aby3ML {
public:
    aby3ML(Sh3Runtime& rt, Sh3Encryptor& enc, Sh3Evaluator& eval, u64 D) : mRt(rt), mEnc(enc), mEval(eval), mD(D) {}

    // mul: asyncMul(left, right, dest) with shift D (aby3ML.h:103-108), matrix product
    void mul(const si64Matrix& left, const si64Matrix& right, si64Matrix& dest);
    // mulTruncate: shift D + shift (aby3ML.h:110-116)
    void mulTruncate(const si64Matrix& left, const si64Matrix& right, si64Matrix& dest, u64 shift);
    // logisticFunc: piecewise sigmoid, thresholds -0.5 / 0.5, f = 0 | 0.5 + x | 1 (aby3ML.h:121-139)
    void logisticFunc(const si64Matrix& Y, si64Matrix& out);

    Sh3Runtime& mRt;
    Sh3Encryptor& mEnc;
    Sh3Evaluator& mEval;
    u64 mD;
    Sh3Piecewise mLogistic;
};

struct SgdState {
    si64Matrix XX, YY, XXt, xw, fxw, err, update;
    DeviceBuffer idx;
};

// One SGD_Logistic iteration on the batch of B row indices at device pointer
// `batchIdx` (e.g. a slice of a device-resident permutation, so no host
// upload or stream sync sits in the iteration) of (X, Y):
//   XX, YY = extractBatch; xw = mul(XX, w); fxw = logistic(xw);
//   err = fxw - YY; update = mulTruncate(XX^T, err, aB); w = w - update
// (Regression.h:252-287).
void sgdLogisticStep(aby3ML& ml, const si64Matrix& X, const si64Matrix& Y, si64Matrix& w,
                     const u32* batchIdx, u64 B, u64 aB, SgdState& st);
// Host-index convenience form: uploads the indices (and waits for the upload).
void sgdLogisticStep(aby3ML& ml, const si64Matrix& X, const si64Matrix& Y, si64Matrix& w,
                     const std::vector<u32>& batchIdx, u64 aB, SgdState& st);

}  // namespace aby3
