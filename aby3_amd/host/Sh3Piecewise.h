// Piecewise-linear functions of a shared input (aby3/sh3/Sh3Piecewise.h/.cpp):
// f(x) = sum over regions [t_{c-1} <= x < t_c] * (a_c x + b_c), used for the
// logistic sigmoid of aby3-ML (aby3ML.h:121-139).
#pragma once
#include "Sh3BinaryEvaluator.h"
#include "Sh3Evaluator.h"

namespace aby3 {

class Sh3Piecewise {
public:
    struct Coef {
        Coef() = default;
        Coef(int i) { *this = (i64)i; }
        Coef(i64 i) { *this = i; }
        Coef(double d) { *this = d; }
        bool mIsInteger = false;
        i64 mInt = 0;
        double mDouble = 0;
        void operator=(i64 i) {
            mIsInteger = true;
            mInt = i;
        }
        void operator=(int i) {
            mIsInteger = true;
            mInt = i;
        }
        void operator=(double d) {
            mIsInteger = false;
            mDouble = d;
        }
        double getDouble() const { return mIsInteger ? (double)mInt : mDouble; }
        // Sh3Piecewise.h:55-61
        i64 getFixedPoint(u64 D) const {
            return mIsInteger ? (i64)((u64)mInt * (1ull << D)) : (i64)(mDouble * (double)(1ull << D));
        }
        i64 getInteger() const {
            if (!mIsInteger) throw std::runtime_error(LOCATION);
            return mInt;
        }
    };

    std::vector<Coef> mThresholds;
    std::vector<std::vector<Coef>> mCoefficients;

    // plaintext evaluation (Sh3Piecewise.cpp:90-181)
    void eval(const std::vector<double>& in, std::vector<double>& out) const;

    // 3-party evaluation (Sh3Piecewise.cpp:184-378); inputs/outputs n x 1.
    // Intended semantics of the OT product: A is read before C is written
    // (the reference aliases them).
    Sh3Task eval(Sh3Task dep, const si64Matrix& inputs, si64Matrix& outputs, u64 D, Sh3Evaluator& evaluator);
    template <Decimal D>
    Sh3Task eval(Sh3Task dep, const sf64Matrix<D>& in, sf64Matrix<D>& out, Sh3Evaluator& evaluator) {
        return eval(dep, in.i64Cast(), out.i64Cast(), (u64)D, evaluator);
    }

    std::vector<sbMatrix> mInputRegions;
    std::vector<si64Matrix> functionOutputs;

private:
    void getInputRegions(const si64Matrix& inputs, u64 D, Sh3Runtime& rt, Sh3ShareGen& gen);
    void getFunctionValues(const si64Matrix& inputs, Sh3Runtime& rt, u64 D);
    CircuitLibrary lib;
    Sh3BinaryEvaluator binEng;
};

}  // namespace aby3
