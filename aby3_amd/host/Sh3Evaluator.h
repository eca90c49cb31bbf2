// Arithmetic evaluator (aby3/sh3/Sh3Evaluator.h/.cpp) on the GPU.
//
// Every asyncMul keeps the reference's rounds and message schedule; the
// local compute of each round is one or two C-ABI calls on the party's
// stream, and messages are device-to-device copies on the same stream.
#pragma once
#include "Sh3Runtime.h"
#include "Sh3ShareGen.h"
#include "Sh3Types.h"

namespace aby3 {

// Local product semantics of asyncMul on matrices: the fork computes the
// element-wise (Hadamard) product (Sh3Evaluator.cpp:101-103, 667-668), upstream
// the matrix product (:96-99). Both are available; Gemm is the default
// (the upstream tests, aby3-ML and BASELINE name it).
enum class MulMode { Hadamard = ABY3G_MUL_HADAMARD, Gemm = ABY3G_MUL_GEMM };

struct TruncationPair {
    DeviceBuffer mR;      // r (rows x cols), added before the reveal
    si64Matrix mRTrunc;   // shares of r / 2^d
    u64 rows = 0, cols = 0;
};

class Sh3Evaluator {
public:
    void init(u64 partyIdx, block prevSeed, block nextSeed);
    void init(u64 partyIdx, CommPkg& comm, block seed);

    bool DEBUG_disable_randomization = false;
    MulMode mMulMode = MulMode::Gemm;

    // C = A * B, no truncation (Sh3Evaluator.cpp:92-116)
    Sh3Task asyncMul(Sh3Task dep, const si64Matrix& A, const si64Matrix& B, si64Matrix& C);
    Sh3Task asyncMul(Sh3Task dep, const si64Matrix& A, const si64Matrix& B, si64Matrix& C, MulMode mode);
    // C = (A * B) >> shift with a truncation pair (:651-730)
    Sh3Task asyncMul(Sh3Task dep, const si64Matrix& A, const si64Matrix& B, si64Matrix& C, u64 shift);
    Sh3Task asyncMul(Sh3Task dep, const si64Matrix& A, const si64Matrix& B, si64Matrix& C, u64 shift,
                     MulMode mode);

    // Rows [rowOffset, rowOffset + A.rows()) of the truncated matrix product
    // of a totalRows-row A (A holds those rows, B all of B): the randomness
    // of the whole product is taken and the slice's rows used, so C holds
    // those rows of the unsplit product's shares and the party's streams end
    // where the unsplit product leaves them. One party's rows split over
    // GPUs: each GPU runs its slice with the matching slice
    // of the other parties, no exchange between one party's GPUs.
    Sh3Task asyncMulRows(Sh3Task dep, const si64Matrix& A, const si64Matrix& B, si64Matrix& C, u64 shift,
                         u64 rowOffset, u64 totalRows);

    template <Decimal D>
    Sh3Task asyncMul(Sh3Task dep, const sf64Matrix<D>& A, const sf64Matrix<D>& B, sf64Matrix<D>& C) {
        return asyncMul(dep, A.i64Cast(), B.i64Cast(), C.i64Cast(), (u64)D);
    }
    template <Decimal D>
    Sh3Task asyncMul(Sh3Task dep, const sf64Matrix<D>& A, const sf64Matrix<D>& B, sf64Matrix<D>& C, u64 shift) {
        return asyncMul(dep, A.i64Cast(), B.i64Cast(), C.i64Cast(), (u64)D + shift);
    }

    // shared i64 x shared bit via 3-party OT (:119-263)
    Sh3Task asyncMul(Sh3Task dep, const si64Matrix& A, const sbMatrix& B, si64Matrix& C);
    // public i64 x shared bit (:418-501)
    Sh3Task asyncMul(Sh3Task dep, i64 a, const sbMatrix& B, si64Matrix& C);
    // the same product with the zero shares drawn from `zeroGen` (pi_cb_mul,
    // BuildingBlocks.cpp:334-391, draws them from the Encryptor's generator)
    Sh3Task asyncMul(Sh3Task dep, i64 a, const sbMatrix& B, si64Matrix& C, Sh3ShareGen& zeroGen);

    TruncationPair getTruncationTuple(u64 rows, u64 cols, u64 d);

    u64 mPartyIdx = (u64)-1;
    Sh3ShareGen mShareGen;
    // SharedOT keys and counters: mOtPrevRecver (key = next stream bytes
    // [16,32)) and mOtNextRecver (prev stream bytes [16,32)) (:13-14)
    block mOtPrevKey, mOtNextKey;
    u64 mOtPrevIdx = 0, mOtNextIdx = 0;

private:
    DeviceBuffer mWs;  // GEMM workspace (digit planes + split-K slabs), reused
    void* workspace(MulMode mode, u64 M, u64 K, u64 N, size_t& bytes, Gpu& g);
    void shape(MulMode mode, const si64Matrix& A, const si64Matrix& B, u64& M, u64& K, u64& N) const;
    // asyncMul(.., shift, mode); totalRows != 0: rows from rowOffset of a totalRows-row product
    Sh3Task mulTrunc(Sh3Task dep, const si64Matrix& A, const si64Matrix& B, si64Matrix& C, u64 shift, MulMode mode,
                     u64 rowOffset, u64 totalRows);
};

}  // namespace aby3
