// Share containers of the host runtime (aby3/sh3/Sh3Types.h, Sh3FixedPoint.h).
//
// Device layout: one party's shared matrix is ONE contiguous allocation
// [2][rows][cols] of i64 in HBM -- share 0 (x_i) then share 1 (x_{i-1}) --
// where the reference keeps two separate Eigen heap buffers
// (Sh3Types.h:198-271). Binary matrices keep the reference's packing: rows x
// ceil(bits/64) i64 words per share (Sh3Types.h:335-387).
#pragma once
#include "Device.h"
#include <vector>

namespace aby3 {

// Plaintext matrix on the host (eMatrix<i64>, RowMajor).
struct i64Matrix {
    u64 mRows = 0, mCols = 0;
    std::vector<i64> mData;
    i64Matrix() = default;
    i64Matrix(u64 r, u64 c) { resize(r, c); }
    void resize(u64 r, u64 c) {
        mRows = r;
        mCols = c;
        mData.assign(r * c, 0);
    }
    u64 rows() const { return mRows; }
    u64 cols() const { return mCols; }
    u64 size() const { return mData.size(); }
    i64* data() { return mData.data(); }
    const i64* data() const { return mData.data(); }
    i64& operator()(u64 r, u64 c) { return mData[r * mCols + c]; }
    i64 operator()(u64 r, u64 c) const { return mData[r * mCols + c]; }
    i64& operator()(u64 i) { return mData[i]; }
    i64 operator()(u64 i) const { return mData[i]; }
    void setZero() { std::fill(mData.begin(), mData.end(), 0); }
};

// Two device shares of `cols`-wide i64 rows.
class SharedMat {
public:
    SharedMat() = default;
    SharedMat(u64 rows, u64 cols) { resize(rows, cols); }
    SharedMat(SharedMat&&) = default;
    SharedMat& operator=(SharedMat&&) = default;

    void resize(u64 rows, u64 cols);
    u64 rows() const { return mRows; }
    u64 cols() const { return mCols; }
    u64 size() const { return mRows * mCols; }  // elements per share
    i64* share(int s) const { return mBuf.as<i64>() + (u64)s * size(); }
    i64* data() const { return mBuf.as<i64>(); }  // [2][rows][cols]
    Gpu& gpu() const { return *mBuf.gpu(); }
    bool empty() const { return size() == 0; }

    // host views for tests and reveals (synchronize the owning stream)
    std::vector<i64> shareToHost(int s) const;
    void shareFromHost(int s, const i64* src);
    void setZero();
    void copyFrom(const SharedMat& o);  // deep copy on this party's stream

protected:
    DeviceBuffer mBuf;
    u64 mRows = 0, mCols = 0;
};

// si64Matrix (Sh3Types.h:198-274)
class si64Matrix : public SharedMat {
public:
    using SharedMat::SharedMat;
};

// sf64Matrix<D> = si64Matrix + decimal (Sh3FixedPoint.h:327-443)
template <Decimal D>
class sf64Matrix : public si64Matrix {
public:
    static const Decimal mDecimal = D;
    using si64Matrix::si64Matrix;
    si64Matrix& i64Cast() { return *this; }
    const si64Matrix& i64Cast() const { return *this; }
};

// sbMatrix (Sh3Types.h:335-387): rows x ceil(bitCount/64) words per share.
// si64 (Sh3Types.h:113-170): one replicated 64-bit share pair, host values.
struct si64 {
    i64 mData[2] = {0, 0};
};

class sbMatrix : public SharedMat {
public:
    sbMatrix() = default;
    sbMatrix(u64 rows, u64 bitCount) { resize(rows, bitCount); }
    void resize(u64 rows, u64 bitCount) {
        mBitCount = bitCount;
        SharedMat::resize(rows, (bitCount + 63) / 64);
    }
    u64 bitCount() const { return mBitCount; }
    u64 i64Cols() const { return cols(); }
    u64 i64Size() const { return size(); }

private:
    u64 mBitCount = 0;
};

// sPackedBin (Sh3Types.h:451-560): the bit-transposed form of shareCount
// values of bitCount bits -- bitCount rows of ceil(shareCount/64) words per
// share (row b holds bit b of every value, 64 values per word).
class sPackedBin : public SharedMat {
public:
    sPackedBin() = default;
    sPackedBin(u64 shareCount, u64 bitCount) { reset(shareCount, bitCount); }
    void reset(u64 shareCount, u64 bitCount) {
        mShareCount = shareCount;
        SharedMat::resize(bitCount, (shareCount + 63) / 64);
    }
    u64 shareCount() const { return mShareCount; }
    u64 bitCount() const { return rows(); }
    u64 simdWidth() const { return cols(); }

private:
    u64 mShareCount = 0;
};

// Fixed-point helpers (Sh3FixedPoint.h:21-112)
inline i64 toFixed(double v, u64 D) { return (i64)(v * (double)(1ull << D)); }
inline double fromFixed(i64 v, u64 D) { return (double)v / (double)(1ull << D); }

}  // namespace aby3
