#include "Sh3Types.h"

namespace aby3 {

void SharedMat::resize(u64 rows, u64 cols) {
    if (rows == mRows && cols == mCols && mBuf.data()) return;
    mRows = rows;
    mCols = cols;
    Gpu& g = mBuf.gpu() ? *mBuf.gpu() : Gpu::current();
    mBuf.reset(g, 2 * rows * cols * sizeof(i64));
}

std::vector<i64> SharedMat::shareToHost(int s) const {
    std::vector<i64> v(size());
    if (size()) toHost(v.data(), share(s), size() * sizeof(i64), gpu());
    return v;
}

void SharedMat::shareFromHost(int s, const i64* src) {
    if (size()) toDevice(share(s), src, size() * sizeof(i64), gpu());
}

void SharedMat::setZero() {
    if (size()) GPU_CALL(aby3g_memset(data(), 0, 2 * size() * sizeof(i64), gpu().stream()));
}

void SharedMat::copyFrom(const SharedMat& o) {
    resize(o.rows(), o.cols());
    if (size()) d2d(data(), o.data(), 2 * size() * sizeof(i64), gpu());
}

}  // namespace aby3
