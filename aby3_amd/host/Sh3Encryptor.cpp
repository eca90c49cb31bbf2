#include "Sh3Encryptor.h"

namespace aby3 {

void Sh3Encryptor::init(u64 partyIdx, block prevSeed, block nextSeed) {
    mPartyIdx = partyIdx;
    mShareGen.init(prevSeed, nextSeed);
}
void Sh3Encryptor::init(u64 partyIdx, CommPkg& comm, block seed) {
    mPartyIdx = partyIdx;
    mShareGen.init(comm, seed);
}

Sh3Task Sh3Encryptor::shareImpl(Sh3Task dep, const i64Matrix* m, SharedMat& dest, int kind, u64 rowOffset,
                                 u64 totalRows) {
    if (totalRows && rowOffset + dest.rows() > totalRows)
        throw std::invalid_argument("sharing rows [" + std::to_string(rowOffset) + ", " +
                                    std::to_string(rowOffset + dest.rows()) + ") of a " + std::to_string(totalRows) +
                                    "-row matrix " LOCATION);
    return dep
        .then([this, m, &dest, kind, rowOffset, totalRows](CommPkg& comm, Sh3Task& self) {
            Gpu& g = self.getRuntime().gpu();
            if (m && (m->rows() != dest.rows() || m->cols() != dest.cols()))
                throw std::runtime_error("localMatrix: shape mismatch " LOCATION);
            const u64 n = dest.size();
            const u64 bytes = n * sizeof(i64);
            auto addend = std::make_shared<DeviceBuffer>();
            if (m && n) {
                addend->reset(g, bytes);
                toDevice(addend->data(), m->data(), bytes, g);
            }
            // a row slice: the whole matrix's draws are taken, the slice's used
            const u64 all = totalRows ? totalRows * dest.cols() : n;
            aby3g_zero_share zs = mShareGen.zeroShare(mShareGen.takeDraws(all) + rowOffset * dest.cols());
            GPU_CALL(aby3g_share_draws(kind, zs.k_prev, zs.k_next, zs.draw_base, n,
                                       m ? addend->as<i64>() : nullptr, dest.share(0), nullptr, g.stream()));
            comm.mNext.asyncSendDevice(dest.share(0), bytes, g);
            auto fu = comm.mPrev.asyncRecvDevice(dest.share(1), bytes, g);
            self.then([fu, addend](CommPkg&, Sh3Task&) { fu.get(); });
        })
        .getClosure();
}

Sh3Task Sh3Encryptor::localIntMatrix(Sh3Task dep, const i64Matrix& m, si64Matrix& dest) {
    return shareImpl(dep, &m, dest, ABY3G_DRAW_ARITH);
}
Sh3Task Sh3Encryptor::remoteIntMatrix(Sh3Task dep, si64Matrix& dest) {
    return shareImpl(dep, nullptr, dest, ABY3G_DRAW_ARITH);
}
Sh3Task Sh3Encryptor::localIntMatrixRows(Sh3Task dep, const i64Matrix& m, si64Matrix& dest, u64 rowOffset,
                                         u64 totalRows) {
    return shareImpl(dep, &m, dest, ABY3G_DRAW_ARITH, rowOffset, totalRows);
}
Sh3Task Sh3Encryptor::remoteIntMatrixRows(Sh3Task dep, si64Matrix& dest, u64 rowOffset, u64 totalRows) {
    return shareImpl(dep, nullptr, dest, ABY3G_DRAW_ARITH, rowOffset, totalRows);
}
Sh3Task Sh3Encryptor::localBinMatrix(Sh3Task dep, const i64Matrix& m, sbMatrix& dest) {
    return shareImpl(dep, &m, dest, ABY3G_DRAW_BIN);
}
Sh3Task Sh3Encryptor::remoteBinMatrix(Sh3Task dep, sbMatrix& dest) {
    return shareImpl(dep, nullptr, dest, ABY3G_DRAW_BIN);
}

Sh3Task Sh3Encryptor::localFixedMatrix(Sh3Task dep, const std::vector<double>& m, u64 rows, u64 cols, u64 D,
                                       si64Matrix& dest) {
    auto im = std::make_shared<i64Matrix>(rows, cols);
    for (u64 i = 0; i < rows * cols; ++i) (*im)(i) = toFixed(m[i], D);
    // keep the scaled copy alive until the sharing task has run
    return shareImpl(dep, im.get(), dest, ABY3G_DRAW_ARITH).then([im](Sh3Task&) {});
}

Sh3Task Sh3Encryptor::revealImpl(Sh3Task dep, const SharedMat& x, i64Matrix& dest, bool binary) {
    return dep.then([&x, &dest, binary](CommPkg& comm, Sh3Task& self) {
        Gpu& g = self.getRuntime().gpu();
        const u64 n = x.size();
        DeviceBuffer other(g, n * sizeof(i64)), sum(g, n * sizeof(i64));
        comm.mNext.asyncRecvDevice(other.data(), n * sizeof(i64), g).get();
        if (binary) {
            GPU_CALL(aby3g_u64_bitop(0, n, (const u64*)x.share(0), (const u64*)x.share(1), sum.as<u64>(), g.stream()));
            GPU_CALL(aby3g_u64_bitop(0, n, sum.as<u64>(), other.as<u64>(), sum.as<u64>(), g.stream()));
        } else {
            GPU_CALL(aby3g_i64_lincomb(n, 1, x.share(0), 1, x.share(1), 0, sum.as<i64>(), g.stream()));
            GPU_CALL(aby3g_i64_lincomb(n, 1, sum.as<i64>(), 1, other.as<i64>(), 0, sum.as<i64>(), g.stream()));
        }
        dest.resize(x.rows(), x.cols());
        toHost(dest.data(), sum.data(), n * sizeof(i64), g);
    });
}

Sh3Task Sh3Encryptor::revealSend(Sh3Task dep, u64 partyIdx, const SharedMat& x) {
    const bool send = ((mPartyIdx + 2) % 3) == partyIdx;
    return dep.then([send, &x](CommPkg& comm, Sh3Task& self) {
        if (send) comm.mPrev.asyncSendDevice(x.share(0), x.size() * sizeof(i64), self.getRuntime().gpu());
    });
}

Sh3Task Sh3Encryptor::reveal(Sh3Task dep, const si64Matrix& x, i64Matrix& dest) {
    return revealImpl(dep, x, dest, false);
}
Sh3Task Sh3Encryptor::reveal(Sh3Task dep, const sbMatrix& x, i64Matrix& dest) { return revealImpl(dep, x, dest, true); }
Sh3Task Sh3Encryptor::reveal(Sh3Task dep, u64 partyIdx, const si64Matrix& x) { return revealSend(dep, partyIdx, x); }
Sh3Task Sh3Encryptor::reveal(Sh3Task dep, u64 partyIdx, const sbMatrix& x) { return revealSend(dep, partyIdx, x); }

Sh3Task Sh3Encryptor::revealAll(Sh3Task dep, const si64Matrix& x, i64Matrix& dest) {
    revealSend(dep, (mPartyIdx + 2) % 3, x);
    return revealImpl(dep, x, dest, false);
}
Sh3Task Sh3Encryptor::revealAll(Sh3Task dep, const sbMatrix& x, i64Matrix& dest) {
    revealSend(dep, (mPartyIdx + 2) % 3, x);
    return revealImpl(dep, x, dest, true);
}

}  // namespace aby3
