#include "Sh3Evaluator.h"

namespace aby3 {

void Sh3Evaluator::init(u64 partyIdx, block prevSeed, block nextSeed) {
    mShareGen.init(prevSeed, nextSeed);
    mPartyIdx = partyIdx;
    mOtPrevKey = mShareGen.getNextBlock();  // mOtPrevRecver.setSeed(mNextCommon.get<block>())
    mOtNextKey = mShareGen.getPrevBlock();  // mOtNextRecver.setSeed(mPrevCommon.get<block>())
    mOtPrevIdx = mOtNextIdx = 0;
}

void Sh3Evaluator::init(u64 partyIdx, CommPkg& comm, block seed) {
    mShareGen.init(comm, seed);
    mPartyIdx = partyIdx;
    mOtPrevKey = mShareGen.getNextBlock();
    mOtNextKey = mShareGen.getPrevBlock();
    mOtPrevIdx = mOtNextIdx = 0;
}

void Sh3Evaluator::shape(MulMode mode, const si64Matrix& A, const si64Matrix& B, u64& M, u64& K, u64& N) const {
    if (mode == MulMode::Gemm) {
        if (A.cols() != B.rows()) throw std::runtime_error("asyncMul: inner dimensions differ " LOCATION);
        M = A.rows();
        K = A.cols();
        N = B.cols();
    } else {
        if (A.rows() != B.rows() || A.cols() != B.cols())
            throw std::runtime_error("asyncMul (Hadamard): shapes differ " LOCATION);
        M = A.rows();
        K = N = A.cols();
    }
}

void* Sh3Evaluator::workspace(MulMode mode, u64 M, u64 K, u64 N, size_t& bytes, Gpu& g) {
    bytes = aby3g_mul_workspace_bytes((int)mode, M, K, N);
    if (!bytes) return nullptr;
    if (mWs.bytes() < bytes || mWs.gpu() != &g) mWs.reset(g, bytes);
    bytes = mWs.bytes();
    return mWs.data();
}

Sh3Task Sh3Evaluator::asyncMul(Sh3Task dep, const si64Matrix& A, const si64Matrix& B, si64Matrix& C) {
    return asyncMul(dep, A, B, C, mMulMode);
}

// C's storage overlaps an operand's (C = A * B with C == A, say): the
// reference evaluates the product into an Eigen temporary before assigning,
// so the product goes to a private matrix that replaces C once complete.
static bool aliases(const SharedMat& C, const SharedMat& X) {
    if (&C == &X) return true;
    if (C.empty() || X.empty()) return false;
    const char *c = (const char*)C.data(), *x = (const char*)X.data();
    return c < x + 2 * X.size() * sizeof(i64) && x < c + 2 * C.size() * sizeof(i64);
}

Sh3Task Sh3Evaluator::asyncMul(Sh3Task dep, const si64Matrix& A, const si64Matrix& B, si64Matrix& C, MulMode mode) {
    return dep
        .then([this, &A, &B, &C, mode](CommPkg& comm, Sh3Task& self) {
            Gpu& g = self.getRuntime().gpu();
            u64 M, K, N;
            shape(mode, A, B, M, K, N);
            std::shared_ptr<si64Matrix> tmp;
            if (aliases(C, A) || aliases(C, B)) tmp = std::make_shared<si64Matrix>();
            si64Matrix& out = tmp ? *tmp : C;
            out.resize(M, N);
            const u64 n = M * N;
            size_t wsBytes = 0;
            void* ws = workspace(mode, M, K, N, wsBytes, g);
            // C0 = share product + getShare() per element (Sh3Evaluator.cpp:101-105)
            aby3g_zero_share zs = mShareGen.zeroShare(mShareGen.takeDraws(n));
            GPU_CALL(aby3g_mul_local((int)mode, A.data(), B.data(), out.share(0), M, K, N,
                                     DEBUG_disable_randomization ? nullptr : &zs, ws, wsBytes, g.stream()));
            comm.mNext.asyncSendDevice(out.share(0), n * sizeof(i64), g);
            auto fu = comm.mPrev.asyncRecvDevice(out.share(1), n * sizeof(i64), g);
            si64Matrix* caller = &C;
            self.then([fu, tmp, caller](CommPkg&, Sh3Task&) {
                fu.get();
                if (tmp) *caller = std::move(*tmp);
            });
        })
        .getClosure();
}

TruncationPair Sh3Evaluator::getTruncationTuple(u64 rows, u64 cols, u64 d) {
    Gpu& g = Gpu::current();
    TruncationPair p;
    p.rows = rows;
    p.cols = cols;
    const u64 n = rows * cols;
    p.mR.reset(g, n * sizeof(i64));
    p.mRTrunc.resize(rows, cols);
    if (DEBUG_disable_randomization) {
        GPU_CALL(aby3g_memset(p.mR.data(), 0, n * sizeof(i64), g.stream()));
        p.mRTrunc.setZero();
        return p;
    }
    aby3g_trunc_streams ts;
    std::memcpy(ts.next_seed, mShareGen.mNextSeed.data(), 16);
    std::memcpy(ts.prev_seed, mShareGen.mPrevSeed.data(), 16);
    ts.next_off = mShareGen.takeNext(8 * n);
    ts.prev_off = mShareGen.takePrev(8 * n);
    GPU_CALL(aby3g_trunc_tuple(&ts, n, (unsigned)d, p.mR.as<i64>(), p.mRTrunc.data(), g.stream()));
    return p;
}

Sh3Task Sh3Evaluator::asyncMul(Sh3Task dep, const si64Matrix& A, const si64Matrix& B, si64Matrix& C, u64 shift) {
    return asyncMul(dep, A, B, C, shift, mMulMode);
}

Sh3Task Sh3Evaluator::asyncMul(Sh3Task dep, const si64Matrix& A, const si64Matrix& B, si64Matrix& C, u64 shift,
                               MulMode mode) {
    return mulTrunc(dep, A, B, C, shift, mode, 0, 0);
}

Sh3Task Sh3Evaluator::asyncMulRows(Sh3Task dep, const si64Matrix& A, const si64Matrix& B, si64Matrix& C, u64 shift,
                                   u64 rowOffset, u64 totalRows) {
    if (!totalRows || rowOffset + A.rows() > totalRows)
        throw std::invalid_argument("asyncMulRows: rows [" + std::to_string(rowOffset) + ", " +
                                    std::to_string(rowOffset + A.rows()) + ") of a " + std::to_string(totalRows) +
                                    "-row product " LOCATION);
    return mulTrunc(dep, A, B, C, shift, MulMode::Gemm, rowOffset, totalRows);
}

Sh3Task Sh3Evaluator::mulTrunc(Sh3Task dep, const si64Matrix& A, const si64Matrix& B, si64Matrix& C, u64 shift,
                               MulMode mode, u64 rowOffset, u64 totalRows) {
    return dep
        .then([this, &A, &B, &Cref = C, shift, mode, rowOffset, totalRows](CommPkg& comm, Sh3Task& self) {
            Gpu& g = self.getRuntime().gpu();
            u64 M, K, N;
            shape(mode, A, B, M, K, N);
            const u64 n = M * N, bytes = n * sizeof(i64);
            // a row slice takes the whole product's truncation words and uses
            // its rows' (the words are row-major: row r starts at word r * N)
            const u64 allWords = totalRows ? totalRows * N : n, skip = rowOffset * N;
            std::shared_ptr<si64Matrix> tmp;
            if (aliases(Cref, A) || aliases(Cref, B)) tmp = std::make_shared<si64Matrix>();
            si64Matrix& C = tmp ? *tmp : Cref;
            C.resize(M, N);
            // z = product - r is revealed to P0 and P1 zero-copy: the buffer
            // itself is the message (Channel::asyncSendShared); between
            // processes it is produced straight into a staging slot of the
            // first channel it goes to (linkSendBuffer: no staging copy)
            const u64 pIdx = self.getRuntime().mPartyIdx;
            const bool toNext = (pIdx + 1) % 3 < 2;
            auto z = (toNext ? comm.mNext : comm.mPrev).linkSendBuffer(g, bytes);
            size_t wsBytes = 0;
            void* ws = workspace(mode, M, K, N, wsBytes, g);
            if (DEBUG_disable_randomization) {
                // zero truncation pair: z = product, C = 0
                GPU_CALL(aby3g_mul_local((int)mode, A.data(), B.data(), z->as<i64>(), M, K, N, nullptr, ws, wsBytes,
                                         g.stream()));
                C.setZero();
            } else {
                // round 1 (Sh3Evaluator.cpp:658-673): z = product - r, C = RT
                aby3g_trunc_streams ts;
                std::memcpy(ts.next_seed, mShareGen.mNextSeed.data(), 16);
                std::memcpy(ts.prev_seed, mShareGen.mPrevSeed.data(), 16);
                ts.next_off = mShareGen.takeNext(8 * allWords) + 8 * skip;
                ts.prev_off = mShareGen.takePrev(8 * allWords) + 8 * skip;
                // The truncation pair's AES-CTR runs in the product's epilogue
                // pass (k_finish_trunc): the element-wise / small-GEMM epilogue,
                // or, after a share GEMM, the pass that reads its product (or
                // reduces its split-K slabs) and writes z = product - R, RT.
                // (Drawing the pair first on the auxiliary stream, with the
                // GEMM's epilogue subtracting R, measured slower for C2.)
                GPU_CALL(aby3g_mul_trunc_local((int)mode, A.data(), B.data(), M, K, N, (unsigned)shift, &ts,
                                               z->as<i64>(), C.data(), ws, wsBytes, g.stream()));
            }
            // reveal z to parties 0 and 1 (:681-684)
            const u64 p = self.getRuntime().mPartyIdx;
            const u64 next = (p + 1) % 3, prev = (p + 2) % 3;
            if (next < 2) comm.mNext.asyncSendSharedEvent(z, bytes, g);  // z's own channel first (toNext)
            if (prev < 2) comm.mPrev.asyncSendSharedEvent(z, bytes, g);
            if (p < 2) {
                auto fu0 = comm.mNext.asyncRecvShared(bytes, g);
                auto fu1 = comm.mPrev.asyncRecvShared(bytes, g);
                // round 2 (:703-719): C[p] += (z0 + z1 + z2) >> d
                si64Matrix* dst = &C;     // the product (C itself or the private matrix)
                si64Matrix* caller = &Cref;  // the caller's C (outlives the task)
                self.then([z, fu0, fu1, dst, caller, tmp, shift, p, n](CommPkg&, Sh3Task& self2) {
                    Gpu& g2 = self2.getRuntime().gpu();
                    auto zn = fu0.getShared();
                    auto zp = fu1.getShared();
                    GPU_CALL(aby3g_trunc_finalize((int)p, zn->as<i64>(), zp->as<i64>(), z->as<i64>(), (unsigned)shift,
                                                  dst->data(), n, g2.stream()));
                    zn->fence(g2.stream());
                    zp->fence(g2.stream());
                    if (tmp) *caller = std::move(*tmp);
                });
            } else if (tmp) {
                Cref = std::move(*tmp);
            }
        })
        .getClosure();
}

Sh3Task Sh3Evaluator::asyncMul(Sh3Task dep, const si64Matrix& A, const sbMatrix& B, si64Matrix& C) {
    return dep
        .then([this, &A, &B, &C](CommPkg& comm, Sh3Task& self) {
            Gpu& g = self.getRuntime().gpu();
            if (A.cols() != 1 || B.rows() != A.rows() || B.bitCount() != 1)
                throw std::runtime_error("asyncMul(si64, sb): expects n x 1 and a 1-bit sbMatrix " LOCATION);
            const u64 n = A.rows(), b8 = n * sizeof(i64);
            // A may alias C (Sh3Piecewise.cpp:300-304): keep a private copy of A
            auto a = std::make_shared<si64Matrix>();
            a->copyFrom(A);
            C.resize(n, 1);
            switch (self.getRuntime().mPartyIdx) {
                case 0: {  // OT sender for P1 (with P2 helping), helper for P2's send (:132-163)
                    // the OT messages go zero-copy: P1 reads these buffers in place
                    auto send = std::make_shared<DeviceBuffer>(g, 2 * b8);
                    auto help = std::make_shared<DeviceBuffer>(g, b8);
                    aby3g_stream_pos pv, nx;
                    std::memcpy(pv.seed, mShareGen.mPrevSeed.data(), 16);
                    pv.off = mShareGen.takePrev(16 * n);
                    std::memcpy(nx.seed, mShareGen.mNextSeed.data(), 16);
                    nx.off = mShareGen.takeNext(8 * n);
                    GPU_CALL(aby3g_bitmul_p0(a->data(), B.data(), n, &pv, &nx, mOtNextKey.data(), mOtNextIdx,
                                             C.data(), send->as<i64>(), help->as<i64>(), g.stream()));
                    mOtNextIdx += 2 * n;
                    comm.mNext.asyncSendShared(send, 2 * b8, g);
                    comm.mNext.asyncSendShared(help, b8, g);
                    break;
                }
                case 1: {  // receiver (:165-200)
                    GPU_CALL(aby3g_prng_fill(mShareGen.mPrevSeed.data(), mShareGen.takePrev(8 * n), 8 * n,
                                             C.share(1), g.stream()));
                    // f0 = (sender prev, helper next), f1 = (sender next, helper prev);
                    // all four are read in place from the senders' buffers
                    auto f0s = comm.mPrev.asyncRecvShared(2 * b8, g);
                    auto f0h = comm.mNext.asyncRecvShared(b8, g);
                    auto f1s = comm.mNext.asyncRecvShared(2 * b8, g);
                    auto f1h = comm.mPrev.asyncRecvShared(b8, g);
                    self.then([f0s, f0h, f1s, f1h, &B, &C, n, b8](CommPkg& comm2, Sh3Task& s2) {
                        Gpu& g2 = s2.getRuntime().gpu();
                        auto m0 = f0s.getShared(), h0 = f0h.getShared(), m1 = f1s.getShared(), h1 = f1h.getShared();
                        // c0 = recv1 (choice b1 = B[1]) + recv0 (choice b0 = B[0])
                        GPU_CALL(aby3g_ot_recv(m1->as<i64>(), h1->as<i64>(), B.share(1), n, 0, C.share(0),
                                               g2.stream()));
                        GPU_CALL(aby3g_ot_recv(m0->as<i64>(), h0->as<i64>(), B.share(0), n, 1, C.share(0),
                                               g2.stream()));
                        for (auto* b : {&m0, &h0, &m1, &h1}) (*b)->fence(g2.stream());
                        comm2.mNext.asyncSendDevice(C.share(0), b8, g2);
                    });
                    break;
                }
                case 2: {  // OT sender for P1 (with P0 helping), helper for P0's send (:202-240)
                    auto send = std::make_shared<DeviceBuffer>(g, 2 * b8);
                    auto help = std::make_shared<DeviceBuffer>(g, b8);
                    aby3g_stream_pos nx;
                    std::memcpy(nx.seed, mShareGen.mNextSeed.data(), 16);
                    nx.off = mShareGen.takeNext(16 * n);
                    GPU_CALL(aby3g_bitmul_p2(a->data(), B.data(), n, &nx, mOtPrevKey.data(), mOtPrevIdx, C.data(),
                                             help->as<i64>(), send->as<i64>(), g.stream()));
                    mOtPrevIdx += 2 * n;
                    comm.mPrev.asyncSendShared(help, b8, g);
                    comm.mPrev.asyncSendShared(send, 2 * b8, g);
                    self.then([&C, b8](CommPkg& comm2, Sh3Task& s2) {
                        auto f = comm2.mPrev.asyncRecvDevice(C.share(1), b8, s2.getRuntime().gpu());
                        s2.then([f](CommPkg&, Sh3Task&) { f.get(); });
                    });
                    break;
                }
                default:
                    throw RTE_LOC;
            }
            self.then([a](Sh3Task&) {});  // A's copy lives until the product is done
        })
        .getClosure();
}

Sh3Task Sh3Evaluator::asyncMul(Sh3Task dep, i64 a, const sbMatrix& B, si64Matrix& C) {
    return asyncMul(dep, a, B, C, mShareGen);
}

Sh3Task Sh3Evaluator::asyncMul(Sh3Task dep, i64 a, const sbMatrix& B, si64Matrix& C, Sh3ShareGen& zeroGen) {
    return dep
        .then([this, a, &B, &C, &zeroGen](CommPkg& comm, Sh3Task& self) {
            Gpu& g = self.getRuntime().gpu();
            if (B.bitCount() != 1) throw RTE_LOC;
            const u64 n = B.rows(), b8 = n * sizeof(i64);
            C.resize(n, 1);
            switch (self.getRuntime().mPartyIdx) {
                case 0: {  // (:430-447)
                    auto mn = std::make_shared<DeviceBuffer>(g, 2 * b8);
                    auto mp = std::make_shared<DeviceBuffer>(g, 2 * b8);
                    aby3g_zero_share zs = zeroGen.zeroShare(zeroGen.takeDraws(n));
                    GPU_CALL(aby3g_pubmul_p0(a, B.data(), n, &zs, mOtNextKey.data(), mOtNextIdx, mOtPrevKey.data(),
                                             mOtPrevIdx, mn->as<i64>(), mp->as<i64>(), g.stream()));
                    mOtNextIdx += n;
                    mOtPrevIdx += n;
                    comm.mNext.asyncSendShared(mn, 2 * b8, g);
                    comm.mPrev.asyncSendShared(mp, 2 * b8, g);
                    auto fu1 = comm.mNext.asyncRecvDevice(C.share(0), b8, g);
                    auto fu2 = comm.mPrev.asyncRecvDevice(C.share(1), b8, g);
                    self.then([fu1, fu2](CommPkg&, Sh3Task&) {
                        fu1.get();
                        fu2.get();
                    });
                    break;
                }
                case 1:
                case 2: {  // (:452-487)
                    const bool p1 = self.getRuntime().mPartyIdx == 1;
                    auto help = std::make_shared<DeviceBuffer>(g, b8);
                    aby3g_zero_share zs = zeroGen.zeroShare(zeroGen.takeDraws(n));
                    i64* mine = p1 ? C.share(1) : C.share(0);
                    const u8* key = p1 ? mOtNextKey.data() : mOtPrevKey.data();
                    u64& ctr = p1 ? mOtNextIdx : mOtPrevIdx;
                    GPU_CALL(aby3g_pubmul_helper(p1 ? B.share(0) : B.share(1), n, &zs, key, ctr, mine,
                                                 help->as<i64>(), g.stream()));
                    ctr += n;
                    Channel& toHelped = p1 ? comm.mNext : comm.mPrev;   // the other receiver
                    Channel& toSender = p1 ? comm.mPrev : comm.mNext;   // party 0
                    toHelped.asyncSendShared(help, b8, g);
                    toSender.asyncSendDevice(mine, b8, g);
                    // the OT messages and the helper's pads are read in place
                    auto fs = toSender.asyncRecvShared(2 * b8, g);
                    auto fh = toHelped.asyncRecvShared(b8, g);
                    i64* theirs = p1 ? C.share(0) : C.share(1);
                    const i64* choice = p1 ? B.share(0) : B.share(1);
                    self.then([fs, fh, theirs, choice, n](CommPkg&, Sh3Task& s2) {
                        auto msgs = fs.getShared(), hm = fh.getShared();
                        aby3g_stream st = s2.getRuntime().gpu().stream();
                        GPU_CALL(aby3g_ot_recv(msgs->as<i64>(), hm->as<i64>(), choice, n, 0, theirs, st));
                        msgs->fence(st);
                        hm->fence(st);
                    });
                    break;
                }
                default:
                    throw RTE_LOC;
            }
        })
        .getClosure();
}

}  // namespace aby3
