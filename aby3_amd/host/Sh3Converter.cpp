#include "Sh3Converter.h"
#include <cstring>

namespace aby3 {

namespace {

aby3g_stream_pos streamPos(const block& seed, u64 off) {
    aby3g_stream_pos p;
    std::memcpy(p.seed, seed.data(), 16);
    p.off = off;
    return p;
}

u64 lastWordMask(u64 bitCount) { return bitCount % 64 ? (1ull << (bitCount % 64)) - 1 : ~0ull; }

}  // namespace

void Sh3Converter::init(Sh3Runtime& rt, Sh3ShareGen& gen) {
    mRandGen = &gen;
    // mOT12.mIdx = mOT02.mIdx = party (Sh3Converter.h:28-29); setSeed resets to 0
    mOT12Idx = mOT02Idx = rt.mPartyIdx;
    switch (rt.mPartyIdx) {
        case 0:
            mOT02Key = gen.getPrevBlock();
            mOT02Idx = 0;
            break;
        case 1:
            mOT12Key = gen.getNextBlock();
            mOT12Idx = 0;
            break;
        case 2:
            mOT12Key = gen.getPrevBlock();
            mOT02Key = gen.getNextBlock();
            mOT12Idx = mOT02Idx = 0;
            break;
        default:
            throw RTE_LOC;
    }
}

const u32* Sh3Converter::wireIds(u64 bitCount, Gpu& g) {
    if (mIotaCount < bitCount || mIota.gpu() != &g) {
        std::vector<u32> ids(bitCount);
        for (u64 i = 0; i < bitCount; ++i) ids[i] = (u32)i;
        mIota.reset(g, bitCount * sizeof(u32));
        toDevice(mIota.data(), ids.data(), bitCount * sizeof(u32), g);
        mIotaCount = bitCount;
    }
    return mIota.as<u32>();
}

void Sh3Converter::toPackedBin(const sbMatrix& in, sPackedBin& dest) {
    dest.reset(in.rows(), in.bitCount());
    if (!in.rows() || !in.bitCount()) return;
    if (in.bitCount() > 0xffffffffull) throw std::runtime_error("toPackedBin: bitCount exceeds 2^32 " LOCATION);
    Gpu& g = Gpu::current();
    GPU_CALL(aby3g_bits_to_wires2(in.data(), in.rows(), in.cols(), (u32)in.bitCount(), (uint64_t*)dest.data(),
                                  dest.size(), dest.simdWidth(), g.stream()));
}

void Sh3Converter::toBinaryMatrix(const sPackedBin& in, sbMatrix& dest) {
    dest.resize(in.shareCount(), in.bitCount());
    if (!in.bitCount() || !in.shareCount()) return;
    if (in.bitCount() > 0xffffffffull) throw std::runtime_error("toBinaryMatrix: bitCount exceeds 2^32 " LOCATION);
    Gpu& g = Gpu::current();
    GPU_CALL(aby3g_wires_to_bits2((const uint64_t*)in.data(), in.size(), wireIds(in.bitCount(), g),
                                  (u32)in.bitCount(), in.simdWidth(), dest.data(), dest.rows(), g.stream()));
}

void Sh3Converter::buildArithToBinCircuit(BetaCircuit& cir, u64 base, u64 bitCount) {
    if (!base || !bitCount) throw std::runtime_error("getArithToBinCircuit: empty " LOCATION);
    const BetaBundle in0 = cir.addInputBundle((u32)bitCount), in1 = cir.addInputBundle((u32)bitCount);
    BetaBundle out;
    out.reserve(bitCount);
    const u64 numWords = (base + bitCount - 1) / base;
    for (u64 i = 0; i < numWords; ++i) {
        const u64 begin = i * base, end = std::min<u64>(begin + base, bitCount);
        BetaBundle a(in0.begin() + begin, in0.begin() + end), b(in1.begin() + begin, in1.begin() + end);
        BetaBundle s = circuits::add(cir, a, b, false);  // add_build(..., Optimized::Depth)
        out.insert(out.end(), s.begin(), s.end());
    }
    cir.addOutputBundle(out);
}

BetaCircuit Sh3Converter::getArithToBinCircuit(u64 base, u64 bitCount) {
    BetaCircuit cir;
    buildArithToBinCircuit(cir, base, bitCount);
    cir.levelByAndDepth();
    return cir;
}

BetaCircuit* Sh3Converter::arithToBinCircuit(u64 bitCount) {
    auto& c = mA2B[bitCount];
    if (!c) {
        c = std::make_unique<BetaCircuit>();
        buildArithToBinCircuit(*c, 64, bitCount);
        c->levelByAndDepth();
    }
    return c.get();
}

Sh3Task Sh3Converter::toBinaryMatrix(Sh3Task dep, const si64Matrix& in, sbMatrix& dest) {
    struct State {
        sbMatrix x0, x1;
    };
    auto state = std::make_shared<State>();
    return dep
        .then([this, &in, &dest, state](CommPkg& comm, Sh3Task& self) {
            const u64 p = self.getRuntime().mPartyIdx;
            if (p > 2) throw std::runtime_error("logic error. " LOCATION);
            if (!mRandGen) throw std::runtime_error("init was not called. " LOCATION);
            Gpu& g = self.getRuntime().gpu();
            aby3g_stream st = g.stream();
            if (dest.rows() == 0) dest.resize(in.rows(), 64 * in.cols());
            const u64 bits = dest.bitCount();
            sbMatrix& x0 = state->x0;  // = in.0 + in.2, reshared by P0
            sbMatrix& x1 = state->x1;  // = in.1
            x0.resize(in.rows(), bits);
            x1.resize(in.rows(), bits);
            // the reference indexes x and in flat (:90-93)
            if (x0.size() != in.size() || dest.rows() != in.rows())
                throw std::runtime_error("toBinaryMatrix: dest must be in.rows() x 64 * in.cols() " LOCATION);
            const u64 n = x0.size(), b8 = n * sizeof(i64), cols64 = x0.cols(), mask = lastWordMask(bits);
            if (n) switch (p) {
                    case 0: {  // (:74-113) x0 = ((in0 + in1) ^ r, r), x1 = 0
                        aby3g_stream_pos pv = streamPos(mRandGen->mPrevSeed, mRandGen->takePrev(b8));
                        GPU_CALL(aby3g_a2b_reshare(&pv, n, cols64, mask, in.share(0), in.share(1), 1, x0.share(0),
                                                   x0.share(1), st));
                        GPU_CALL(aby3g_memset(x1.data(), 0, 2 * b8, st));
                        comm.mNext.asyncSendDevice(x0.share(0), b8, g);
                        break;
                    }
                    case 1: {  // (:115-159) x0 = (0, P0's message), x1 = (in0, 0)
                        GPU_CALL(aby3g_memset(x0.share(0), 0, b8, st));
                        GPU_CALL(aby3g_memset(x1.share(1), 0, b8, st));
                        GPU_CALL(aby3g_a2b_reshare(nullptr, n, cols64, mask, in.share(0), nullptr, 0, x1.share(0),
                                                   nullptr, st));
                        auto f = comm.mPrev.asyncRecvDevice(x0.share(1), b8, g);
                        self.then([f](CommPkg&, Sh3Task&) { f.get(); });
                        break;
                    }
                    case 2: {  // (:160-199) x0 = (r, 0), x1 = (0, in1)
                        aby3g_stream_pos nx = streamPos(mRandGen->mNextSeed, mRandGen->takeNext(b8));
                        GPU_CALL(aby3g_a2b_reshare(&nx, n, cols64, mask, nullptr, nullptr, 0, nullptr, x0.share(0),
                                                   st));
                        GPU_CALL(aby3g_memset(x0.share(1), 0, b8, st));
                        GPU_CALL(aby3g_memset(x1.share(0), 0, b8, st));
                        GPU_CALL(aby3g_a2b_reshare(nullptr, n, cols64, mask, in.share(1), nullptr, 0, x1.share(1),
                                                   nullptr, st));
                        break;
                    }
                }
            if (!n || !bits) return;
            BetaCircuit* cir = arithToBinCircuit(bits);
            mBin.asyncEvaluate(self, cir, *mRandGen, {&x0, &x1}, {&dest}).then([state](Sh3Task&) {});
        })
        .getClosure();
}

Sh3Task Sh3Converter::bitInjection(Sh3Task dep, const sbMatrix& in, si64Matrix& dest, bool twoRounds) {
    return dep
        .then([this, &in, &dest, twoRounds](CommPkg& comm, Sh3Task& self) {
            if (!mRandGen) throw std::runtime_error("init was not called. " LOCATION);
            Gpu& g = self.getRuntime().gpu();
            aby3g_stream st = g.stream();
            const u64 rows = in.rows(), bits = in.bitCount(), cols64 = in.cols();
            const u64 n = rows * bits, b8 = n * sizeof(i64);
            dest.resize(rows, bits);
            if (!n) return;  // same on every party: no messages
            switch (self.getRuntime().mPartyIdx) {
                case 0: {  // receiver of mOT12, helper of mOT02 (:236-276)
                    auto fs = comm.mPrev.asyncRecvShared(2 * b8, g);  // P2's messages, read in place
                    auto fh = comm.mNext.asyncRecvShared(b8, g);      // P1's pads
                    self.then([fs, fh, &in, &dest, twoRounds, rows, cols64, bits, b8](CommPkg& comm2, Sh3Task& s2) {
                        Gpu& g2 = s2.getRuntime().gpu();
                        auto m = fs.getShared(), h = fh.getShared();
                        GPU_CALL(aby3g_ot_recv_bits(m->as<i64>(), h->as<i64>(), in.share(0), rows, cols64, bits,
                                                    dest.share(0), g2.stream()));
                        m->fence(g2.stream());
                        h->fence(g2.stream());
                        if (twoRounds) comm2.mNext.asyncSendDevice(dest.share(0), b8, g2);
                    });
                    if (!twoRounds) {
                        auto help = std::make_shared<DeviceBuffer>(g, b8);
                        GPU_CALL(aby3g_ot_help_bits(in.share(0), rows, cols64, bits, mOT02Key.data(), mOT02Idx,
                                                    help->as<i64>(), st));
                        mOT02Idx += n;
                        comm.mNext.asyncSendShared(help, b8, g);
                    }
                    GPU_CALL(aby3g_prng_fill(mRandGen->mPrevSeed.data(), mRandGen->takePrev(b8), b8, dest.share(1),
                                             st));
                    break;
                }
                case 1: {  // helper of mOT12, receiver of mOT02 (:278-318)
                    auto help = std::make_shared<DeviceBuffer>(g, b8);
                    GPU_CALL(aby3g_ot_help_bits(in.share(1), rows, cols64, bits, mOT12Key.data(), mOT12Idx,
                                                help->as<i64>(), st));
                    mOT12Idx += n;
                    comm.mPrev.asyncSendShared(help, b8, g);
                    GPU_CALL(aby3g_prng_fill(mRandGen->mNextSeed.data(), mRandGen->takeNext(b8), b8, dest.share(0),
                                             st));
                    if (!twoRounds) {
                        auto fs = comm.mNext.asyncRecvShared(2 * b8, g);
                        auto fh = comm.mPrev.asyncRecvShared(b8, g);
                        self.then([fs, fh, &in, &dest, rows, cols64, bits](CommPkg&, Sh3Task& s2) {
                            aby3g_stream st2 = s2.getRuntime().gpu().stream();
                            auto m = fs.getShared(), h = fh.getShared();
                            GPU_CALL(aby3g_ot_recv_bits(m->as<i64>(), h->as<i64>(), in.share(1), rows, cols64, bits,
                                                        dest.share(1), st2));
                            m->fence(st2);
                            h->fence(st2);
                        });
                    } else {
                        auto f = comm.mPrev.asyncRecvDevice(dest.share(1), b8, g);
                        self.then([f](CommPkg&, Sh3Task&) { f.get(); });
                    }
                    break;
                }
                case 2: {  // sender of both OTs (:319-363), one launch
                    auto ma = std::make_shared<DeviceBuffer>(g, 2 * b8);
                    std::shared_ptr<DeviceBuffer> mb;
                    if (!twoRounds) mb = std::make_shared<DeviceBuffer>(g, 2 * b8);
                    aby3g_stream_pos nx = streamPos(mRandGen->mNextSeed, mRandGen->takeNext(b8));
                    aby3g_stream_pos pv = streamPos(mRandGen->mPrevSeed, mRandGen->takePrev(b8));
                    GPU_CALL(aby3g_bitinj_send(in.data(), rows, cols64, bits, &nx, &pv, mOT12Key.data(), mOT12Idx,
                                               mOT02Key.data(), mOT02Idx, dest.data(), ma->as<i64>(),
                                               mb ? mb->as<i64>() : nullptr, st));
                    mOT12Idx += n;
                    comm.mNext.asyncSendShared(ma, 2 * b8, g);
                    if (mb) {
                        mOT02Idx += n;
                        comm.mPrev.asyncSendShared(mb, 2 * b8, g);
                    }
                    break;
                }
                default:
                    throw std::runtime_error("logic error");
            }
        })
        .getClosure();
}

}  // namespace aby3
