#include "Sh3BinaryEvaluator.h"
#include <cstring>
#include <map>
#include <mutex>

namespace aby3 {

// defaults of the binary engine's fused forms (A/B-measured)
constexpr bool kFuseInputsDefault = true;

void Sh3BinaryEvaluator::setCir(BetaCircuit* cir, u64 width, Sh3ShareGen& gen) {
    block p = gen.getPrevBlock();
    block n = gen.getNextBlock();
    setCirImpl(cir, width, p, n, 0, 0);
}

void Sh3BinaryEvaluator::setCir(BetaCircuit* cir, u64 width, block prevSeed, block nextSeed) {
    setCirImpl(cir, width, prevSeed, nextSeed, 0, 0);
}

void Sh3BinaryEvaluator::setCirRows(BetaCircuit* cir, u64 width, Sh3ShareGen& gen, u64 rowOffset, u64 totalRows) {
    if (rowOffset % 2048 || rowOffset + width > totalRows || (width % 2048 && rowOffset + width != totalRows))
        throw std::invalid_argument("setCirRows: rows [" + std::to_string(rowOffset) + ", " +
                                    std::to_string(rowOffset + width) + ") of " + std::to_string(totalRows) +
                                    ": the slice must start at a multiple of 2048 rows and end at one or at the "
                                    "last row " LOCATION);
    block p = gen.getPrevBlock();
    block n = gen.getNextBlock();
    setCirImpl(cir, width, p, n, rowOffset / 64, 32 * ((totalRows + 2047) / 2048));
}

void Sh3BinaryEvaluator::upload(Gpu& g) {
    const BetaCircuit& c = *mCir;
    // key: circuit serial (unique per levelized form), tagged to stay clear of other attachment kinds
    const u64 key = (c.serial() << 8) | 0x01;
    mCur = std::static_pointer_cast<DevCircuit>(g.attachment(key, [&]() -> std::shared_ptr<void> {
        auto d = std::make_shared<DevCircuit>();
        std::vector<u8> host;
        auto put = [&](const void* p, size_t bytes) {
            const size_t off = (host.size() + 15) / 16 * 16;
            host.resize(off + bytes);
            if (bytes) std::memcpy(host.data() + off, p, bytes);
            return off;
        };
        std::vector<aby3g_gate> gs(c.mBatchGates.size());
        for (size_t i = 0; i < gs.size(); ++i) {
            const BetaGate& b = c.mBatchGates[i];
            gs[i] = aby3g_gate{b.in0, b.in1, b.out, (u32)b.type, c.mBatchZRow[i], c.mBatchSendRow[i]};
        }
        const size_t oGates = put(gs.data(), gs.size() * sizeof(aby3g_gate));
        // per gate, the recv row of each input that the previous level's AND
        // outputs deliver (its share 1 is read from the received buffer)
        std::vector<u32> rr(2 * gs.size(), ~0u);
        {
            size_t lg = 0, first = 0;  // level-list index / batch-order index of the level's first gate
            std::map<u32, u32> prevAnd, curAnd;
            for (size_t L = 0; L < c.mLevelCounts.size(); ++L) {
                curAnd.clear();
                for (u32 k = 0; k < c.mLevelCounts[L]; ++k) {
                    const BetaGate& lgate = c.mLevelGates[lg + k];
                    if (isAndType(lgate.type)) {
                        const u32 row = (u32)curAnd.size();
                        curAnd[lgate.out] = row;
                    }
                }
                for (u32 k = 0; k < c.mLevelCounts[L]; ++k) {
                    const BetaGate& b = c.mBatchGates[first + k];
                    auto a0 = prevAnd.find(b.in0), a1 = prevAnd.find(b.in1);
                    if (a0 != prevAnd.end()) rr[2 * (first + k)] = a0->second;
                    if (a1 != prevAnd.end()) rr[2 * (first + k) + 1] = a1->second;
                }
                lg += c.mLevelCounts[L];
                first += c.mLevelCounts[L];
                prevAnd.swap(curAnd);
            }
        }
        const size_t oRr = put(rr.data(), rr.size() * 4);
        std::vector<u32> ends;
        for (const auto& batches : c.mLevelBatches) {
            d->levelFirstGate.push_back(batches.empty() ? 0 : batches.front().begin);
            d->levelBatchOffset.push_back((u32)ends.size());
            d->levelBatches.push_back((u32)batches.size());
            for (const auto& b : batches) ends.push_back(b.begin + b.count - d->levelFirstGate.back());
        }
        const size_t oEnds = put(ends.data(), ends.size() * 4);
        // per level, the AND outputs in level-list order = send/recv row order
        std::vector<size_t> oLevel;
        size_t gi = 0;
        for (size_t L = 0; L < c.mLevelCounts.size(); ++L) {
            std::vector<u32> v;
            for (u32 k = 0; k < c.mLevelCounts[L]; ++k, ++gi)
                if (isAndType(c.mLevelGates[gi].type)) v.push_back(c.mLevelGates[gi].out);
            oLevel.push_back(put(v.data(), v.size() * 4));
        }
        std::vector<u32> all;
        for (auto& o : c.mOutputs) {
            d->outputOffsets.push_back((u32)all.size());
            all.insert(all.end(), o.begin(), o.end());
        }
        const size_t oOut = put(all.data(), all.size() * 4);
        for (size_t L = 0; L <= c.mLevelCounts.size(); ++L)
            if ((L < c.mLevelCounts.size() && !c.mLevelBatches[L].empty()) || (L > 0 && c.mLevelAndCounts[L - 1]))
                d->lastLaunchLevel = L;
        // fused first level: the inputs' wire range, and who else reads them
        if (!c.mInputs.empty() && !c.mLevelCounts.empty()) {
            u32 lo = ~0u, hi = 0;
            for (const auto& in : c.mInputs)
                for (u32 w : in) lo = std::min(lo, w), hi = std::max(hi, w + 1);
            if (lo < hi && hi - lo <= ABY3G_LEVEL_IN_MAX_WIRES) {
                d->fuseInputs = true;
                d->inLo = lo;
                d->inHi = hi;
                auto isIn = [&](u32 w) { return w >= lo && w < hi; };
                for (size_t k = c.mLevelCounts[0]; k < c.mLevelGates.size() && !d->inputsReadLater; ++k)
                    d->inputsReadLater = isIn(c.mLevelGates[k].in0) || isIn(c.mLevelGates[k].in1);
                for (u32 w : all) d->inputsReadLater = d->inputsReadLater || isIn(w);
            }
        }
        d->blob.reset(g, host.size() ? host.size() : 16);
        if (!host.empty()) toDevice(d->blob.data(), host.data(), host.size(), g);
        u8* base = d->blob.as<u8>();
        d->gates = reinterpret_cast<const aby3g_gate*>(base + oGates);
        d->recvRows = reinterpret_cast<const u32*>(base + oRr);
        d->batchEnds = reinterpret_cast<const u32*>(base + oEnds);
        for (size_t o : oLevel) d->outWires.push_back(reinterpret_cast<const u32*>(base + o));
        d->allOutputWires = reinterpret_cast<const u32*>(base + oOut);
        return d;
    }));
}

void Sh3BinaryEvaluator::setCirImpl(BetaCircuit* cir, u64 width, block prevSeed, block nextSeed, u64 wordOffset,
                                    u64 rowStride) {
    if (!cir->levelized()) cir->levelByAndDepth();
    mCir = cir;
    mRows = width;
    mWords = 32 * ((width + 2047) / 2048);
    mLevel = 0;
    mKeyPrev = prevSeed;
    mKeyNext = nextSeed;
    mPendingIn.clear();  // held inputs belong to the previous circuit
    mPendingHold.clear();
    Gpu& g = Gpu::current();
    mGpu = &g;
    upload(g);
    const u64 memBytes = 2 * (u64)cir->mWireCount * mWords * 8;
    if (mMem.bytes() < memBytes || mMem.gpu() != &g) mMem.reset(g, memBytes ? memBytes : 8);
    // all AND masks of the circuit: z[k][w] = binary draw k*words + w, drawn on
    // another stream while the inputs are transposed on the main one
    if (mZPending) waitZ();  // setCir again before evaluating: the old draw lands first
    releaseZ();
    mSendAll.reset();
    mArenaLease.reset();
    mPerLevelSends = false;
    mAndDone = 0;
    mZByLevel = false;
    mZDrawn = 0;
    // (a whole evaluation is the slice of itself: the contiguous draws)
    mZWordOffset = rowStride == mWords ? 0 : wordOffset;
    mZRowStride = rowStride == mWords ? 0 : rowStride;
    const u64 zWords = (u64)cir->mAndCount * mWords;
    if (zWords) {
        mZStream = g.drawStream() ? g.drawStream() : g.aux();
        const bool other = mZStream != g.stream();
        auto ring = std::static_pointer_cast<ZRing>(
            g.attachment(0x2a02, [] { return std::static_pointer_cast<void>(std::make_shared<ZRing>()); }));
        mRing = ring;
        ZRing& r = *ring;
        r.stream = g.stream();
        int b = -1;
        for (int k = 0; k < 2 && b < 0; ++k)
            if (!r.busy[(r.next + k) % 2]) b = (r.next + k) % 2;
        bool fresh = true;
        if (b >= 0) {
            r.next = (b + 1) % 2;
            r.busy[b] = true;
            mZSlot = b;
            if (r.buf[b].bytes() < zWords * 8 || r.buf[b].gpu() != &g) {
                r.buf[b].reset(g, zWords * 8);
                r.recorded[b] = false;
            }
            fresh = !r.recorded[b];
            if (!fresh && other) GPU_CALL(aby3g_stream_wait_event(mZStream, r.done[b]->get()));
            mZPtr = r.buf[b].as<u64>();
        } else {
            // both ring buffers held by evaluations not yet evaluated
            if (mZ.bytes() < zWords * 8 || mZ.gpu() != &g) mZ.reset(g, zWords * 8);
            mZPtr = mZ.as<u64>();
        }
        if (fresh && other) {
            // memory from the main stream's pool: the draws wait for the main stream
            if (!mZFresh) mZFresh = std::make_unique<Event>();
            mZFresh->record(g.stream());
            GPU_CALL(aby3g_stream_wait_event(mZStream, mZFresh->get()));
        }
        mZByLevel = !other && levelDraws() != 0;
        if (mZByLevel)
            drawZThrough(0);  // the first AND level's masks; the rest in roundCallback (levelDraws)
        else
            drawZRows(0, cir->mAndCount);
        if (other) {
            if (!mZEv) mZEv = std::make_unique<Event>();
            mZEv->record(mZStream);
        }
        mZPending = true;
    }
}

// Where a party alone on its stream draws an evaluation's masks
// (ABY3_LEVEL_DRAWS, A/B runs): 0 all in setCir; 1 the first AND level's in
// setCir, each later level's behind the launch before it; 2 (default) the
// first AND level's in setCir, all the others behind its launch. Three party
// processes on one GPU, same box: C3 0.3326-0.3367 ms with 2, 0.3455-0.3499
// with 1, 0.3526-0.3541 with 0; C5 64.8-65.4 / 68.3-68.6 / 65.2-65.9 ms (one
// more launch per level costs the sort's many small evaluations more than
// it hides).
int Sh3BinaryEvaluator::levelDraws() {
    static const int mode = [] {
        const char* e = getenv("ABY3_LEVEL_DRAWS");
        return e && *e ? atoi(e) : 2;
    }();
    return mode;
}

void Sh3BinaryEvaluator::drawZThrough(u64 level) {
    // masks of the AND gates of levels 0 .. L, where L is the first level at
    // or after `level` with AND gates (z rows are AND ordinals in level order)
    const auto& c = mCir->mLevelAndCounts;
    u64 end = 0, L = 0;
    for (; L < c.size() && (L < level || !c[L]); ++L) end += c[L];
    if (L < c.size()) end += c[L];
    if (end <= mZDrawn) return;
    drawZRows(mZDrawn, end);
    mZDrawn = end;
}

void Sh3BinaryEvaluator::drawZRows(u64 first, u64 end) {
    if (end <= first) return;
    if (mZRowStride)  // a row slice: words [offset, offset + mWords) of each AND row
        GPU_CALL(aby3g_share_draws_rows(ABY3G_DRAW_BIN, mKeyPrev.data(), mKeyNext.data(),
                                        first * mZRowStride + mZWordOffset, mWords, mZRowStride, end - first,
                                        (i64*)(mZPtr + first * mWords), mZStream));
    else
        GPU_CALL(aby3g_share_draws(ABY3G_DRAW_BIN, mKeyPrev.data(), mKeyNext.data(), first * mWords,
                                   (end - first) * mWords, nullptr, (i64*)(mZPtr + first * mWords), nullptr,
                                   mZStream));
}

void Sh3BinaryEvaluator::waitZ() {
    if (mZPending && mZEv && mZStream != mGpu->stream()) GPU_CALL(aby3g_stream_wait_event(mGpu->stream(), mZEv->get()));
    mZPending = false;
}

void Sh3BinaryEvaluator::releaseZ() {
    auto ring = mRing.lock();
    if (mZSlot < 0 || !ring) {
        mZSlot = -1;
        return;
    }
    ZRing& r = *ring;
    if (!r.done[mZSlot]) r.done[mZSlot] = std::make_unique<Event>();
    r.done[mZSlot]->record(r.stream);
    r.recorded[mZSlot] = true;
    r.busy[mZSlot] = false;
    mZSlot = -1;
}

void Sh3BinaryEvaluator::setInput(u64 i, const sbMatrix& in) {
    if (!mCir) throw RTE_LOC;
    if (i >= mCir->mInputs.size()) throw std::invalid_argument("input index out of bounds");
    const auto& wires = mCir->mInputs[i];
    if (in.bitCount() != wires.size()) throw std::invalid_argument("input data wrong size");
    if (in.rows() != mRows) throw std::invalid_argument("incorrect number of rows");
    for (size_t k = 1; k < wires.size(); ++k)
        if (wires[k] != wires[k - 1] + 1) throw std::runtime_error("expecting contiguous input wires. " LOCATION);
    Gpu& g = *mGpu;
    const u64 W = mCir->mWireCount;
    GPU_CALL(aby3g_bits_to_wires2(in.data(), mRows, in.i64Cols(), (u32)wires.size(), mMem.as<u64>() + wires[0] * mWords,
                                  W * mWords, mWords, g.stream()));
    mLevel = 0;
}

void Sh3BinaryEvaluator::setInput(u64 i, const sbMatrix& in, const aby3g_rowmap& map) {
    if (!mCir) throw RTE_LOC;
    if (i >= mCir->mInputs.size()) throw std::invalid_argument("input index out of bounds");
    const auto& wires = mCir->mInputs[i];
    if (in.bitCount() != wires.size()) throw std::invalid_argument("input data wrong size");
    for (size_t k = 1; k < wires.size(); ++k)
        if (wires[k] != wires[k - 1] + 1) throw std::runtime_error("expecting contiguous input wires. " LOCATION);
    Gpu& g = *mGpu;
    const u64 W = mCir->mWireCount;
    GPU_CALL(aby3g_bits_to_wires_map(in.data(), in.rows(), in.i64Cols(), (u32)wires.size(), &map, mRows,
                                     mMem.as<u64>() + wires[0] * mWords, W * mWords, mWords, g.stream()));
    mLevel = 0;
}

void Sh3BinaryEvaluator::setInputs(u64 i, const aby3g_rowmap& mi, u64 j, const aby3g_rowmap& mj,
                                   const sbMatrix& in) {
    if (!mCir) throw RTE_LOC;
    if (i >= mCir->mInputs.size() || j >= mCir->mInputs.size()) throw std::invalid_argument("input index out of bounds");
    const auto& wi = mCir->mInputs[i];
    const auto& wj = mCir->mInputs[j];
    if (in.bitCount() != wi.size() || in.bitCount() != wj.size()) throw std::invalid_argument("input data wrong size");
    for (const auto* wires : {&wi, &wj})
        for (size_t k = 1; k < wires->size(); ++k)
            if ((*wires)[k] != (*wires)[k - 1] + 1) throw std::runtime_error("expecting contiguous input wires. " LOCATION);
    Gpu& g = *mGpu;
    const u64 W = mCir->mWireCount;
    const aby3g_rowmap maps[2] = {mi, mj};
    u64* dst[2] = {mMem.as<u64>() + wi[0] * mWords, mMem.as<u64>() + wj[0] * mWords};
    GPU_CALL(aby3g_bits_to_wires_map_n(in.data(), in.rows(), in.i64Cols(), (u32)wi.size(), maps, dst, 2, mRows,
                                       W * mWords, mWords, g.stream()));
    mLevel = 0;
}

// ABY3_FUSE_INPUTS=1 / 0 turns the fused first level on / off (A/B runs)
static bool fuseInputsEnabled() {
    static const bool on = [] {
        const char* e = getenv("ABY3_FUSE_INPUTS");
        return e ? e[0] == '1' : kFuseInputsDefault;
    }();
    return on;
}

void Sh3BinaryEvaluator::flushPendingInputs(bool dropHolds) {
    if (mPendingIn.empty()) return;
    GPU_CALL(aby3g_bits_to_wires_lin(mPendingIn.data(), (u32)mPendingIn.size(), mRows, mWords, mGpu->stream()));
    mPendingIn.clear();
    readHeld(dropHolds);
}

void Sh3BinaryEvaluator::holdForInputs(std::shared_ptr<DeviceBuffer> b) {
    if (b) mPendingHold.push_back(std::move(b));
}

void Sh3BinaryEvaluator::readHeld(bool drop) {
    // the launch that reads the held sources is enqueued: fence each buffer
    // behind it (a no-op for this party's own pool, reused in stream order)
    for (auto& b : mPendingHold) b->fence(mGpu->stream());
    if (drop) mPendingHold.clear();
}

bool Sh3BinaryEvaluator::pendingCoversInputs() const {
    if (mPendingIn.empty()) return false;
    const u64 W = mCir->mWireCount, stride = W * mWords;
    const u32 n = mCur->inHi - mCur->inLo;
    std::vector<u8> have(2 * (size_t)n, 0);
    for (const auto& src : mPendingIn) {
        const u64 off = (u64)(src.wire_rows - mMem.as<u64>());
        const u64 sh = off / stride, w = (off % stride) / mWords;
        for (u64 b = 0; b < src.nbits; ++b)
            if (w + b >= mCur->inLo && w + b < mCur->inHi) have[2 * (w + b - mCur->inLo) + sh] = 1;
    }
    for (const auto& in : mCir->mInputs)
        for (u32 w : in)
            if (!have[2 * (w - mCur->inLo)] || !have[2 * (w - mCur->inLo) + 1]) return false;
    return true;
}

void Sh3BinaryEvaluator::setInputs(const std::vector<WireInput>& in) {
    if (!mCir) throw RTE_LOC;
    Gpu& g = *mGpu;
    const u64 W = mCir->mWireCount;
    std::vector<aby3g_wire_src> srcs;
    // Held for the first level's launch when the circuit allows it and every
    // source is one 64-bit column: the copy-outs (a message, e.g. P0's
    // reshared value) are made now, the transposes inside that launch.
    bool defer = fuseInputsEnabled() && mCur->fuseInputs;
    for (const WireInput& w : in) {
        if (w.input >= mCir->mInputs.size() || mCir->mInputs[w.input].size() > 64) defer = false;
        // a constant without terms: the separate transpose applies it, the fused level does not
        if (!w.term[0] && !w.term[1] && !w.term[2] && !w.term[3] && w.constant) defer = false;
    }
    auto flush = [&] {
        if (srcs.empty()) return;
        if (defer) {
            GPU_CALL(aby3g_lin_copy_out(srcs.data(), (u32)srcs.size(), mRows, g.stream()));
            for (auto& s : srcs) {
                if (s.copy_out) {
                    // the level reads the copy (one term) instead of its terms again
                    s.term[0] = s.copy_out;
                    s.coef[0] = 1;
                    for (int t = 1; t < 4; ++t) s.term[t] = nullptr, s.coef[t] = 0;
                }
                s.copy_out = nullptr;
                if (mPendingIn.size() == ABY3G_WIRE_SRC_MAX) flushPendingInputs(false);  // more sources follow
                mPendingIn.push_back(s);
            }
        } else {
            GPU_CALL(aby3g_bits_to_wires_lin(srcs.data(), (u32)srcs.size(), mRows, mWords, g.stream()));
        }
        srcs.clear();
    };
    for (const WireInput& w : in) {
        if (w.input >= mCir->mInputs.size()) throw std::invalid_argument("input index out of bounds");
        if (w.share < 0 || w.share > 1) throw std::invalid_argument("share index");
        const auto& wires = mCir->mInputs[w.input];
        for (size_t k = 1; k < wires.size(); ++k)
            if (wires[k] != wires[k - 1] + 1) throw std::runtime_error("expecting contiguous input wires. " LOCATION);
        aby3g_wire_src s{};
        for (int t = 0; t < 4; ++t) {
            s.term[t] = w.term[t];
            s.coef[t] = w.coef[t];
        }
        s.constant = w.constant;
        s.cols64 = (wires.size() + 63) / 64;
        s.nbits = (u32)wires.size();
        s.wire_rows = mMem.as<u64>() + ((u64)w.share * W + wires[0]) * mWords;
        s.copy_out = w.copyOut;
        srcs.push_back(s);
        if (srcs.size() == ABY3G_WIRE_SRC_MAX) flush();
    }
    flush();
    // transposed now (not held for the first level): the buffers the terms
    // read are fenced behind that launch and released
    if (mPendingIn.empty()) readHeld(true);
    mLevel = 0;
}

void setTwoInputSharing(Sh3BinaryEvaluator& eng, int pIdx, const std::vector<std::pair<const si64Matrix*, i64>>& x,
                        i64 sign, const std::vector<u64>& in0, const std::vector<i64>& offsets, u64 in1, CommPkg& comm,
                        Gpu& g) {
    if (x.empty() || x.size() > 2 || in0.size() != offsets.size()) throw std::invalid_argument("setTwoInputSharing");
    const u64 n = x[0].first->size(), b8 = n * sizeof(i64);
    for (auto& t : x)
        if (t.first->size() != n) throw std::invalid_argument("setTwoInputSharing: shapes");
    using WI = Sh3BinaryEvaluator::WireInput;
    std::vector<WI> w;
    auto zero = [&](u64 input, int share) {
        WI z;
        z.input = input;
        z.share = share;
        w.push_back(z);
    };
    // sum over the terms of share s of x (times c)
    auto xshare = [&](WI& d, int s, i64 c, int at) {
        for (auto& t : x) {
            d.term[at] = t.first->share(s);
            d.coef[at++] = (i64)((u64)c * (u64)t.second);
        }
        return at;
    };
    std::shared_ptr<DeviceBuffer> v;
    if (pIdx == 0) {
        // in0 = (sign (x0 + x2) + off, 0); the share itself goes to P1
        v = std::make_shared<DeviceBuffer>(g, b8);
        for (size_t k = 0; k < in0.size(); ++k) {
            WI d;
            d.input = in0[k];
            d.share = 0;
            xshare(d, 1, sign, xshare(d, 0, sign, 0));
            d.constant = offsets[k];
            if (k == 0) d.copyOut = v->as<i64>();
            w.push_back(d);
            zero(in0[k], 1);
        }
        zero(in1, 0);
        zero(in1, 1);
        // the first level may read the copy-out v later (fused inputs): keep
        // it out of the pool until that launch is enqueued
        eng.holdForInputs(v);
        eng.setInputs(w);
        comm.mNext.asyncSendShared(v, b8, g);
    } else if (pIdx == 1) {
        // in0 = (0, sign (x0 + x2) + off) received from P0, in1 = (x1, 0)
        WI d1;
        d1.input = in1;
        d1.share = 0;
        xshare(d1, 0, 1, 0);
        w.push_back(d1);
        zero(in1, 1);
        v = comm.mPrev.asyncRecvShared(b8, g).getShared();
        for (size_t k = 0; k < in0.size(); ++k) {
            zero(in0[k], 0);
            WI d;
            d.input = in0[k];
            d.share = 1;
            d.term[0] = v->as<i64>();
            d.coef[0] = 1;
            d.constant = offsets[k];
            w.push_back(d);
        }
        // v is P0's buffer, read in place by the first level's launch (fused
        // inputs, enqueued later in roundCallback) or by the transpose now:
        // held until that launch is enqueued, then fenced behind it
        eng.holdForInputs(v);
        eng.setInputs(w);
    } else {
        // in0 = (0, 0), in1 = (0, x1)
        for (size_t k = 0; k < in0.size(); ++k) {
            zero(in0[k], 0);
            zero(in0[k], 1);
        }
        zero(in1, 0);
        WI d1;
        d1.input = in1;
        d1.share = 1;
        xshare(d1, 1, 1, 0);
        w.push_back(d1);
        eng.setInputs(w);
    }
}

void Sh3BinaryEvaluator::setReplicatedInput(u64 i, const sbMatrix& in) {
    if (!mCir) throw RTE_LOC;
    if (i >= mCir->mInputs.size()) throw std::invalid_argument("input index out of bounds");
    const auto& wires = mCir->mInputs[i];
    if (in.bitCount() != wires.size()) throw std::invalid_argument("input data wrong size");
    if (in.rows() != 1) throw std::invalid_argument("incorrect number of simd rows");
    Gpu& g = *mGpu;
    const u64 W = mCir->mWireCount;
    for (int s = 0; s < 2; ++s) {
        // every row of wire j takes bit j of the single input row: all-zero or all-one words
        const std::vector<i64> row = in.shareToHost(s);
        for (size_t j = 0; j < wires.size(); ++j) {
            const int v = ((u64)row[j / 64] >> (j % 64)) & 1 ? 0xff : 0;
            GPU_CALL(aby3g_memset(mMem.as<u64>() + ((u64)s * W + wires[j]) * mWords, v, mWords * 8, g.stream()));
        }
    }
    mLevel = 0;
}

// ABY3_LEVEL_SLOTS=0: a level's sends between processes without an arena
// are staged copies out of one evaluation buffer (A/B runs)
static bool levelSlotSends() {
    static const bool on = [] {
        const char* e = getenv("ABY3_LEVEL_SLOTS");
        return !e || e[0] != '0';
    }();
    return on;
}

void Sh3BinaryEvaluator::roundCallback(CommPkg& comm, Sh3Task task) {
    if (mLevel > mCir->mLevelCounts.size())
        throw std::runtime_error("evaluateRound() was called but no rounds remain... " LOCATION);
    Gpu& g = task.getRuntime().gpu();
    const u64 W = mCir->mWireCount;
    const u64 rowBytes = mWords * 8;
    // share 1 of last level's AND outputs arrived from prev (:555-573); they
    // are unpacked, straight from the sender's buffer, by the same launch that
    // runs this level's gates
    // Co-located parties hand the AND shares over inside the level kernels
    // (aby3g_handoff): this launch waits, per 2048-row workgroup, for the
    // previous party's same rows and publishes its own send rows for the next
    // party -- no stream operation between the parties' streams. Otherwise
    // the channel enqueues a stream wait here and the flags stay null.
    u32 nUnpack = 0;
    std::shared_ptr<DeviceBuffer> recv;
    aby3g_handoff hw{nullptr, 0, nullptr}, hp{nullptr, 0, nullptr};
    if (mLevel) {
        nUnpack = mCir->mLevelAndCounts[mLevel - 1];
        if (nUnpack) recv = mRecvFutr.getSharedHandoff(hw);
    }
    const bool gatesHere = mLevel < mCir->mLevelCounts.size();
    const u32 nb = gatesHere ? mCur->levelBatches[mLevel] : 0;
    const u32 nAnd = gatesHere ? mCir->mLevelAndCounts[mLevel] : 0;
    if (mLevel == 0 && mAndDone) {  // evaluated again after setCir: a fresh send buffer
        mSendAll.reset();
        mArenaLease.reset();
        mPerLevelSends = false;
        mAndDone = 0;
    }
    std::shared_ptr<DeviceBuffer> send;
    if (nAnd) {
        if (!mSendAll && !mPerLevelSends) {
            // the evaluation's first AND level: between processes on one GPU
            // its messages live in the channel's IPC-mapped arena, read in
            // place by the receiver; between processes without an arena each
            // level's AND shares are produced straight into a staging slot of
            // the link (no staging copy); else one buffer of this party
            u64 andLevels = 0;
            for (u32 c : mCir->mLevelAndCounts) andLevels += c != 0;
            mSendAll = comm.mNext.evalSendBuffer(g, (u64)mCir->mAndCount * rowBytes, andLevels, &mArenaLease);
            if (!mSendAll) {
                if (comm.mNext.linked() && levelSlotSends())
                    mPerLevelSends = true;
                else
                    mSendAll = std::make_shared<DeviceBuffer>(g, (u64)mCir->mAndCount * rowBytes);
            }
        }
        send = mPerLevelSends ? comm.mNext.linkSendBuffer(g, nAnd * rowBytes)
                              : DeviceBuffer::view(mSendAll, mAndDone * rowBytes, nAnd * rowBytes);
    }
    mAndDone += nAnd;
    // this level's bytes (about 72 per gate and 64-row word)
    if (nAnd) hp = comm.mNext.handoffPost(g, mRows, (u64)mCir->mLevelCounts[mLevel] * mWords * 72, send->data());
    if (nAnd && mZByLevel) drawZThrough(mLevel);  // (normally drawn already, behind an earlier launch)
    if (nb && mZPending) waitZ();
    // the first level with its inputs (aby3g_bin_level_in) when the held
    // sources make up every input wire (an input set another way lives in
    // mMem, which the fused launch does not read for input wires)
    const bool fused = mLevel == 0 && nb && pendingCoversInputs();
    if (!fused) flushPendingInputs();
    if (fused) {
        GPU_CALL(aby3g_bin_level_in(mPendingIn.data(), (u32)mPendingIn.size(), mRows, mCur->inLo, mCur->inHi,
                                    mCur->inputsReadLater ? 1 : 0, mCur->gates + mCur->levelFirstGate[0],
                                    mCur->batchEnds + mCur->levelBatchOffset[0], nb, mMem.as<u64>(), W, mWords, mZPtr,
                                    send ? send->as<u64>() : nullptr, &hp, g.stream()));
        mPendingIn.clear();
        readHeld(true);
    } else if (nb || nUnpack) {
        const aby3g_gate* gl = nb ? mCur->gates + mCur->levelFirstGate[mLevel] : nullptr;
        const u32* be = nb ? mCur->batchEnds + mCur->levelBatchOffset[mLevel] : nullptr;
        const u32* rr = (nb && recv) ? mCur->recvRows + 2 * (u64)mCur->levelFirstGate[mLevel] : nullptr;
        GPU_CALL(aby3g_bin_level_hs(gl, rr, be, nb, recv ? recv->as<u64>() : nullptr,
                                    nUnpack ? mCur->outWires[mLevel - 1] : nullptr, nUnpack, mMem.as<u64>(), W, mWords,
                                    mZPtr, send ? send->as<u64>() : nullptr, &hw, &hp, g.stream()));
    }

    if (recv) {
        // views of one sender buffer: fenced after the last of them is read
        bool last = true;
        for (size_t L = mLevel; L < mCir->mLevelAndCounts.size() && last; ++L) last = mCir->mLevelAndCounts[L] == 0;
        if (last) recv->fence(g.stream());
    }
    if (nAnd) {
        comm.mNext.asyncSendShared(send, nAnd * rowBytes, g, hp);
        mRecvFutr = comm.mPrev.asyncRecvShared(nAnd * rowBytes, g);
        // the evaluation's last message is sent: the arena may serve the next one
        if (mAndDone == mCir->mAndCount) mArenaLease.reset();
    }
    // a party alone on its stream: the later levels' masks run here, after
    // this level's send, while the peers' messages for the next level are
    // still in flight, instead of all in front of the first level
    if (mZByLevel) drawZThrough(levelDraws() == 2 ? mCir->mLevelAndCounts.size() : mLevel + 1);
    ++mLevel;
    if (hasMoreRounds()) task.then([this](CommPkg& c, Sh3Task& t) { roundCallback(c, t); }, "callback");
}

Sh3Task Sh3BinaryEvaluator::asyncEvaluate(Sh3Task dep) {
    return dep.then([this](CommPkg& comm, Sh3Task& self) { roundCallback(comm, self); }, "bin-eval-closure")
        .getClosure();
}

Sh3Task Sh3BinaryEvaluator::asyncEvaluate(Sh3Task dep, BetaCircuit* cir, Sh3ShareGen& gen,
                                          std::vector<const sbMatrix*> inputs, std::vector<sbMatrix*> outputs) {
    if (cir->mInputs.size() != inputs.size() || cir->mOutputs.size() != outputs.size()) throw RTE_LOC;
    return dep
        .then([this, cir, &gen, inputs](CommPkg& comm, Sh3Task& self) {
            const u64 width = inputs[0]->rows();
            setCir(cir, width, gen);
            for (size_t i = 0; i < inputs.size(); ++i) {
                if (inputs[i]->rows() != width) throw RTE_LOC;
                setInput(i, *inputs[i]);
            }
            roundCallback(comm, self);
        })
        .getClosure()
        .then([this, outputs](Sh3Task&) {
            for (size_t i = 0; i < outputs.size(); ++i) getOutput(i, *outputs[i]);
        });
}

void Sh3BinaryEvaluator::getOutput(u64 i, sbMatrix& out) {
    if (i >= mCir->mOutputs.size()) throw RTE_LOC;
    const auto& wires = mCir->mOutputs[i];
    out.resize(mRows, wires.size());
    Gpu& g = *mGpu;
    const u64 W = mCir->mWireCount;
    const u32* dw = mCur->allOutputWires + mCur->outputOffsets[i];
    GPU_CALL(aby3g_wires_to_bits2(mMem.as<u64>(), W * mWords, dw, (u32)wires.size(), mWords, out.data(), mRows,
                                  g.stream()));
}

void Sh3BinaryEvaluator::getOutputs(u64 i, const aby3g_rowmap& mi, u64 j, const aby3g_rowmap& mj, sbMatrix& out) {
    if (i >= mCir->mOutputs.size() || j >= mCir->mOutputs.size()) throw RTE_LOC;
    if (out.bitCount() != mCir->mOutputs[i].size() || out.bitCount() != mCir->mOutputs[j].size())
        throw std::invalid_argument("output matrix wrong size");
    Gpu& g = *mGpu;
    const u64 W = mCir->mWireCount;
    const u32* dw[2] = {mCur->allOutputWires + mCur->outputOffsets[i], mCur->allOutputWires + mCur->outputOffsets[j]};
    const aby3g_rowmap maps[2] = {mi, mj};
    GPU_CALL(aby3g_wires_to_bits_map_n(mMem.as<u64>(), W * mWords, dw, (u32)out.bitCount(), mWords, out.data(),
                                       out.rows(), maps, 2, mRows, g.stream()));
}

void Sh3BinaryEvaluator::getOutput(u64 i, sbMatrix& out, const aby3g_rowmap& map) {
    if (i >= mCir->mOutputs.size()) throw RTE_LOC;
    const auto& wires = mCir->mOutputs[i];
    if (out.bitCount() != wires.size()) throw std::invalid_argument("output matrix wrong size");
    Gpu& g = *mGpu;
    const u64 W = mCir->mWireCount;
    const u32* dw = mCur->allOutputWires + mCur->outputOffsets[i];
    GPU_CALL(aby3g_wires_to_bits_map(mMem.as<u64>(), W * mWords, dw, (u32)wires.size(), mWords, out.data(), out.rows(),
                                     &map, mRows, g.stream()));
}

}  // namespace aby3
