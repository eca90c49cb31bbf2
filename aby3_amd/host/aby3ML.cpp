#include "aby3ML.h"
#include <algorithm>
#include <iterator>
#include <unordered_map>
#include <cmath>
#include <cstring>
#include <random>
#include <thread>

namespace aby3 {

void aby3ML::mul(const si64Matrix& left, const si64Matrix& right, si64Matrix& dest) {
    mEval.asyncMul(mRt.noDependencies(), left, right, dest, mD, MulMode::Gemm).get();
}

void aby3ML::mulTruncate(const si64Matrix& left, const si64Matrix& right, si64Matrix& dest, u64 shift) {
    mEval.asyncMul(mRt.noDependencies(), left, right, dest, mD + shift, MulMode::Gemm).get();
}

Sh3Piecewise& aby3ML::logistic() {
    if (mLogistic.mThresholds.empty()) {
        mLogistic.mThresholds = {Sh3Piecewise::Coef(-0.5), Sh3Piecewise::Coef(0.5)};
        mLogistic.mCoefficients.resize(3);
        mLogistic.mCoefficients[1] = {Sh3Piecewise::Coef(0.5), Sh3Piecewise::Coef(1)};
        mLogistic.mCoefficients[2] = {Sh3Piecewise::Coef(1)};
    }
    return mLogistic;
}

void aby3ML::logisticFunc(const si64Matrix& Y, si64Matrix& out) {
    logistic().eval(mRt.noDependencies(), Y, out, mD, mEval).get();
}

// ---- the fused iteration (aby3g_lr_iteration) ------------------------------
// One launch per party and iteration. The host side keeps the op-by-op
// path's bookkeeping exactly -- every stream offset, zero-share draw, OT
// counter and setCir key is taken here in the order that path takes them --
// so the kernel reproduces its shares bit for bit.
struct FusedLr {
    CircuitLibrary lib;        // the same int_Sh3Piecewise_helper(64, 2) as Sh3Piecewise builds
    DeviceBuffer circuit;      // levelized gate list (aby3g_lr_circuit arrays)
    aby3g_lr_circuit cir{};
    DeviceBuffer scratch, mailbox;
    const void* nextBox = nullptr;
    const void* prevBox = nullptr;
    // one party per process: this party's mailbox is a raw allocation exported
    // through IPC, the neighbours' are IPC mappings
    void* ownBox = nullptr;
    void* mapped[2] = {nullptr, nullptr};
    int device = 0;
    bool sysScope = false;
    u64 epoch = 0;
    u64 d = 0, B = 0;
    aby3g_lr_rand pred{};   // the next iteration's randomness as predicted by the last step
    bool havePred = false;
    i64 thrOff[2] = {0, 0}, half = 0, slope = 0, one = 0;

    ~FusedLr() {
        if (!ownBox && !mapped[0] && !mapped[1]) return;
        // at teardown: every party's last iteration has completed (a session
        // drains its stream before it ends), and a neighbour's IPC mapping
        // keeps this allocation alive until it closes it
        aby3g_set_device(device);
        aby3g_device_sync();
        for (void* m : mapped)
            if (m) aby3g_ipc_close(m);
        if (ownBox) aby3g_free(ownBox);
    }

    // The fused form applies to the logistic piecewise of aby3ML (regions
    // {}, {c, integer slope}, {c}) with randomization on, B <= 2048 rows, and
    // a ring whose parties' kernels may poll each other's memory: co-located
    // parties of one process (Channel::handoffCapable), or one party per
    // process (Channel::linkedConcurrent; the mailboxes exchanged as IPC
    // handles, on one GPU or across GPUs). Every party decides alike.
    static std::shared_ptr<FusedLr> make(aby3ML& ml, u64 d, u64 B) {
        Gpu& g = ml.mRt.gpu();
        CommPkg& comm = ml.mRt.mComm;
        const bool local = comm.mNext.handoffCapable(g) && comm.mPrev.handoffCapable(g);
        const bool linked = !local && comm.mNext.linkedConcurrent() && comm.mPrev.linkedConcurrent();
        if (!local && !linked) return nullptr;
        if (ml.mEval.DEBUG_disable_randomization || B == 0 || B > 2048 || d == 0 || d > 4096) return nullptr;
        Sh3Piecewise& pw = ml.logistic();
        const auto& co = pw.mCoefficients;
        if (pw.mThresholds.size() != 2 || co.size() != 3 || !co[0].empty() || co[1].size() != 2 ||
            !co[1][1].mIsInteger || co[2].size() != 1)
            return nullptr;
        auto f = std::make_shared<FusedLr>();
        f->d = d;
        f->B = B;
        f->device = g.device();
        for (int t = 0; t < 2; ++t) f->thrOff[t] = (i64)(0 - (u64)pw.mThresholds[t].getFixedPoint(ml.mD));
        f->half = co[1][0].getFixedPoint(ml.mD);
        f->slope = co[1][1].getInteger();
        f->one = co[2][0].getFixedPoint(ml.mD);
        f->upload(g);
        const u64 mb = aby3g_lr_mailbox_bytes((u32)B, (u32)d, &f->cir);
        f->scratch.reset(g, aby3g_lr_scratch_bytes((u32)B, (u32)d, &f->cir));
        if (local) {
            f->mailbox.reset(g, mb);
            // zeroed before any peer can poll it: the address leaves only after
            // this stream has drained the memset
            GPU_CALL(aby3g_memset(f->mailbox.data(), 0, mb, g.stream()));
            g.sync();
            const u64 mine = (u64)(uintptr_t)f->mailbox.data();
            comm.mNext.asyncSendCopy(mine);
            comm.mPrev.asyncSendCopy(mine);
            u64 nb = 0, pb = 0;
            comm.mNext.recv(nb);
            comm.mPrev.recv(pb);
            f->nextBox = (const void*)(uintptr_t)nb;
            f->prevBox = (const void*)(uintptr_t)pb;
            return f;
        }
        // one party per process: which GPUs the neighbours run on decides the
        // scope of the messages (the three parties reach the same answer: in
        // a ring of three every party neighbours both others)
        u8 uuid[16], un[16], up[16];
        GPU_CALL(aby3g_device_uuid(g.device(), uuid));
        comm.mNext.asyncSendCopy(uuid, 16);
        comm.mPrev.asyncSendCopy(uuid, 16);
        comm.mNext.recv(un, 16);
        comm.mPrev.recv(up, 16);
        // (forceRemote: the three-GPU branch on one GPU, for tests and the
        // bench -- uncached mailboxes and system-scope messages)
        f->sysScope = comm.forceRemote || std::memcmp(un, uuid, 16) != 0 || std::memcmp(up, uuid, 16) != 0;
        GPU_CALL(aby3g_set_device(g.device()));
        const size_t mbx = ipcBytes(mb);  // exported: whole 2 MiB blocks
        GPU_CALL(f->sysScope ? aby3g_malloc_uncached(&f->ownBox, mbx) : aby3g_malloc(&f->ownBox, mbx));
        GPU_CALL(aby3g_memset(f->ownBox, 0, mbx, g.stream()));
        g.sync();  // zeroed before its handle leaves
        aby3g_ipc_handle h{}, hn{}, hp{};
        GPU_CALL(aby3g_ipc_get_handle(f->ownBox, &h));
        comm.mNext.asyncSendCopy(h);
        comm.mPrev.asyncSendCopy(h);
        comm.mNext.recv(hn);
        comm.mPrev.recv(hp);
        GPU_CALL(aby3g_ipc_open(&hn, &f->mapped[0]));
        GPU_CALL(aby3g_ipc_open(&hp, &f->mapped[1]));
        f->nextBox = f->mapped[0];
        f->prevBox = f->mapped[1];
        // Every party's earlier work (the setup's copies in and out of the
        // peers' staging slots) drained before any party's first fused launch,
        // whose workgroups spin on the peers' mailboxes: a three-process run
        // once ended its first iteration with every party's waits timed out.
        g.sync();
        const u64 token = 1;
        u64 tn = 0, tp = 0;
        comm.mNext.asyncSendCopy(token);
        comm.mPrev.asyncSendCopy(token);
        comm.mNext.recv(tn);
        comm.mPrev.recv(tp);
        return f;
    }

    // the levelized circuit as device arrays: gates in batch order, batch
    // ends, per level (first gate, batches, AND gates, AND output wires)
    void upload(Gpu& g) {
        BetaCircuit* c = lib.int_Sh3Piecewise_helper(64, 2);
        if (!c->levelized()) c->levelByAndDepth();
        if (c->mInputs.size() != 3 || c->mOutputs.size() != 3) throw std::runtime_error("piecewise helper shape");
        for (const auto& in : c->mInputs) {
            if (in.size() != 64) throw std::runtime_error("piecewise helper inputs");
            for (size_t k = 1; k < in.size(); ++k)
                if (in[k] != in[k - 1] + 1) throw std::runtime_error("piecewise helper inputs not contiguous");
        }
        for (const auto& o : c->mOutputs)
            if (o.size() != 1) throw std::runtime_error("piecewise helper outputs");
        std::vector<aby3g_gate> gates(c->mBatchGates.size());
        for (size_t i = 0; i < gates.size(); ++i) {
            const BetaGate& b = c->mBatchGates[i];
            gates[i] = aby3g_gate{b.in0, b.in1, b.out, (u32)b.type, c->mBatchZRow[i], c->mBatchSendRow[i]};
        }
        std::vector<u32> ends, andWires;
        std::vector<aby3g_lr_level> levels;
        std::vector<aby3g_lr_gate_ext> ext;
        const bool fold = foldLevels(*c, gates, ext);
        size_t gi = 0;
        for (size_t L = 0; L < c->mLevelCounts.size(); ++L) {
            aby3g_lr_level lv{};
            const auto& batches = c->mLevelBatches[L];
            lv.first_gate = batches.empty() ? 0 : batches.front().begin;
            lv.batch_off = (u32)ends.size();
            if (fold && !batches.empty()) {
                // one batch: the later batches' gates folded into the first (foldLevels)
                lv.nbatch = 1;
                ends.push_back(batches.back().begin + batches.back().count - lv.first_gate);
                lv.fused_first = batches.front().count;
                lv.ext_off = (u32)foldOff[L];
            } else {
                lv.nbatch = (u32)batches.size();
                for (const auto& b : batches) ends.push_back(b.begin + b.count - lv.first_gate);
            }
            lv.and_wire_off = (u32)andWires.size();
            for (u32 k = 0; k < c->mLevelCounts[L]; ++k, ++gi)
                if (isAndType(c->mLevelGates[gi].type)) andWires.push_back(c->mLevelGates[gi].out);
            lv.nand = (u32)andWires.size() - lv.and_wire_off;
            if (lv.nand != c->mLevelAndCounts[L]) throw std::runtime_error("level AND count");
            levels.push_back(lv);
        }
        std::vector<u8> host;
        auto put = [&](const void* p, size_t bytes) {
            const size_t off = (host.size() + 15) / 16 * 16;
            host.resize(off + bytes);
            if (bytes) std::memcpy(host.data() + off, p, bytes);
            return off;
        };
        const size_t oG = put(gates.data(), gates.size() * sizeof(aby3g_gate));
        const size_t oE = put(ends.data(), ends.size() * 4);
        const size_t oL = put(levels.data(), levels.size() * sizeof(aby3g_lr_level));
        const size_t oA = put(andWires.data(), andWires.size() * 4);
        const size_t oX = put(ext.data(), ext.size() * sizeof(aby3g_lr_gate_ext));
        circuit.reset(g, host.size());
        toDevice(circuit.data(), host.data(), host.size(), g);
        const u8* base = circuit.as<u8>();
        cir.nlevels = (u32)levels.size();
        cir.wires = c->mWireCount;
        cir.nand = c->mAndCount;
        cir.ngates = (u32)gates.size();
        for (int i = 0; i < 3; ++i) {
            cir.in_wire[i] = c->mInputs[(size_t)i][0];
            cir.out_wire[i] = c->mOutputs[(size_t)i][0];
        }
        cir.gates = reinterpret_cast<const aby3g_gate*>(base + oG);
        cir.batch_ends = reinterpret_cast<const u32*>(base + oE);
        cir.levels = reinterpret_cast<const aby3g_lr_level*>(base + oL);
        cir.and_wires = reinterpret_cast<const u32*>(base + oA);
        cir.ext = fold && !ext.empty() ? reinterpret_cast<const aby3g_lr_gate_ext*>(base + oX) : nullptr;
        cir.next = fold ? (u32)ext.size() : 0;
    }

    // Folds every level's later gate batches into its first: the local
    // XOR / NXOR / INV / COPY gates of the level (whose outputs the later
    // batches read) are substituted into the later gates' operands, each
    // operand then the XOR of at most four wires available when the level
    // starts, optionally inverted (aby3g_lr_gate_ext). The values, and so the
    // shares, are the same as evaluating batch after batch; a level then takes
    // one workgroup barrier instead of one per batch. Gates keep their batch
    // order (the first batch, then the folded ones) and their z / send rows.
    // Returns false (nothing folded) when an operand would need more terms or
    // reduces to a constant.
    std::vector<size_t> foldOff;  // per level: its first ext entry
    bool foldLevels(const BetaCircuit& c, std::vector<aby3g_gate>& gates, std::vector<aby3g_lr_gate_ext>& ext) {
        if (c.mWireCount >= 0xFFFF) return false;
        struct Expr {
            std::vector<u32> t;  // XOR terms, sorted, no repeats
            bool inv = false;
        };
        auto xorInto = [](Expr& a, const Expr& b) {
            std::vector<u32> r;
            std::set_symmetric_difference(a.t.begin(), a.t.end(), b.t.begin(), b.t.end(), std::back_inserter(r));
            a.t.swap(r);
            a.inv ^= b.inv;
        };
        std::vector<aby3g_gate> out = gates;
        std::vector<aby3g_lr_gate_ext> ex;
        std::vector<size_t> offs;
        for (size_t L = 0; L < c.mLevelCounts.size(); ++L) {
            offs.push_back(ex.size());
            const auto& batches = c.mLevelBatches[L];
            std::unordered_map<u32, Expr> local;  // outputs of this level's local gates
            auto expr = [&](u32 w) {
                auto it = local.find(w);
                if (it != local.end()) return it->second;
                Expr e;
                e.t = {w};
                return e;
            };
            for (size_t b = 0; b < batches.size(); ++b)
                for (u32 k = batches[b].begin; k < batches[b].begin + batches[b].count; ++k) {
                    const aby3g_gate& gt = gates[k];
                    const bool unary = gt.type == ABY3G_GATE_COPY || gt.type == ABY3G_GATE_INV;
                    Expr x = expr(gt.in0), y = unary ? x : expr(gt.in1);
                    if (b > 0) {
                        for (const Expr* e : {&x, &y})
                            if (e->t.empty() || e->t.size() > 4) return false;
                        aby3g_lr_gate_ext e{};
                        for (int i = 0; i < 3; ++i) {
                            e.x[i] = (uint16_t)(i + 1 < (int)x.t.size() ? x.t[(size_t)i + 1] : 0xFFFF);
                            e.y[i] = (uint16_t)(i + 1 < (int)y.t.size() ? y.t[(size_t)i + 1] : 0xFFFF);
                        }
                        e.flags = (uint16_t)((x.inv ? 1 : 0) | (y.inv ? 2 : 0));
                        out[k].in0 = x.t[0];
                        out[k].in1 = y.t[0];
                        ex.push_back(e);
                    }
                    if (!isAndType((GateType)gt.type)) {  // a local gate: its output as an expression
                        Expr o = x;
                        if (gt.type == ABY3G_GATE_XOR || gt.type == ABY3G_GATE_NXOR) xorInto(o, y);
                        if (gt.type == ABY3G_GATE_NXOR || gt.type == ABY3G_GATE_INV) o.inv = !o.inv;
                        local[gt.out] = o;
                    }
                }
        }
        gates.swap(out);
        ext.swap(ex);
        foldOff.swap(offs);
        return true;
    }

    // One iteration's randomness, in the order the op-by-op path takes it.
    aby3g_lr_rand takeRand(Sh3ShareGen& gen, u64& otNext, u64& otPrev, int p) const {
        aby3g_lr_rand r{};
        // mul(XX, w): the truncation pair (Sh3Evaluator.cpp:526-527)
        r.t1_next_off = gen.takeNext(8 * B);
        r.t1_prev_off = gen.takePrev(8 * B);
        // the piecewise circuit's setCir keys (Sh3BinaryEvaluator.h:96-102)
        const block kp = gen.getPrevBlock(), kn = gen.getNextBlock();
        std::memcpy(r.mask_prev, kp.data(), 16);
        std::memcpy(r.mask_next, kn.data(), 16);
        // region 1: the OT product (Sh3Evaluator.cpp:132-263)
        if (p == 0) {
            r.ot_prev_off = gen.takePrev(16 * B);
            r.ot_next_off = gen.takeNext(8 * B);
            r.ot_ctr = otNext;
            otNext += 2 * B;
        } else if (p == 1) {
            r.ot_prev_off = gen.takePrev(8 * B);
        } else {
            r.ot_next_off = gen.takeNext(16 * B);
            r.ot_ctr = otPrev;
            otPrev += 2 * B;
        }
        // region 2: the public product (:430-487)
        r.pm_draw = gen.takeDraws(B);
        if (p == 0 || p == 1) {
            r.pm_ctr_next = otNext;
            otNext += B;
        }
        if (p == 0 || p == 2) {
            r.pm_ctr_prev = otPrev;
            otPrev += B;
        }
        // mulTruncate(XX^T, err): the truncation pair
        r.t2_next_off = gen.takeNext(8 * d);
        r.t2_prev_off = gen.takePrev(8 * d);
        return r;
    }

    void step(aby3ML& ml, const si64Matrix& X, const si64Matrix& Y, si64Matrix& w, const u32* batchIdx, u64 aB,
              u64* phaseTicks, const u32* nextBatch) {
        Gpu& g = ml.mRt.gpu();
        Sh3Evaluator& ev = ml.mEval;
        Sh3ShareGen& gen = ev.mShareGen;
        const int p = (int)ml.mRt.mPartyIdx;
        aby3g_lr_iter it{};
        it.party = p;
        it.B = (u32)B;
        it.d = (u32)d;
        it.D = (u32)ml.mD;
        it.aB = (u32)aB;
        it.n = X.rows();
        it.X = X.data();
        it.Y = Y.data();
        it.w = w.data();
        it.batch = batchIdx;
        it.next_batch = nextBatch;
        it.cir = cir;
        it.scratch = scratch.data();
        it.mailbox = ownBox ? ownBox : mailbox.data();
        it.sys_scope = sysScope ? 1 : 0;
        it.next_mailbox = nextBox;
        it.prev_mailbox = prevBox;
        it.epoch = ++epoch;
        it.wait_ticks = g.waitTicks();
        it.phase_ticks = phaseTicks;
        std::memcpy(it.prev_seed, gen.mPrevSeed.data(), 16);
        std::memcpy(it.next_seed, gen.mNextSeed.data(), 16);
        std::memcpy(it.zs_prev, gen.mKeyPrev.data(), 16);
        std::memcpy(it.zs_next, gen.mKeyNext.data(), 16);
        std::memcpy(it.ot_next_key, ev.mOtNextKey.data(), 16);
        std::memcpy(it.ot_prev_key, ev.mOtPrevKey.data(), 16);
        // this iteration's randomness, taken from the party's state exactly as
        // the op-by-op path takes it
        const aby3g_lr_rand cur = takeRand(gen, ev.mOtNextIdx, ev.mOtPrevIdx, p);
        it.t1_next_off = cur.t1_next_off;
        it.t1_prev_off = cur.t1_prev_off;
        std::memcpy(it.mask_prev, cur.mask_prev, 16);
        std::memcpy(it.mask_next, cur.mask_next, 16);
        it.ot_prev_off = cur.ot_prev_off;
        it.ot_next_off = cur.ot_next_off;
        it.ot_ctr = cur.ot_ctr;
        it.pm_ctr_next = cur.pm_ctr_next;
        it.pm_ctr_prev = cur.pm_ctr_prev;
        it.pm_draw = cur.pm_draw;
        it.t2_next_off = cur.t2_next_off;
        it.t2_prev_off = cur.t2_prev_off;
        // Drawn ahead: the previous launch's helpers drew this iteration's
        // randomness if they predicted it right (nothing else took from the
        // party's streams in between); this launch's draw the next one's, as
        // predicted from a copy of the state (the real state is not advanced).
        it.pre_have = havePred && std::memcmp(&pred, &cur, sizeof cur) == 0;
        {
            Sh3ShareGen g2 = gen;
            u64 on = ev.mOtNextIdx, op = ev.mOtPrevIdx;
            pred = takeRand(g2, on, op, p);
        }
        it.pre_next = 1;
        it.next_rand = pred;
        havePred = true;
        it.thr_off[0] = thrOff[0];
        it.thr_off[1] = thrOff[1];
        it.half = half;
        it.slope = slope;
        it.one = one;
        GPU_CALL(aby3g_lr_iteration(&it, g.stream()));
    }
};

void sgdLogisticStepOps(aby3ML& ml, const si64Matrix& X, const si64Matrix& Y, si64Matrix& w, const u32* batchIdx,
                        u64 B, u64 aB, SgdState& st);

void sgdLogisticStep(aby3ML& ml, const si64Matrix& X, const si64Matrix& Y, si64Matrix& w, const u32* batchIdx,
                     u64 B, u64 aB, SgdState& st) {
    if (!st.fusedChecked) {
        st.fused = FusedLr::make(ml, X.cols(), B);
        st.fusedChecked = true;
        st.fusedSysScope = st.fused && st.fused->sysScope;
    }
    if (st.fused && st.fused->B == B && st.fused->d == X.cols()) {
        st.fused->step(ml, X, Y, w, batchIdx, aB, st.phaseTicks, st.nextBatch);
        return;
    }
    sgdLogisticStepOps(ml, X, Y, w, batchIdx, B, aB, st);
}

// the op-by-op iteration (every step a C-ABI call, messages over the channels)
void sgdLogisticStepOps(aby3ML& ml, const si64Matrix& X, const si64Matrix& Y, si64Matrix& w, const u32* batchIdx,
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
            randomShuffle(mPool.data(), mPool.size(), mPrng);
            mIter = 0;
        }
    }
}

// Pool k (k = 0: the identity, then one reshuffle per epoch) lives in pinned
// host buffer k & 1 and device buffer k & 1. The host thread that shuffles
// pool k + 1 starts when pool k becomes current: it copies pool k into the
// other pinned buffer (pool k - 1's, whose upload finished an epoch ago) and
// shuffles it in place. When pool k runs out, next() joins the thread and
// enqueues the upload of pool k + 1 into the other device buffer. Every
// device-side reuse (a pool buffer, a batch slot) is ordered behind the
// iterations that read it by the party's stream itself; the host waits only
// before it rewrites a pinned buffer whose upload might still be in flight.
struct DeviceBatchSampler::Impl {
    Gpu& g;
    u64 n, B;
    HostPrng prng{toBlock(234543234)};
    u32* pinned[2] = {nullptr, nullptr};  // pool k & 1 (host)
    u32* bslot = nullptr;                 // [2][B] pinned: batches across a reshuffle
    DeviceBuffer dpool[2], dbatch[2];
    Event upEv[2], bEv[2];
    bool upRec[2] = {false, false}, bRec[2] = {false, false};
    u64 k = 0, iter = 0, bnext = 0;
    std::thread shuffler;

    Impl(Gpu& gg, u64 n_, u64 B_) : g(gg), n(n_), B(B_) {
        if (!n || !B || B > n || n > 0xffffffffull)
            throw std::runtime_error("DeviceBatchSampler: need 0 < B <= n < 2^32");
        for (auto& p : pinned) GPU_CALL(aby3g_host_malloc((void**)&p, n * 4));
        GPU_CALL(aby3g_host_malloc((void**)&bslot, 2 * B * 4));
        for (u64 i = 0; i < n; ++i) pinned[0][i] = (u32)i;
        for (auto& d : dpool) d.reset(g, n * 4);
        for (auto& d : dbatch) d.reset(g, B * 4);
        toDevice(dpool[0].data(), pinned[0], n * 4, g);
        iter = n;  // idxIter = indices.end(): the first getSubset reshuffles (Regression.h:236)
        startShuffle();
    }
    ~Impl() {
        if (shuffler.joinable()) shuffler.join();
        for (int b = 0; b < 2; ++b) {  // uploads out of the pinned buffers
            if (upRec[b]) upEv[b].sync();
            if (bRec[b]) bEv[b].sync();
        }
        for (auto* p : pinned) aby3g_host_free(p);
        aby3g_host_free(bslot);
    }
    void startShuffle() {
        const int b = (int)((k + 1) & 1);
        if (upRec[b]) upEv[b].sync();  // pool k - 1's upload (an epoch ago)
        const u32* src = pinned[k & 1];
        u32* dst = pinned[b];
        shuffler = std::thread([this, src, dst] {
            std::memcpy(dst, src, n * 4);
            randomShuffle(dst, n, prng);
        });
    }
    // pool k ran out: pool k + 1 becomes current
    void reshuffle() {
        shuffler.join();
        const int b = (int)((k + 1) & 1);
        GPU_CALL(aby3g_memcpy(dpool[b].data(), pinned[b], n * 4, 0, g.stream()));
        upEv[b].record(g.stream());
        upRec[b] = true;
        ++k;
        iter = 0;
        startShuffle();
    }
    const u32* next() {
        if (iter == n) reshuffle();
        if (iter + B <= n) {
            const u32* p = dpool[k & 1].as<u32>() + iter;
            iter += B;
            if (iter == n) reshuffle();
            return p;
        }
        // the batch spans a reshuffle: the tail of this pool, the head of the next
        const int s = (int)(bnext++ & 1);
        if (bRec[s]) bEv[s].sync();
        u32* dst = bslot + (u64)s * B;
        u64 d = 0;
        while (d != B) {
            const u64 step = std::min<u64>(n - iter, B - d);
            std::memcpy(dst + d, pinned[k & 1] + iter, step * 4);
            iter += step;
            d += step;
            if (iter == n) reshuffle();
        }
        GPU_CALL(aby3g_memcpy(dbatch[s].data(), dst, B * 4, 0, g.stream()));
        bEv[s].record(g.stream());
        bRec[s] = true;
        return dbatch[s].as<u32>();
    }
};

DeviceBatchSampler::DeviceBatchSampler(Gpu& g, u64 n, u64 B) : mImpl(std::make_unique<Impl>(g, n, B)) {}
DeviceBatchSampler::~DeviceBatchSampler() = default;
const u32* DeviceBatchSampler::next() { return mImpl->next(); }
u64 DeviceBatchSampler::reshuffles() const { return mImpl->k; }

void SGD_Logistic(RegressionParam& params, aby3ML& engine, const si64Matrix& X, const si64Matrix& Y, si64Matrix& w) {
    if (X.rows() != Y.rows() || Y.cols() != 1) throw std::runtime_error(LOCATION);
    const u64 B = params.mBatchSize;
    // the learning rate in log2 form: truncate this many bits (Regression.h:246)
    const u64 aB = (u64)std::log2(1 / (params.mLearningRate / (double)B));
    DeviceBatchSampler sampler(engine.mRt.gpu(), X.rows(), B);
    SgdState st;
    for (u64 i = 0; i < params.mIterations; ++i)
        sgdLogisticStep(engine, X, Y, w, sampler.next(), B, aB, st);
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
