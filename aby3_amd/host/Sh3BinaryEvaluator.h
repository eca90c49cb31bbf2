// Bit-sliced binary evaluator (aby3/sh3/Sh3BinaryEvaluator.h/.cpp) on the GPU.
//
// Memory: one device allocation [2][wires][words] (wire-major, 64 rows per
// u64, rows padded to a multiple of 2048 as mMem.reset(width, wires, 8)).
// AND masks: the z words of the circuit are generated on device before the
// rounds that use them (they depend only on the setCir keys), z[k][w] = draw
// k*words + w of the (prev, next) keys -- exactly getShares()'s counter
// schedule (Sh3BinaryEvaluator.cpp:1406-1434).
// One communication round per AND level, as roundCallback (:539-1196):
// unpack last level's received shares, run this level's gate batches, send
// the AND outputs' share 0 to next, post the receive from prev.
#pragma once
#include "Circuit.h"
#include "Sh3Runtime.h"
#include "Sh3ShareGen.h"
#include "Sh3Types.h"

namespace aby3 {

class Sh3BinaryEvaluator {
public:
    Sh3BinaryEvaluator() = default;
    Sh3BinaryEvaluator(const Sh3BinaryEvaluator&) = delete;
    Sh3BinaryEvaluator& operator=(const Sh3BinaryEvaluator&) = delete;
    ~Sh3BinaryEvaluator() {
        // the masks' buffer is reused behind its draw
        try {
            // (a ring slot whose Gpu is gone needs nothing: the ring went with it)
            if (mZPending && mGpu && (mZSlot < 0 || !mRing.expired())) waitZ();
            releaseZ();
        } catch (...) {
        }
    }
    // consumes 16 bytes of the prev and next streams for the AND keys
    // (Sh3BinaryEvaluator.h:96-102)
    void setCir(BetaCircuit* cir, u64 width, Sh3ShareGen& gen);
    void setCir(BetaCircuit* cir, u64 width, block prevSeed, block nextSeed);
    // setCir for rows [rowOffset, rowOffset + width) of a totalRows-row
    // evaluation (one party's rows split over GPUs): the AND
    // masks are the slice's words of every gate's row of draws, so the
    // slice's shares are those rows of the unsplit evaluation's. rowOffset is
    // a multiple of 2048 (the engine's row padding), and so is width unless
    // the slice ends at totalRows.
    void setCirRows(BetaCircuit* cir, u64 width, Sh3ShareGen& gen, u64 rowOffset, u64 totalRows);
    void setInput(u64 i, const sbMatrix& in);
    // setInput from mapped rows of `in` (circuit row p <- row map(p)): the
    // compare-exchange gather of a merge round fused into the transpose
    void setInput(u64 i, const sbMatrix& in, const aby3g_rowmap& map);
    // setInput(i, in, mi) and setInput(j, in, mj) in one launch
    void setInputs(u64 i, const aby3g_rowmap& mi, u64 j, const aby3g_rowmap& mj, const sbMatrix& in);
    // a one-row shared input broadcast to every row (Sh3BinaryEvaluator.cpp:105-138)
    void setReplicatedInput(u64 i, const sbMatrix& in);
    // Inputs straight from arithmetic shares, several in one launch (no
    // sbMatrix in between): share `share` of circuit input `input` takes the
    // value sum_t coef[t] * term[t][.] + constant (all terms null: zero).
    struct WireInput {
        u64 input = 0;
        int share = 0;
        const i64* term[4] = {nullptr, nullptr, nullptr, nullptr};
        i64 coef[4] = {0, 0, 0, 0};
        i64 constant = 0;
        i64* copyOut = nullptr;  // optional: receives sum_t coef[t] * term[t][.]
    };
    // The terms are raw pointers and may be read by the first level's launch
    // (fused inputs), which roundCallback enqueues later: a caller whose
    // term buffer could go back to a pool before then hands it to
    // holdForInputs first (kept until that launch is enqueued, then fenced).
    void setInputs(const std::vector<WireInput>& in);
    void holdForInputs(std::shared_ptr<DeviceBuffer> b);
    Sh3Task asyncEvaluate(Sh3Task dep);
    Sh3Task asyncEvaluate(Sh3Task dep, BetaCircuit* cir, Sh3ShareGen& gen, std::vector<const sbMatrix*> inputs,
                          std::vector<sbMatrix*> outputs);
    void getOutput(u64 i, sbMatrix& out);
    // getOutput into mapped rows of an existing `out` (row map(p) <- circuit
    // row p; other rows untouched): the round's scatter
    void getOutput(u64 i, sbMatrix& out, const aby3g_rowmap& map);
    // getOutput(i, out, mi) and getOutput(j, out, mj) in one launch (the maps' rows disjoint)
    void getOutputs(u64 i, const aby3g_rowmap& mi, u64 j, const aby3g_rowmap& mj, sbMatrix& out);

    bool hasMoreRounds() const { return mLevel <= mCir->mLevelCounts.size(); }
    void roundCallback(CommPkg& comm, Sh3Task task);

    BetaCircuit* mCir = nullptr;
    u64 mRows = 0, mWords = 0, mLevel = 0;
    block mKeyPrev, mKeyNext;
    DeviceBuffer mMem, mZ;
    u64* mZPtr = nullptr;   // the AND masks: a slot of the Gpu's z ring, or mZ
    RecvFuture mRecvFutr;   // previous level's AND shares (zero-copy: the sender's buffer)
    bool mZPending = false;  // z masks still being drawn on the auxiliary stream

private:
    // The levelized circuit in device memory, one packed buffer uploaded once
    // per (circuit, Gpu): gates | batch ends | per-level AND output wires |
    // output-bundle wires. Cached on the Gpu (Gpu::attachment), so every
    // evaluator instance -- aby3-Basic makes one per call -- reuses it.
    struct DevCircuit {
        DeviceBuffer blob;
        const aby3g_gate* gates = nullptr;
        const u32* recvRows = nullptr;         // 2 per gate: recv row of in0 / in1 (aby3g_bin_level_rr)
        const u32* batchEnds = nullptr;        // relative to the level's first gate
        std::vector<u32> levelFirstGate, levelBatchOffset, levelBatches;
        std::vector<const u32*> outWires;      // per level
        const u32* allOutputWires = nullptr;
        std::vector<u32> outputOffsets;
        // the first level may take its inputs straight from setInputs'
        // linear combinations (aby3g_bin_level_in): the input wires' range,
        // when it spans at most ABY3G_LEVEL_IN_MAX_WIRES, and whether a later
        // level or an output reads them (then they are written to mMem too)
        bool fuseInputs = false;
        u32 inLo = 0, inHi = 0;
        bool inputsReadLater = false;
        // the round whose launch is the evaluation's last
        u64 lastLaunchLevel = 0;
    };
    std::shared_ptr<DevCircuit> mCur;
    Gpu* mGpu = nullptr;
    void upload(Gpu& g);
    // The AND masks are drawn on the Gpu's draw stream when it has one (the
    // co-located parties' shared fourth stream), else on aux(). Consecutive
    // evaluations alternate between two mask buffers kept on the Gpu, so the
    // draws of the next evaluation wait only for the last evaluation that
    // used the same buffer (its done event), not for everything enqueued so
    // far: their AES runs beside the previous evaluation's latency-bound
    // levels instead of in front of the next one's.
    struct ZRing {
        DeviceBuffer buf[2];
        std::unique_ptr<Event> done[2];
        bool busy[2] = {false, false}, recorded[2] = {false, false};
        int next = 0;
        aby3g_stream stream = nullptr;  // the owning party's main stream
    };
    std::weak_ptr<ZRing> mRing;  // owned by the Gpu (attachment): gone with it
    // one send buffer per evaluation, a view of it per level: one pool
    // allocation per evaluation, and the receiver fences once, after its
    // last level, instead of per level
    std::shared_ptr<DeviceBuffer> mSendAll;
    u64 mAndDone = 0;  // AND outputs of the levels already run (their rows in mSendAll)
    // held while mSendAll is the channel's arena slot (Channel::evalSendBuffer);
    // dropped with mSendAll, after the evaluation's last message, or with this
    std::shared_ptr<void> mArenaLease;
    bool mPerLevelSends = false;  // each level's sends in a staging slot of the link (Channel::linkSendBuffer)
    // setInputs' sources held for the first level's launch (DevCircuit::fuseInputs)
    std::vector<aby3g_wire_src> mPendingIn;
    // buffers the held sources read (e.g. a received message): kept alive
    // until the launch that reads them is enqueued (holdForInputs)
    std::vector<std::shared_ptr<DeviceBuffer>> mPendingHold;
    void readHeld(bool drop);
    // writes them to mMem the separate way (dropHolds false: more held
    // sources that read the same buffers follow)
    void flushPendingInputs(bool dropHolds = true);
    bool pendingCoversInputs() const;
    int mZSlot = -1;
    aby3g_stream mZStream = nullptr;     // the stream the masks are drawn on
    // Masks drawn on the party's own stream (no draw stream: one party per
    // process) are drawn in pieces: the first AND level's in setCir, the
    // later levels' behind the first level's launch and send, where the
    // stream would otherwise idle until the peers' shares arrive
    // (levelDraws()).
    bool mZByLevel = false;
    u64 mZDrawn = 0;  // AND rows (ordinals) whose masks are enqueued
    // a row slice (setCirRows): the slice's first word and the unsplit
    // evaluation's words per AND row (0: not a slice)
    u64 mZWordOffset = 0, mZRowStride = 0;
    void setCirImpl(BetaCircuit* cir, u64 width, block prevSeed, block nextSeed, u64 wordOffset, u64 rowStride);
    void drawZRows(u64 first, u64 end);  // the masks of AND rows [first, end)
    static int levelDraws();
    void drawZThrough(u64 level);
    std::unique_ptr<Event> mZEv, mZFresh; // draws done / main stream's position for fresh memory
    void waitZ();      // main stream waits for the draws
    // the ring slot is free once the main stream passes this point (at the
    // next setCir or destruction: an evaluation may be re-run on its masks)
    void releaseZ();
};

// The two-input binary resharing of an arithmetic value x (BuildingBlocks.cpp
// :475-502, Sh3Piecewise.cpp:392-470), written straight into `eng`'s input
// wires: input in0[k] := sign * (x0 + x2) + offsets[k], reshared by P0 (the
// one message, P0 -> P1, zero-copy), and input in1 := x1 (P1 and P2 hold it);
// x's shares are sums of coef * X.share(s) over the (X, coef) terms (at most
// two matrices). The circuit must already be set on `eng`.
void setTwoInputSharing(Sh3BinaryEvaluator& eng, int pIdx, const std::vector<std::pair<const si64Matrix*, i64>>& x,
                        i64 sign, const std::vector<u64>& in0, const std::vector<i64>& offsets, u64 in1, CommPkg& comm,
                        Gpu& g);

}  // namespace aby3
