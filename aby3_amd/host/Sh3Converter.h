// Share conversions (aby3/sh3/Sh3Converter.h/.cpp) on the GPU engine.
//
//   toBinaryMatrix(dep, si64Matrix, sbMatrix)  arithmetic -> binary: P0
//       reshares x0 + x2 binary-randomized with its prev stream, P1/P2 expose
//       x1, then 64-bit adder circuits (getArithToBinCircuit) (:61-207)
//   bitInjection(dep, sbMatrix, si64Matrix)     every bit of a binary matrix
//       -> an arithmetic 0/1 value via a 3-party OT, P2 sending (:209-371)
//   toPackedBin / toBinaryMatrix(sPackedBin)    local bit transposes (:11-59)
//
// Same task semantics, stream consumption and message order as the
// reference; the local compute of every round is one or two C-ABI launches
// (include/aby3gpu.h: aby3g_a2b_reshare, aby3g_bitinj_send,
// aby3g_ot_help_bits, aby3g_ot_recv_bits, the bit transposes).
#pragma once
#include "Circuit.h"
#include "Sh3BinaryEvaluator.h"
#include "Sh3Runtime.h"
#include "Sh3ShareGen.h"
#include "Sh3Types.h"
#include <map>
#include <memory>

namespace aby3 {

class Sh3Converter {
public:
    CircuitLibrary mLib;
    Sh3ShareGen* mRandGen = nullptr;
    Sh3BinaryEvaluator mBin;
    // SharedOT mOT12 / mOT02: AES key + counter (SharedOT.h:9-12; the
    // reference sets mIdx = party, then setSeed resets it to 0)
    block mOT12Key, mOT02Key;
    u64 mOT12Idx = ~0ull, mOT02Idx = ~0ull;

    // Sh3Converter::init (Sh3Converter.h:25-40): P0 seeds mOT02 from its prev
    // stream, P1 mOT12 from its next stream, P2 mOT12 from prev then mOT02
    // from next (16 bytes each).
    void init(Sh3Runtime& rt, Sh3ShareGen& gen);

    void toPackedBin(const sbMatrix& in, sPackedBin& dest);
    void toBinaryMatrix(const sPackedBin& in, sbMatrix& dest);

    // dest is resized to in.rows() x 64 * in.cols() when empty; a pre-sized
    // dest must keep ceil(bitCount / 64) == in.cols() (the reference indexes
    // both flat)
    Sh3Task toBinaryMatrix(Sh3Task dep, const si64Matrix& in, sbMatrix& dest);

    // dest: in.rows() x in.bitCount(), element (i, j) = bit j of row i.
    // twoRounds: P0 forwards its share to P1 instead of helping a second OT.
    Sh3Task bitInjection(Sh3Task dep, const sbMatrix& in, si64Matrix& dest, bool twoRounds = false);

    // numWords = ceil(bitCount / base) independent `base`-bit adders, output =
    // in0 + in1 per word (Sh3Converter.cpp:373-409)
    static void buildArithToBinCircuit(BetaCircuit& cir, u64 base, u64 bitCount);
    BetaCircuit getArithToBinCircuit(u64 base, u64 bitCount);
    // getArithToBinCircuit(64, bitCount), levelized once per bitCount (the
    // reference rebuilds mCir every call, :110)
    BetaCircuit* arithToBinCircuit(u64 bitCount);

private:
    std::map<u64, std::unique_ptr<BetaCircuit>> mA2B;
    DeviceBuffer mIota;  // wire ids 0..mIotaCount-1 for the packed -> sbMatrix transpose
    u64 mIotaCount = 0;
    const u32* wireIds(u64 bitCount, Gpu& g);
};

}  // namespace aby3
