// Boolean circuits for the bit-sliced engine: a gate-list IR with
// AND-depth levelization (the role of cryptoTools' BetaCircuit /
// levelByAndDepth) and the circuit library of the hot path
// (aby3/Circuit/CircuitLibrary.cpp + the BetaLibrary circuits it calls).
//
// cryptoTools' BetaLibrary is not vendored in the reference, so these are
// this engine's own circuits: depth-optimized parallel-prefix (Brent-Kung
// tree / Sklansky) adders in the generate/propagate form, where the OR of a
// prefix combine is an XOR because g and p&G are never both 1. Gate order
// defines which AND mask (z counter) a gate uses, so share-level parity with
// the reference's binary engine is not defined; parity is at revealed values
//  and share-level against the oracle on the same gate list.
#pragma once
#include "Defines.h"
#include <iosfwd>
#include <map>
#include <memory>
#include <vector>

namespace aby3 {

enum class GateType : u32 { Xor = 0, Nxor = 1, And = 2, Or = 3, Nor = 4, na_And = 5, a = 6, Inv = 7 };
inline bool isAndType(GateType t) {
    return t == GateType::And || t == GateType::Or || t == GateType::Nor || t == GateType::na_And;
}

struct BetaGate {
    u32 in0, in1, out;
    GateType type;
};

using BetaBundle = std::vector<u32>;  // wire ids, LSB first

class BetaCircuit {
public:
    BetaCircuit();
    // process-unique id of this circuit's levelized form (device caches key on it,
    // never on the address, which a later circuit may reuse)
    u64 serial() const { return mSerial; }
    u32 mWireCount = 0;
    std::vector<BetaGate> mGates;           // construction order (topological)
    std::vector<BetaBundle> mInputs, mOutputs;

    BetaBundle addInputBundle(u32 bits);
    void addOutputBundle(const BetaBundle& b) { mOutputs.push_back(b); }
    u32 addGate(u32 in0, u32 in1, GateType t);  // returns the output wire
    u32 addUnary(u32 in, GateType t) { return addGate(in, in, t); }

    // ---- levelized form (levelByAndDepth) --------------------------------
    // Level L holds the gates whose inputs are complete at the start of
    // communication round L; an AND-type output is complete one round later.
    // Inside a level the gates are kept in construction order (mLevelGates)
    // and split into batches of mutually independent gates for the GPU.
    std::vector<BetaGate> mLevelGates;
    std::vector<u32> mLevelCounts, mLevelAndCounts;
    struct Batch {
        u32 begin, count;  // into mBatchGates
    };
    std::vector<std::vector<Batch>> mLevelBatches;
    std::vector<BetaGate> mBatchGates;       // gates grouped by batch
    std::vector<u32> mBatchZRow, mBatchSendRow;  // per mBatchGates entry (AND-type only)
    u32 mAndCount = 0;
    bool levelized() const { return !mLevelCounts.empty() || mGates.empty(); }
    void levelByAndDepth();

    // plaintext evaluation on 64-bit words (tests; row r of a word = bit r)
    std::vector<std::vector<u64>> evalPlain(const std::vector<std::vector<u64>>& inputs) const;

    // Binary circuit files (cryptoTools BetaCircuit::writeBin / readBin, used
    // by aby3-DB/DBServer.cpp:48-54 and aby3-DB_tests/lowMC.cpp:296-324 to
    // store and reload externally built circuits). cryptoTools is not vendored
    // in the reference, so the layout is this restatement of its published
    // form, all fields little-endian:
    //   u64 wireCount, u64 nonXorGateCount,
    //   u64 #inputs,  per bundle: u64 size, u32 wire[size],
    //   u64 #outputs, per bundle: u64 size, u32 wire[size],
    //   u64 #gates,   per gate: u32 in0, u32 in1, u32 out, u8 type, u8 pad[3]
    // with `type` cryptoTools' GateType code (the gate's truth table, bit
    // a + 2b = output: Xor 6, Nxor 9, And 8, Or 14, Nor 1, na_And 4, a 10,
    // na 5). readBin checks every index and the topological order and
    // returns the circuit unlevelized (levelByAndDepth() before evaluation).
    void writeBin(std::ostream& out) const;
    void readBin(std::istream& in);

private:
    u64 mSerial;
};

// The circuit library of the hot path. Circuits are cached per shape.
class CircuitLibrary {
public:
    // MSB(a + b) of two `size`-bit two's complement inputs
    // (int_comp_helper, CircuitLibrary.cpp:350-394; fetch_msb)
    BetaCircuit* int_comp_helper(u64 size);
    // [a < b], signed (cryptoTools int_int_lt; bool_cipher_lt passes (B, A),
    // BoolBasic.cpp:20-40 -- here input 0 is a, input 1 is b)
    BetaCircuit* int_int_lt(u64 size);
    // [a == b] (int_eq)
    BetaCircuit* int_eq(u64 size);
    // a + b mod 2^size (int_int_add)
    BetaCircuit* int_int_add(u64 size);
    // a - b mod 2^size (int_int_sub)
    BetaCircuit* int_int_sub(u64 size);
    // bitwise a & b, a | b (int_int_bitwiseAnd / Or)
    BetaCircuit* int_int_bitwiseAnd(u64 size);
    BetaCircuit* int_int_bitwiseOr(u64 size);
    // bitwise NOR (bits_nor_helper, CircuitLibrary.cpp:396-428)
    BetaCircuit* bits_nor_helper(u64 size);
    // region bits of a piecewise function with T thresholds
    // (int_Sh3Piecewise_helper, CircuitLibrary.cpp:38-137): inputs aa_0..aa_{T-1}
    // (= x - t_t partial) then b; outputs c_0..c_T (1 bit each)
    BetaCircuit* int_Sh3Piecewise_helper(u64 size, u64 numThresholds);
    // compare-and-swap of two signed `size`-bit keys: outputs (min, max)
    // (bool_cipher_max_min_split, BoolBasic.cpp:275-312, fused into one circuit)
    BetaCircuit* cmp_swap(u64 size);

    // any of the above by its name (param = thresholds for the piecewise helper);
    // throws std::runtime_error for an unknown name
    BetaCircuit* byName(const std::string& name, u64 size, u64 param = 0);

private:
    std::map<std::pair<std::string, u64>, std::unique_ptr<BetaCircuit>> mCirMap;
    BetaCircuit* get(const std::string& name, u64 key);
};

// Building blocks (exposed for composite circuits)
namespace circuits {
// carry into bit `upto` of a + b (+ cin), with g_i = ga[i], p_i = pa[i]
u32 prefixCarry(BetaCircuit& c, const std::vector<u32>& g, const std::vector<u32>& p, u64 n);
u32 msbOfAdd(BetaCircuit& c, const BetaBundle& a, const BetaBundle& b);
u32 lessThanSigned(BetaCircuit& c, const BetaBundle& a, const BetaBundle& b);
BetaBundle add(BetaCircuit& c, const BetaBundle& a, const BetaBundle& b, bool subtract);
}  // namespace circuits

}  // namespace aby3
