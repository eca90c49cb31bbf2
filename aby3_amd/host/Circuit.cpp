#include "Circuit.h"
#include <atomic>
#include <algorithm>
#include <fstream>
#include <istream>
#include <ostream>

namespace aby3 {

namespace {
std::atomic<u64> g_circuitSerial{1};
}
BetaCircuit::BetaCircuit() : mSerial(g_circuitSerial++) {}

BetaBundle BetaCircuit::addInputBundle(u32 bits) {
    BetaBundle b(bits);
    for (u32 i = 0; i < bits; ++i) b[i] = mWireCount++;
    mInputs.push_back(b);
    mLevelCounts.clear();
    return b;
}

u32 BetaCircuit::addGate(u32 in0, u32 in1, GateType t) {
    if (in0 >= mWireCount || in1 >= mWireCount) throw std::runtime_error("gate input is not a wire " LOCATION);
    if (in0 == in1 && t != GateType::a && t != GateType::Inv)
        throw std::runtime_error("binary gate with identical inputs " LOCATION);
    u32 out = mWireCount++;
    mGates.push_back(BetaGate{in0, in1, out, t});
    mLevelCounts.clear();
    return out;
}

void BetaCircuit::levelByAndDepth() {
    std::vector<u32> avail(mWireCount, 0), level(mGates.size());
    u32 maxLevel = 0;
    for (size_t i = 0; i < mGates.size(); ++i) {
        const BetaGate& g = mGates[i];
        u32 L = std::max(avail[g.in0], avail[g.in1]);
        level[i] = L;
        avail[g.out] = isAndType(g.type) ? L + 1 : L;
        maxLevel = std::max(maxLevel, L);
    }
    const u32 nLevels = mGates.empty() ? 0 : maxLevel + 1;
    mLevelCounts.assign(nLevels, 0);
    mLevelAndCounts.assign(nLevels, 0);
    mLevelGates.clear();
    std::vector<std::vector<size_t>> byLevel(nLevels);
    for (size_t i = 0; i < mGates.size(); ++i) byLevel[level[i]].push_back(i);

    mLevelBatches.assign(nLevels, {});
    mBatchGates.clear();
    mBatchZRow.clear();
    mBatchSendRow.clear();
    std::vector<int> batchOf(mWireCount, -1);  // batch of the in-level producer of a wire
    u32 andOrdinal = 0;
    for (u32 L = 0; L < nLevels; ++L) {
        std::vector<std::vector<std::pair<BetaGate, std::pair<u32, u32>>>> batches;
        u32 sendRow = 0;
        for (size_t gi : byLevel[L]) {
            const BetaGate& g = mGates[gi];
            mLevelGates.push_back(g);
            ++mLevelCounts[L];
            int b = 0;
            const u32 ins[2] = {g.in0, g.in1};
            for (u32 w : ins)
                if (batchOf[w] >= 0) b = std::max(b, batchOf[w] + 1);
            u32 z = 0, s = 0;
            if (isAndType(g.type)) {
                ++mLevelAndCounts[L];
                z = andOrdinal++;
                s = sendRow++;
            } else {
                batchOf[g.out] = b;  // local outputs are usable later in this level
            }
            if ((int)batches.size() <= b) batches.resize(b + 1);
            batches[b].push_back({g, {z, s}});
        }
        // in-level producer marks expire at the end of the level
        for (size_t gi : byLevel[L]) batchOf[mGates[gi].out] = -1;
        for (auto& bt : batches) {
            Batch bb{(u32)mBatchGates.size(), (u32)bt.size()};
            for (auto& e : bt) {
                mBatchGates.push_back(e.first);
                mBatchZRow.push_back(e.second.first);
                mBatchSendRow.push_back(e.second.second);
            }
            mLevelBatches[L].push_back(bb);
        }
    }
    mAndCount = andOrdinal;
    mSerial = g_circuitSerial++;  // a new levelized form: device caches must not reuse the old one
}

std::vector<std::vector<u64>> BetaCircuit::evalPlain(const std::vector<std::vector<u64>>& inputs) const {
    if (inputs.size() != mInputs.size()) throw std::runtime_error("evalPlain: input count");
    const size_t W = inputs.empty() ? 0 : inputs[0].size();
    std::vector<std::vector<u64>> wire(mWireCount, std::vector<u64>(W, 0));
    for (size_t b = 0; b < mInputs.size(); ++b)
        for (size_t i = 0; i < mInputs[b].size(); ++i)
            for (size_t w = 0; w < W; ++w) wire[mInputs[b][i]][w] = (inputs[b][w] >> i) & 1 ? ~0ull : 0;
    for (const BetaGate& g : mGates)
        for (size_t w = 0; w < W; ++w) {
            u64 a = wire[g.in0][w], b = wire[g.in1][w], r = 0;
            switch (g.type) {
                case GateType::Xor: r = a ^ b; break;
                case GateType::Nxor: r = ~(a ^ b); break;
                case GateType::And: r = a & b; break;
                case GateType::Or: r = a | b; break;
                case GateType::Nor: r = ~(a | b); break;
                case GateType::na_And: r = ~a & b; break;
                case GateType::a: r = a; break;
                case GateType::Inv: r = ~a; break;
            }
            wire[g.out][w] = r;
        }
    std::vector<std::vector<u64>> out(mOutputs.size(), std::vector<u64>(W, 0));
    for (size_t o = 0; o < mOutputs.size(); ++o)
        for (size_t i = 0; i < mOutputs[o].size() && i < 64; ++i)
            for (size_t w = 0; w < W; ++w) out[o][w] |= (wire[mOutputs[o][i]][w] & 1) << i;
    return out;
}

// ------------------------------------------------------------------ blocks
namespace circuits {

u32 prefixCarry(BetaCircuit& c, const std::vector<u32>& g, const std::vector<u32>& p, u64 n) {
    // Brent-Kung reduction tree over positions [0, n): returns G[0..n-1].
    // (G_hi, P_hi) o (G_lo, P_lo) = (G_hi ^ (P_hi & G_lo), P_hi & P_lo); the
    // lowest range of every level never needs its P.
    struct GP {
        u32 G, P;
    };
    std::vector<GP> items(n);
    for (u64 i = 0; i < n; ++i) items[i] = {g[i], p[i]};
    while (items.size() > 1) {
        std::vector<GP> next;
        for (size_t j = 0; j < items.size(); j += 2) {
            if (j + 1 == items.size()) {
                next.push_back(items[j]);
                continue;
            }
            const GP& lo = items[j];
            const GP& hi = items[j + 1];
            u32 t = c.addGate(hi.P, lo.G, GateType::And);
            u32 G = c.addGate(hi.G, t, GateType::Xor);
            u32 P = j ? c.addGate(hi.P, lo.P, GateType::And) : ~0u;
            next.push_back({G, P});
        }
        items.swap(next);
    }
    return items[0].G;
}

u32 msbOfAdd(BetaCircuit& c, const BetaBundle& a, const BetaBundle& b) {
    const u64 n = a.size();
    if (b.size() != n || n == 0) throw std::runtime_error("msbOfAdd: sizes");
    u32 pTop = c.addGate(a[n - 1], b[n - 1], GateType::Xor);
    if (n == 1) return pTop;
    std::vector<u32> g(n - 1), p(n - 1);
    for (u64 i = 0; i + 1 < n; ++i) {
        g[i] = c.addGate(a[i], b[i], GateType::And);
        p[i] = c.addGate(a[i], b[i], GateType::Xor);
    }
    u32 carry = prefixCarry(c, g, p, n - 1);
    return c.addGate(pTop, carry, GateType::Xor);
}

u32 lessThanSigned(BetaCircuit& c, const BetaBundle& a, const BetaBundle& b) {
    // a < b  <=>  bit n of the (n+1)-bit sign extension of a + ~b + 1 is set:
    // lt = ~(a_{n-1} ^ b_{n-1} ^ carry_out(a + ~b + 1))
    const u64 n = a.size();
    if (b.size() != n || n == 0) throw std::runtime_error("lessThan: sizes");
    std::vector<u32> g(n), p(n);
    for (u64 i = 0; i < n; ++i) {
        g[i] = c.addGate(b[i], a[i], GateType::na_And);  // a & ~b
        p[i] = c.addGate(a[i], b[i], GateType::Nxor);    // a ^ ~b
    }
    g[0] = c.addGate(g[0], p[0], GateType::Xor);  // carry-in 1 folded into position 0
    u32 cout = prefixCarry(c, g, p, n);
    u32 s = c.addGate(a[n - 1], b[n - 1], GateType::Xor);
    return c.addGate(s, cout, GateType::Nxor);
}

BetaBundle add(BetaCircuit& c, const BetaBundle& a, const BetaBundle& b, bool subtract) {
    // Sklansky parallel prefix: after level k, position i holds the group
    // (G, P) of [block start, i] for blocks of 2^(k+1).
    const u64 n = a.size();
    if (b.size() != n || n == 0) throw std::runtime_error("add: sizes");
    std::vector<u32> G(n), P(n);
    for (u64 i = 0; i < n; ++i) {
        if (subtract) {
            G[i] = c.addGate(b[i], a[i], GateType::na_And);
            P[i] = c.addGate(a[i], b[i], GateType::Nxor);
        } else {
            G[i] = c.addGate(a[i], b[i], GateType::And);
            P[i] = c.addGate(a[i], b[i], GateType::Xor);
        }
    }
    const std::vector<u32> p0 = P;
    if (subtract) G[0] = c.addGate(G[0], P[0], GateType::Xor);
    for (u64 k = 0; (1ull << k) < n; ++k) {
        std::vector<u32> G2 = G, P2 = P;
        for (u64 i = 0; i < n; ++i) {
            if (((i >> k) & 1) == 0) continue;
            const u64 j = ((i >> k) << k) - 1;
            u32 t = c.addGate(P[i], G[j], GateType::And);
            G2[i] = c.addGate(G[i], t, GateType::Xor);
            if ((i >> (k + 1)) != 0) P2[i] = c.addGate(P[i], P[j], GateType::And);
        }
        G.swap(G2);
        P.swap(P2);
    }
    BetaBundle s(n);
    s[0] = subtract ? c.addUnary(p0[0], GateType::Inv) : p0[0];
    for (u64 i = 1; i < n; ++i) s[i] = c.addGate(p0[i], G[i - 1], GateType::Xor);
    return s;
}

}  // namespace circuits

// ----------------------------------------------------------------- library
BetaCircuit* CircuitLibrary::get(const std::string& name, u64 key) {
    auto it = mCirMap.find({name, key});
    return it == mCirMap.end() ? nullptr : it->second.get();
}

#define LIB_CACHED(name, key, ...)                                     \
    do {                                                              \
        if (auto* c_ = get(name, key)) return c_;                     \
        auto cd = std::make_unique<BetaCircuit>();                    \
        BetaCircuit& c = *cd;                                         \
        __VA_ARGS__;                                                  \
        c.levelByAndDepth();                                          \
        BetaCircuit* r_ = cd.get();                                   \
        mCirMap[{name, key}] = std::move(cd);                         \
        return r_;                                                    \
    } while (0)

BetaCircuit* CircuitLibrary::int_comp_helper(u64 size) {
    LIB_CACHED("int_comp_helper", size, {
        auto a = c.addInputBundle((u32)size);
        auto b = c.addInputBundle((u32)size);
        c.addOutputBundle({circuits::msbOfAdd(c, a, b)});
    });
}

BetaCircuit* CircuitLibrary::int_int_lt(u64 size) {
    LIB_CACHED("int_int_lt", size, {
        auto a = c.addInputBundle((u32)size);
        auto b = c.addInputBundle((u32)size);
        c.addOutputBundle({circuits::lessThanSigned(c, a, b)});
    });
}

BetaCircuit* CircuitLibrary::int_eq(u64 size) {
    LIB_CACHED("int_eq", size, {
        auto a = c.addInputBundle((u32)size);
        auto b = c.addInputBundle((u32)size);
        std::vector<u32> e(size);
        for (u64 i = 0; i < size; ++i) e[i] = c.addGate(a[i], b[i], GateType::Nxor);
        while (e.size() > 1) {
            std::vector<u32> n;
            for (size_t j = 0; j + 1 < e.size(); j += 2) n.push_back(c.addGate(e[j], e[j + 1], GateType::And));
            if (e.size() & 1) n.push_back(e.back());
            e.swap(n);
        }
        c.addOutputBundle({e[0]});
    });
}

BetaCircuit* CircuitLibrary::int_int_add(u64 size) {
    LIB_CACHED("int_int_add", size, {
        auto a = c.addInputBundle((u32)size);
        auto b = c.addInputBundle((u32)size);
        c.addOutputBundle(circuits::add(c, a, b, false));
    });
}

BetaCircuit* CircuitLibrary::int_int_sub(u64 size) {
    LIB_CACHED("int_int_sub", size, {
        auto a = c.addInputBundle((u32)size);
        auto b = c.addInputBundle((u32)size);
        c.addOutputBundle(circuits::add(c, a, b, true));
    });
}

BetaCircuit* CircuitLibrary::int_int_bitwiseAnd(u64 size) {
    LIB_CACHED("int_int_bitwiseAnd", size, {
        auto a = c.addInputBundle((u32)size);
        auto b = c.addInputBundle((u32)size);
        BetaBundle o(size);
        for (u64 i = 0; i < size; ++i) o[i] = c.addGate(a[i], b[i], GateType::And);
        c.addOutputBundle(o);
    });
}

BetaCircuit* CircuitLibrary::int_int_bitwiseOr(u64 size) {
    LIB_CACHED("int_int_bitwiseOr", size, {
        auto a = c.addInputBundle((u32)size);
        auto b = c.addInputBundle((u32)size);
        BetaBundle o(size);
        for (u64 i = 0; i < size; ++i) o[i] = c.addGate(a[i], b[i], GateType::Or);
        c.addOutputBundle(o);
    });
}

BetaCircuit* CircuitLibrary::bits_nor_helper(u64 size) {
    LIB_CACHED("bits_nor_helper", size, {
        auto a = c.addInputBundle((u32)size);
        auto b = c.addInputBundle((u32)size);
        BetaBundle o(size);
        for (u64 i = 0; i < size; ++i) o[i] = c.addGate(a[i], b[i], GateType::Nor);
        c.addOutputBundle(o);
    });
}

BetaCircuit* CircuitLibrary::int_Sh3Piecewise_helper(u64 size, u64 T) {
    LIB_CACHED("int_Sh3Piecewise_helper", size * 1024 + T, {
        if (T == 0) throw std::runtime_error("piecewise helper needs a threshold");
        std::vector<BetaBundle> aa(T);
        for (auto& a : aa) a = c.addInputBundle((u32)size);
        auto b = c.addInputBundle((u32)size);
        std::vector<u32> thr(T);
        for (u64 t = 0; t < T; ++t) thr[t] = circuits::msbOfAdd(c, aa[t], b);  // [x < t_t]
        c.addOutputBundle({thr[0]});
        for (u64 t = 1; t < T; ++t) c.addOutputBundle({c.addGate(thr[t - 1], thr[t], GateType::na_And)});
        c.addOutputBundle({c.addUnary(thr[T - 1], GateType::Inv)});
    });
}

BetaCircuit* CircuitLibrary::cmp_swap(u64 size) {
    LIB_CACHED("cmp_swap", size, {
        auto a = c.addInputBundle((u32)size);
        auto b = c.addInputBundle((u32)size);
        u32 lt = circuits::lessThanSigned(c, a, b);
        BetaBundle mn(size), mx(size);
        for (u64 i = 0; i < size; ++i) {
            u32 d = c.addGate(a[i], b[i], GateType::Xor);
            u32 m = c.addGate(lt, d, GateType::And);
            mn[i] = c.addGate(b[i], m, GateType::Xor);  // lt ? a : b
            mx[i] = c.addGate(a[i], m, GateType::Xor);  // lt ? b : a
        }
        c.addOutputBundle(mn);
        c.addOutputBundle(mx);
    });
}

namespace {
// cryptoTools GateType codes (truth tables, bit a + 2b)
constexpr u8 kTruthTable[8] = {6, 9, 8, 14, 1, 4, 10, 5};  // indexed by GateType
GateType fromTruthTable(u8 t) {
    for (u32 i = 0; i < 8; ++i)
        if (kTruthTable[i] == t) return (GateType)i;
    throw std::runtime_error("BetaCircuit::readBin: unsupported gate type " + std::to_string(t));
}
template <class T>
void put(std::ostream& o, T v) {
    o.write(reinterpret_cast<const char*>(&v), sizeof v);
}
template <class T>
T get(std::istream& in) {
    T v{};
    in.read(reinterpret_cast<char*>(&v), sizeof v);
    if (!in) throw std::runtime_error("BetaCircuit::readBin: truncated circuit file");
    return v;
}
}  // namespace

void BetaCircuit::writeBin(std::ostream& out) const {
    u64 nonXor = 0;
    for (const auto& g : mGates) nonXor += isAndType(g.type);
    put<u64>(out, mWireCount);
    put<u64>(out, nonXor);
    for (const auto* bundles : {&mInputs, &mOutputs}) {
        put<u64>(out, bundles->size());
        for (const auto& b : *bundles) {
            put<u64>(out, b.size());
            out.write(reinterpret_cast<const char*>(b.data()), (std::streamsize)(4 * b.size()));
        }
    }
    put<u64>(out, mGates.size());
    for (const auto& g : mGates) {
        put<u32>(out, g.in0);
        put<u32>(out, g.in1);
        put<u32>(out, g.out);
        const u8 rec[4] = {kTruthTable[(u32)g.type], 0, 0, 0};
        out.write(reinterpret_cast<const char*>(rec), 4);
    }
    if (!out) throw std::runtime_error("BetaCircuit::writeBin: write failed");
}

void BetaCircuit::readBin(std::istream& in) {
    BetaCircuit c;
    const u64 wires = get<u64>(in), nonXor = get<u64>(in);
    if (wires > (1ull << 31)) throw std::runtime_error("BetaCircuit::readBin: wire count out of range");
    c.mWireCount = (u32)wires;
    std::vector<u8> defined(wires, 0);
    for (auto* bundles : {&c.mInputs, &c.mOutputs}) {
        const u64 nb = get<u64>(in);
        if (nb > wires + 1) throw std::runtime_error("BetaCircuit::readBin: bundle count out of range");
        bundles->resize(nb);
        for (auto& b : *bundles) {
            const u64 n = get<u64>(in);
            if (n > wires) throw std::runtime_error("BetaCircuit::readBin: bundle size out of range");
            b.resize(n);
            for (auto& w : b) {
                w = get<u32>(in);
                if (w >= wires) throw std::runtime_error("BetaCircuit::readBin: wire index out of range");
            }
        }
    }
    for (const auto& b : c.mInputs)
        for (u32 w : b) defined[w] = 1;
    const u64 ng = get<u64>(in);
    if (ng > wires) throw std::runtime_error("BetaCircuit::readBin: gate count out of range");
    c.mGates.resize(ng);
    u64 ands = 0;
    for (auto& g : c.mGates) {
        g.in0 = get<u32>(in);
        g.in1 = get<u32>(in);
        g.out = get<u32>(in);
        const u32 rec = get<u32>(in);
        g.type = fromTruthTable((u8)(rec & 0xff));
        const bool unary = g.type == GateType::a || g.type == GateType::Inv;
        if (g.in0 >= wires || g.in1 >= wires || g.out >= wires)
            throw std::runtime_error("BetaCircuit::readBin: gate wire out of range");
        if (!defined[g.in0] || (!unary && !defined[g.in1]))
            throw std::runtime_error("BetaCircuit::readBin: gate input used before it is defined");
        if (defined[g.out]) throw std::runtime_error("BetaCircuit::readBin: wire defined twice");
        defined[g.out] = 1;
        ands += isAndType(g.type);
    }
    if (ands != nonXor) throw std::runtime_error("BetaCircuit::readBin: non-XOR gate count mismatch");
    for (const auto& b : c.mOutputs)
        for (u32 w : b)
            if (!defined[w]) throw std::runtime_error("BetaCircuit::readBin: output wire never defined");
    mWireCount = c.mWireCount;
    mGates = std::move(c.mGates);
    mInputs = std::move(c.mInputs);
    mOutputs = std::move(c.mOutputs);
    mLevelGates.clear();
    mLevelCounts.clear();
    mLevelAndCounts.clear();
    mLevelBatches.clear();
    mBatchGates.clear();
    mBatchZRow.clear();
    mBatchSendRow.clear();
    mAndCount = 0;
    mSerial = g_circuitSerial++;  // a new circuit for the device caches
}

BetaCircuit* CircuitLibrary::byName(const std::string& n, u64 size, u64 param) {
    // "bin:<path>": a circuit file (BetaCircuit::readBin), levelized on load
    if (n.compare(0, 4, "bin:") == 0) {
        auto key = std::make_pair(n, (u64)0);
        auto& slot = mCirMap[key];
        if (!slot) {
            std::ifstream f(n.substr(4), std::ios::binary);
            if (!f) throw std::runtime_error("cannot open circuit file " + n.substr(4));
            auto c = std::make_unique<BetaCircuit>();
            c->readBin(f);
            c->levelByAndDepth();
            slot = std::move(c);
        }
        return slot.get();
    }
    if (n == "int_comp_helper") return int_comp_helper(size);
    if (n == "int_int_lt") return int_int_lt(size);
    if (n == "int_eq") return int_eq(size);
    if (n == "int_int_add") return int_int_add(size);
    if (n == "int_int_sub") return int_int_sub(size);
    if (n == "int_int_bitwiseAnd") return int_int_bitwiseAnd(size);
    if (n == "int_int_bitwiseOr") return int_int_bitwiseOr(size);
    if (n == "bits_nor_helper") return bits_nor_helper(size);
    if (n == "cmp_swap") return cmp_swap(size);
    if (n == "int_Sh3Piecewise_helper") return int_Sh3Piecewise_helper(size, param);
    throw std::runtime_error("unknown circuit " + n);
}

}  // namespace aby3
