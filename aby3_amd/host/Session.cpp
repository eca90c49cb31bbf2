// C entry points (include/aby3.h): three persistent party threads running a
// job of the hot path, for bench.py and the Python tests.
#include "Link.h"
#include <aby3.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <deque>
#include <fstream>
#include <functional>
#include <numeric>
#include <thread>
#include "Basic.h"
#include "Sh3Converter.h"
#include "aby3ML.h"

namespace aby3 {

namespace {
thread_local std::string t_err;

// one party per process on a shared GPU: the binary engine's AND-mask draws
// on a second stream of the process (ABY3_PARTY_DRAW_STREAM=1, A/B runs)
static bool partyDrawStream() {
    static const bool on = [] {
        const char* e = getenv("ABY3_PARTY_DRAW_STREAM");
        return e && e[0] == '1';
    }();
    return on;
}

// the share-draw workgroup cap of a party alone in its process
// (aby3g_set_draw_workgroups; ABY3_PARTY_DRAW_WGS for A/B runs)
static int partyDrawWorkgroups() {
    static const int n = [] {
        // 256 (one per CU), as beside co-located parties: 512 and 1024
        // measured no faster for C3 / C5 as three processes on one GPU
        // (0.359 / 0.363-0.367 against 0.355-0.360 ms; C5 70.7-71.4 against 69.7-71.0 ms)
        const char* e = getenv("ABY3_PARTY_DRAW_WGS");
        const int v = e && *e ? atoi(e) : 256;
        return v >= 1 && v <= 4096 ? v : 256;
    }();
    return n;
}

// co-located parties plan each share GEMM for 1/k of the CUs (k = 3 by
// default; ABY3_GEMM_SHARING=1: full-chip plans, for A/B runs)
static int colocatedGemmSharing() {
    static const int k = [] {
        const char* e = getenv("ABY3_GEMM_SHARING");
        const int v = e && *e ? atoi(e) : 3;
        return v >= 1 && v <= 8 ? v : 3;
    }();
    return k;
}

struct PartyCtx {
    int idx = 0;
    Sh3Runtime rt;
    Sh3Encryptor enc;
    Sh3Evaluator eval;
    bool ownProcess = false;  // one party per process (aby3h_party_create)
    // One party per process, during setup: drain the stream and name the step
    // if its work failed -- an asynchronous device fault otherwise surfaces in
    // some later call (party 1's fault reported by a host copy).
    void checkpoint(const char* step) {
        if (!ownProcess) return;
        try {
            rt.gpu().sync();
        } catch (const std::exception& e) {
            throw std::runtime_error(std::string("after ") + step + ": " + e.what());
        }
    }
};

u64 xorshift(u64& x) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    return x;
}
i64Matrix randomMat(u64 r, u64 c, u64 seed, i64 bound) {
    i64Matrix m(r, c);
    u64 x = seed * 0x9E3779B97F4A7C15ull + 12345;
    for (auto& v : m.mData) v = bound ? (i64)(xorshift(x) % (2 * (u64)bound)) - bound : (i64)xorshift(x);
    return m;
}

struct Job {
    virtual ~Job() = default;
    virtual void setup(PartyCtx& p) = 0;
    virtual void step(PartyCtx& p) = 0;
    virtual bool check(PartyCtx&) { return true; }
    // completes every step issued so far (jobs that keep several in flight)
    virtual void drain(PartyCtx&) {}
    virtual void info(double* out) = 0;
    // party i's result matrix of the last step (both shares), for digests
    virtual const SharedMat* result(int) const { return nullptr; }
    // parties seeded as aby3ML::init (aby3ML.cpp:4-17) instead of the unit tests' toBlock(c, i)
    virtual bool mlSeeds() const { return false; }
};

// ---- C2 / C1: asyncMul (+ truncation) ------------------------------------
struct MulJob : Job {
    u64 M, K, N, D;
    MulMode mode;
    bool trunc;
    // products in flight per party: 1 = each step's product completes before
    // the next is issued; 2 = step s issues product s, then waits for product
    // s - 1 (independent products through the runtime's task graph, each
    // into its own output matrix), so one product's reshare round overlaps
    // the next one's share GEMM on the party's stream
    u64 inflight;
    // rows [r0, r1) of the M-row product (a row split): A's
    // slice shared and multiplied with the whole product's randomness taken
    u64 r0 = 0, r1 = 0;
    i64Matrix a, b;
    si64Matrix A[3], B[3], C[3][2];
    std::deque<Sh3Task> pending[3];
    int slot[3] = {0, 0, 0};
    int last[3] = {0, 0, 0};
    MulJob(u64 m, u64 k, u64 n, u64 d, MulMode md, bool t, u64 inf = 1, u64 shard = 0, u64 shards = 1)
        : M(m), K(k), N(n), D(d), mode(md), trunc(t), inflight(inf < 1 ? 1 : inf > 2 ? 2 : inf) {
        if (shards < 1 || shard >= shards)
            throw std::invalid_argument("row split: shard " + std::to_string(shard) + " of " + std::to_string(shards));
        if (shards > 1 && (mode != MulMode::Gemm || !trunc))
            throw std::invalid_argument("row split: the truncated GEMM product only");
        r0 = M * shard / shards;
        r1 = M * (shard + 1) / shards;
        const u64 br = mode == MulMode::Gemm ? K : M, bc = mode == MulMode::Gemm ? N : K;
        // fixed-point operands in [-8, 8) * 2^D
        const i64 bound = trunc ? (8ll << D) : 0;
        a = randomMat(M, K, 1, bound);
        b = randomMat(br, bc, 2, bound);
    }
    bool split() const { return r1 - r0 != M; }
    void setup(PartyCtx& p) override {
        const u64 br = mode == MulMode::Gemm ? K : M, bc = mode == MulMode::Gemm ? N : K;
        A[p.idx].resize(r1 - r0, K);
        B[p.idx].resize(br, bc);
        if (split()) {
            // this slice's rows of A (the whole matrix's draws taken), all of B
            if (p.idx == 0) {
                i64Matrix rows(r1 - r0, K);
                if (r1 > r0) std::memcpy(rows.data(), a.data() + r0 * K, (r1 - r0) * K * sizeof(i64));
                p.enc.localIntMatrixRows(p.rt, rows, A[0], r0, M).get();
                p.enc.localIntMatrix(p.rt, b, B[0]).get();
            } else {
                p.enc.remoteIntMatrixRows(p.rt, A[p.idx], r0, M).get();
                p.enc.remoteIntMatrix(p.rt, B[p.idx]).get();
            }
        } else if (p.idx == 0) {
            p.enc.localIntMatrix(p.rt, a, A[0]).get();
            p.enc.localIntMatrix(p.rt, b, B[0]).get();
        } else {
            p.enc.remoteIntMatrix(p.rt, A[p.idx]).get();
            p.enc.remoteIntMatrix(p.rt, B[p.idx]).get();
        }
    }
    void step(PartyCtx& p) override {
        const int i = (int)p.idx;
        si64Matrix& c = C[i][slot[i]];
        last[i] = slot[i];
        slot[i] = (slot[i] + 1) % (int)inflight;
        pending[i].push_back(split()  ? p.eval.asyncMulRows(p.rt, A[i], B[i], c, D, r0, M)
                             : trunc ? p.eval.asyncMul(p.rt, A[i], B[i], c, D, mode)
                                     : p.eval.asyncMul(p.rt, A[i], B[i], c, mode));
        if (pending[i].size() >= inflight) {
            pending[i].front().get();
            pending[i].pop_front();
        }
    }
    void drain(PartyCtx& p) override {
        auto& q = pending[p.idx];
        while (!q.empty()) {
            q.front().get();
            q.pop_front();
        }
    }
    bool check(PartyCtx& p) override {
        drain(p);
        i64Matrix r;
        p.enc.revealAll(p.rt, C[p.idx][last[p.idx]], r).get();
        if (p.idx != 0) return true;
        // spot-check 64 entries against the plaintext product
        u64 x = 99;
        for (int t = 0; t < 64 && r1 > r0; ++t) {
            const u64 i = r0 + xorshift(x) % (r1 - r0), j = xorshift(x) % N;
            __int128 s = 0;
            if (mode == MulMode::Gemm)
                for (u64 k = 0; k < K; ++k) s += (__int128)a(i, k) * b(k, j);
            else
                s = (__int128)a(i, j) * b(i, j);
            const i64 exact = (i64)(u64)s;
            const i64 got = r(i - r0, j);
            if (trunc) {
                const i64 e = (i64)(s >> D);
                if (got - e > 1 || e - got >= 4) return false;
            } else if (got != exact) {
                return false;
            }
        }
        return true;
    }
    void info(double* o) override {
        o[ABY3H_INFO_MULTS_PER_STEP] = mode == MulMode::Gemm ? (double)(r1 - r0) * N * K : (double)M * N;
        o[ABY3H_INFO_GEMM_INT8_OPS] = mode == MulMode::Gemm ? 144.0 * M * N * K : 0;
    }
    const SharedMat* result(int i) const override { return &C[i][last[i]]; }
};

// gate-kernel algorithmic bytes per padded word
double gateBytes(const BetaCircuit& c) {
    double b = 0;
    for (const auto& g : c.mGates) {
        switch (g.type) {
            case GateType::a:
            case GateType::Inv: b += 32; break;          // 2 reads, 2 writes
            case GateType::Xor:
            case GateType::Nxor: b += 48; break;         // 4 reads, 2 writes
            default: b += 56 + 16; break;                 // 4 reads + z, share 0 + send; unpack 8 + 8
        }
    }
    return b;
}

// ---- C3: fetch_msb / cipher_gt over `rows` values -------------------------
struct MsbJob : Job {
    u64 rows;
    // rows [r0, r1) of the comparison (a row split): slice
    // boundaries at multiples of 2048 rows (the engine's row padding)
    u64 r0 = 0, r1 = 0;
    i64Matrix a, b;
    si64Matrix A[3], B[3];
    sbMatrix R[3];
    CircuitLibrary lib;
    explicit MsbJob(u64 r, u64 shard = 0, u64 shards = 1) : rows(r) {
        if (shards < 1 || shard >= shards)
            throw std::invalid_argument("row split: shard " + std::to_string(shard) + " of " + std::to_string(shards));
        auto edge = [&](u64 k) { return k == shards ? rows : rows * k / shards / 2048 * 2048; };
        r0 = edge(shard);
        r1 = edge(shard + 1);
        a = randomMat(rows, 1, 3, 0);
        b = randomMat(rows, 1, 4, 0);
    }
    bool split() const { return r1 - r0 != rows; }
    void setup(PartyCtx& p) override {
        A[p.idx].resize(r1 - r0, 1);
        B[p.idx].resize(r1 - r0, 1);
        if (p.idx == 0) {
            i64Matrix as(r1 - r0, 1), bs(r1 - r0, 1);
            for (u64 i = r0; i < r1; ++i) as(i - r0, 0) = a(i, 0), bs(i - r0, 0) = b(i, 0);
            p.enc.localIntMatrixRows(p.rt, as, A[0], r0, rows).get();
            p.enc.localIntMatrixRows(p.rt, bs, B[0], r0, rows).get();
        } else {
            p.enc.remoteIntMatrixRows(p.rt, A[p.idx], r0, rows).get();
            p.enc.remoteIntMatrixRows(p.rt, B[p.idx], r0, rows).get();
        }
    }
    void step(PartyCtx& p) override {
        if (split())
            cipher_gt_rows(p.idx, A[p.idx], B[p.idx], R[p.idx], p.eval, p.rt, r0, rows);
        else
            cipher_gt(p.idx, A[p.idx], B[p.idx], R[p.idx], p.eval, p.rt);
    }
    const SharedMat* result(int i) const override { return &R[i]; }
    bool check(PartyCtx& p) override {
        i64Matrix r;
        p.enc.revealAll(p.rt, R[p.idx], r).get();
        if (p.idx != 0) return true;
        for (u64 i = r0; i < r1; ++i)
            if ((r(i - r0, 0) & 1) != (i64)(((u64)b(i, 0) - (u64)a(i, 0)) >> 63)) return false;
        return true;
    }
    void info(double* o) override {
        BetaCircuit* c = lib.int_comp_helper(64);
        const u64 n = r1 - r0;
        const double words = std::ceil(n / 64.0), padded = 32.0 * ((n + 2047) / 2048);
        o[ABY3H_INFO_MULTS_PER_STEP] = c->mAndCount * words;
        o[ABY3H_INFO_AND_WORDS] = c->mAndCount * words;
        o[ABY3H_INFO_GATE_WORDS] = c->mGates.size() * words;
        o[ABY3H_INFO_GATE_BYTES] = gateBytes(*c) * padded;
    }
};

// ---- share conversions (Sh3Converter.cpp) --------------------------------
// seeds of the reference's converter tests (Sh3ConverterTests.cpp:314-316)
struct ConvParty {
    Sh3ShareGen gen;
    Sh3Converter conv;
    void init(PartyCtx& p) {
        gen.init(toBlock(0, (u64)p.idx + 1), toBlock(0, (u64)(p.idx + 1) % 3 + 1));
        conv.init(p.rt, gen);
    }
};

// toBinaryMatrix(si64 -> sb) over rows x 1 values: one step = resharing +
// 64-bit adder circuit (Sh3Converter.cpp:61-207)
struct A2bJob : Job {
    u64 rows;
    i64Matrix a;
    si64Matrix A[3];
    sbMatrix R[3];
    ConvParty cp[3];
    explicit A2bJob(u64 r) : rows(r) { a = randomMat(rows, 1, 5, 0); }
    void setup(PartyCtx& p) override {
        A[p.idx].resize(rows, 1);
        if (p.idx == 0)
            p.enc.localIntMatrix(p.rt, a, A[0]).get();
        else
            p.enc.remoteIntMatrix(p.rt, A[p.idx]).get();
        cp[p.idx].init(p);
    }
    void step(PartyCtx& p) override { cp[p.idx].conv.toBinaryMatrix(p.rt, A[p.idx], R[p.idx]).get(); }
    const SharedMat* result(int i) const override { return &R[i]; }
    bool check(PartyCtx& p) override {
        i64Matrix r;
        p.enc.revealAll(p.rt, R[p.idx], r).get();
        return p.idx != 0 || r.mData == a.mData;
    }
    void info(double* o) override {
        BetaCircuit* c = cp[0].conv.arithToBinCircuit(64);
        const double words = std::ceil(rows / 64.0), padded = 32.0 * ((rows + 2047) / 2048);
        o[ABY3H_INFO_MULTS_PER_STEP] = c->mAndCount * words;
        o[ABY3H_INFO_AND_WORDS] = c->mAndCount * words;
        o[ABY3H_INFO_GATE_WORDS] = c->mGates.size() * words;
        o[ABY3H_INFO_GATE_BYTES] = gateBytes(*c) * padded;
    }
};

// bitInjection(sb -> si64) of rows x bits: one step = the 3-party OTs of
// every bit (Sh3Converter.cpp:209-370)
struct BitInjJob : Job {
    u64 rows, bits;
    i64Matrix a;
    sbMatrix A[3];
    si64Matrix R[3];
    ConvParty cp[3];
    BitInjJob(u64 r, u64 b) : rows(r), bits(b) {
        if (!bits || bits > 64) throw std::runtime_error("bitinj job: 1..64 bits");
        a = randomMat(rows, 1, 6, 0);
        if (bits < 64)
            for (auto& v : a.mData) v &= (i64)((1ull << bits) - 1);
    }
    void setup(PartyCtx& p) override {
        A[p.idx].resize(rows, bits);
        if (p.idx == 0)
            p.enc.localBinMatrix(p.rt, a, A[0]).get();
        else
            p.enc.remoteBinMatrix(p.rt, A[p.idx]).get();
        cp[p.idx].init(p);
    }
    void step(PartyCtx& p) override { cp[p.idx].conv.bitInjection(p.rt, A[p.idx], R[p.idx]).get(); }
    const SharedMat* result(int i) const override { return &R[i]; }
    bool check(PartyCtx& p) override {
        i64Matrix r;
        p.enc.revealAll(p.rt, R[p.idx], r).get();
        if (p.idx != 0) return true;
        for (u64 i = 0; i < rows; ++i)
            for (u64 j = 0; j < bits; ++j)
                if ((u64)r(i, j) != (((u64)a(i, 0) >> j) & 1)) return false;
        return true;
    }
    void info(double* o) override {
        // one OT-based bit product per bit (the metric's unit for asyncMul(si64, sb))
        o[ABY3H_INFO_MULTS_PER_STEP] = (double)rows * bits;
    }
};

// ---- C4: one logistic-regression SGD iteration ----------------------------
// The reference's driver (main-logistic.cpp:82-140, Regression.h:249-293):
// LogisticModelGen data, aby3ML::init seeds, getSubset mini-batches.
// sample = 0: the mini-batches of the first kBatches iterations are drawn at
// construction and kept resident (an iteration is the protocol alone);
// sample = 1: every step draws its batch with getSubset inside the step
// (DeviceBatchSampler), as SGD_Logistic's loop does (Regression.h:249-253).
// ABY3_LR_PREFETCH=0: no prefetch of the next batch's rows (A/B runs)
static bool nextBatchPrefetch() {
    static const bool on = [] {
        const char* e = getenv("ABY3_LR_PREFETCH");
        return !e || e[0] != '0';
    }();
    return on;
}

struct LrJob : Job {
    static constexpr u64 kBatches = 8192;  // mini-batches precomputed (and resident) per session
    u64 n, d, B, D, aB, sample;
    i64Matrix X, Y, w0;
    si64Matrix sX[3], sY[3], sW[3];
    std::unique_ptr<aby3ML> ml[3];
    SgdState st[3];
    std::vector<u32> batches;  // [kBatches][B], getSubset order (sample = 0)
    DeviceBuffer dbatch[3];     // the same, resident per party
    std::unique_ptr<DeviceBatchSampler> sampler[3];  // sample = 1
    u64 iter[3] = {0, 0, 0};
    LrJob(u64 n_, u64 d_, u64 b_, u64 D_, u64 aB_, u64 sample_)
        : n(n_), d(d_), B(b_), D(D_), aB(aB_), sample(sample_) {
        if (!n || !d || !B || B > n) throw std::runtime_error("lr job: need 0 < batch <= rows");
        logisticModelGen(logisticModel(d), n, D, X, Y);
        w0.resize(d, 1);
        if (!sample) batches = drawBatches(kBatches);
    }
    // the first `iters` mini-batches of getSubset, [iters][B]
    std::vector<u32> drawBatches(u64 iters) const {
        BatchSampler s(n);
        std::vector<u64> b(B);
        std::vector<u32> out(iters * B);
        for (u64 t = 0; t < iters; ++t) {
            s.next(b);
            for (u64 i = 0; i < B; ++i) out[t * B + i] = (u32)b[i];
        }
        return out;
    }
    bool mlSeeds() const override { return true; }
    void setup(PartyCtx& p) override {
        sX[p.idx].resize(n, d);
        sY[p.idx].resize(n, 1);
        sW[p.idx].resize(d, 1);
        if (p.idx == 0) {  // localFixedMatrix of train_data, train_label, W2 (main-logistic.cpp:117-121)
            p.enc.localIntMatrix(p.rt, X, sX[0]).get();
            p.checkpoint("sharing X");
            p.enc.localIntMatrix(p.rt, Y, sY[0]).get();
            p.checkpoint("sharing Y");
            p.enc.localIntMatrix(p.rt, w0, sW[0]).get();
            p.checkpoint("sharing w");
        } else {
            p.enc.remoteIntMatrix(p.rt, sX[p.idx]).get();
            p.checkpoint("receiving X");
            p.enc.remoteIntMatrix(p.rt, sY[p.idx]).get();
            p.checkpoint("receiving Y");
            p.enc.remoteIntMatrix(p.rt, sW[p.idx]).get();
            p.checkpoint("receiving w");
        }
        ml[p.idx] = std::make_unique<aby3ML>(p.rt, p.enc, p.eval, D);
        if (sample) {
            sampler[p.idx] = std::make_unique<DeviceBatchSampler>(p.rt.gpu(), n, B);
        } else {
            dbatch[p.idx].reset(p.rt.gpu(), batches.size() * 4);
            toDevice(dbatch[p.idx].data(), batches.data(), batches.size() * 4, p.rt.gpu());
        }
        p.checkpoint("batch indices");
    }
    void step(PartyCtx& p) override {
        const u64 t = iter[p.idx]++;
        const u32* idx;
        if (sample) {
            idx = sampler[p.idx]->next();  // getSubset + the batch's indices on the device
        } else {
            if (t >= kBatches) throw std::runtime_error("lr job: more iterations than precomputed mini-batches");
            idx = dbatch[p.idx].as<u32>() + t * B;
            // resident batches: the next one is known (its rows prefetched)
            st[p.idx].nextBatch = t + 1 < kBatches && nextBatchPrefetch() ? idx + B : nullptr;
        }
        sgdLogisticStep(*ml[p.idx], sX[p.idx], sY[p.idx], sW[p.idx], idx, B, aB, st[p.idx]);
    }
    // Smoke check of the revealed model against a plaintext fixed-point
    // restatement of the same iterations (floor shifts as Sh3FixedPoint.h:
    // 200-210, the sigmoid of aby3ML.h:121-139). The protocol's truncation is
    // off by an ulp now and then, and a product that lands on the other side
    // of a sigmoid threshold (+-0.5) changes that sample's error by up to 1,
    // so the two models drift apart over many iterations: the check bounds the
    // drift relative to the model and requires the same direction. Bit-exact
    // share-level parity with the oracle is tests/test_lr_driver.py.
    bool check(PartyCtx& p) override {
        i64Matrix r;
        p.enc.revealAll(p.rt, sW[p.idx], r).get();
        if (p.idx != 0) return true;
        std::vector<i64> w(w0.mData);
        const i64 half = 1ll << (D - 1), one = 1ll << D;
        const std::vector<u32> drawn = sample ? drawBatches(iter[0]) : std::vector<u32>();
        const std::vector<u32>& bl = sample ? drawn : batches;
        for (u64 t = 0; t < iter[0]; ++t) {
            const u32* rows = bl.data() + t * B;
            std::vector<i64> err(B);
            for (u64 i = 0; i < B; ++i) {
                i64 xw = 0;
                for (u64 j = 0; j < d; ++j) xw += X(rows[i], j) * w[j];
                xw >>= D;
                const i64 f = xw < -half ? 0 : (xw < half ? half + xw : one);
                err[i] = f - Y(rows[i], 0);
            }
            for (u64 j = 0; j < d; ++j) {
                i64 u = 0;
                for (u64 i = 0; i < B; ++i) u += X(rows[i], j) * err[i];
                w[j] -= u >> (D + aB);
            }
        }
        double maxW = 0, maxD = 0, dot = 0, n0 = 0, n1 = 0;
        for (u64 j = 0; j < d; ++j) {
            const double a = fromFixed(r.mData[j], D), b = fromFixed(w[j], D);
            maxW = std::max(maxW, std::abs(b));
            maxD = std::max(maxD, std::abs(a - b));
            dot += a * b;
            n0 += a * a;
            n1 += b * b;
        }
        const bool ok = maxD <= 0.25 * maxW + (double)(iter[0] + 1) / 1024.0 &&
                        (n1 == 0 || (n0 > 0 && dot / std::sqrt(n0 * n1) > 0.5));
        if (!ok)
            std::fprintf(stderr, "lr check: %llu iterations, max |dw| %.5f, max |w| %.5f, cos %.4f\n",
                         (unsigned long long)iter[0], maxD, maxW, n0 > 0 && n1 > 0 ? dot / std::sqrt(n0 * n1) : 0.0);
        return ok;
    }
    void info(double* o) override {
        o[ABY3H_INFO_MULTS_PER_STEP] = 2.0 * B * d;
        o[ABY3H_INFO_LR_FUSED] = (st[0].fused || st[1].fused || st[2].fused) ? 1 : 0;
        o[ABY3H_INFO_LR_SYS_SCOPE] = (st[0].fusedSysScope || st[1].fusedSysScope || st[2].fusedSysScope) ? 1 : 0;
    }
    const SharedMat* result(int i) const override { return &sW[i]; }
};

// ---- C5: odd-even merge sort of `keys` 64-bit keys ------------------------
struct SortJob : Job {
    u64 n;
    i64Matrix k;
    sbMatrix S[3], R[3];
    CircuitLibrary lib;
    MergeOrder order;
    explicit SortJob(u64 keys, u64 ord = 0) : n(keys), order(ord ? MergeOrder::Sequential : MergeOrder::Batched) {
        if (!n || n > (1ull << 20)) throw std::runtime_error("sort job: 1 .. 2^20 keys");
        // distinct keys below 2^63, the low 20 bits an index tag (tag_append,
        // BoolBasic.cpp:992-1004): signed and unsigned order agree
        k.resize(n, 1);
        u64 x = 7;
        for (u64 i = 0; i < n; ++i) k(i, 0) = (i64)(((xorshift(x) % (1ull << 43)) << 20) | i);
    }
    void setup(PartyCtx& p) override {
        S[p.idx].resize(n, 64);
        if (p.idx == 0)
            p.enc.localBinMatrix(p.rt, k, S[0]).get();
        else
            p.enc.remoteBinMatrix(p.rt, S[p.idx]).get();
    }
    void step(PartyCtx& p) override {
        odd_even_multi_merge(S[p.idx], std::vector<u64>(n, 1), R[p.idx], p.idx, p.eval, p.rt, order);
    }
    const SharedMat* result(int i) const override { return &R[i]; }
    // every key, in order: the revealed output equals std::sort of the input
    bool check(PartyCtx& p) override {
        i64Matrix r;
        p.enc.revealAll(p.rt, R[p.idx], r).get();
        if (p.idx != 0) return true;
        std::vector<i64> b(k.mData);
        std::sort(b.begin(), b.end());
        return r.mData == b;
    }
    void info(double* o) override {
        BetaCircuit* c = lib.cmp_swap(64);
        double andW = 0, gateW = 0, bytes = 0;
        for (u64 rows : multiMergeEvalRows(std::vector<u64>(n, 1), order == MergeOrder::Sequential)) {
            const double words = std::ceil(rows / 64.0), padded = 32.0 * ((rows + 2047) / 2048);
            andW += c->mAndCount * words;
            gateW += c->mGates.size() * words;
            bytes += gateBytes(*c) * padded;
        }
        o[ABY3H_INFO_MULTS_PER_STEP] = andW;
        o[ABY3H_INFO_AND_WORDS] = andW;
        o[ABY3H_INFO_GATE_WORDS] = gateW;
        o[ABY3H_INFO_GATE_BYTES] = bytes;
    }
};

}  // namespace

struct Session {
    std::unique_ptr<Job> job;
    std::thread th[3];
    std::vector<int> locals;  // the parties run by this process (all three, or one)
    std::mutex mu;
    std::condition_variable cv, done;
    // command: 0 idle, 1 run, 2 stop, 3 probe read, 4 probe reset, 5 check
    int cmd = 0;
    u64 gen = 0, steps = 0;
    int finished = 0;
    std::string err;
    double probeMs[8] = {0};
    u64 probeN[8] = {0};
    int probeFamily = 0;
    bool checkOk = true;
    u64 digests[3] = {0, 0, 0};
    std::vector<i64> results[3][2];  // command 8: each party's result shares on the host
    std::vector<CommPkg> comms;
    double hostEnqueueUs[3] = {0, 0, 0}, hostDrainUs[3] = {0, 0, 0}, hostRecvWaitUs[3] = {0, 0, 0};
    size_t poolCached[3] = {0, 0, 0};  // each party's cached pool bytes after its last run
    double hostApiUs[3] = {0, 0, 0}, hostApiCalls[3] = {0, 0, 0};
    double deviceWaitUs[3] = {0, 0, 0};  // in-kernel waits for peers per step (Gpu::waitUs)
    int devices[3] = {0, 0, 0};
    bool colocated = false;  // two or more parties on one device
    // co-located parties' shared draw stream per device (Gpu::SharedStream),
    // created once every local party has made its own stream
    std::map<int, std::shared_ptr<Gpu::SharedStream>> drawStreams;

    // Stream creation order. HIP maps streams onto GPU_MAX_HW_QUEUES hardware
    // queues in creation order, so with the three parties on one device the
    // order decides which streams share a queue. Parties create their
    // streams in turn (party 0 first), main and auxiliary together.
    std::mutex turnMu;
    std::condition_variable turnCv;
    int turnNext = 0;
    template <class F>
    void inTurn(int i, F&& f) {
        std::unique_lock<std::mutex> lk(turnMu);
        turnCv.wait(lk, [&] { return turnNext == i; });
        try {
            f();
        } catch (...) {
            ++turnNext;
            turnCv.notify_all();
            throw;
        }
        ++turnNext;
        turnCv.notify_all();
    }

    // One party per process, at close: drain this party's streams and
    // exchange a token with both neighbours before anything is torn down, so
    // that no process frees (or exits with) a staging slot or mailbox a peer
    // is still to open or read. A run that failed skips it (a peer may be gone).
    void leaveTogether(PartyCtx& p) {
        {
            std::lock_guard<std::mutex> lk(mu);
            if (!err.empty()) return;
        }
        try {
            p.rt.gpu().sync();
            const u64 token = 0xC105Eull;
            u64 a = 0, b = 0;
            p.rt.mComm.mNext.asyncSendCopy(token);
            p.rt.mComm.mPrev.asyncSendCopy(token);
            p.rt.mComm.mNext.recv(a);
            p.rt.mComm.mPrev.recv(b);
            LinkEnd::closeAll();  // from here on, this process exiting is no failure to its peers
        } catch (const std::exception&) {
            // a peer that closed on an error: nothing left to wait for
        }
    }

    void worker(int i, int device, int probe) {
        PartyCtx p;
        u64 seen = 0;
        try {
            p.idx = i;
            inTurn(i, [&] {
                p.rt.init(i, comms[i], device);
                // co-located parties: one stream each, so that with HIP's 4
                // hardware queues every party's stream has a queue of its own
                // (measured: 3 streams beat 6 sharing 4 queues on every job)
                if (colocated) p.rt.gpu().aliasAux();
                // their share GEMMs run side by side: each fills its share of the CUs
                if (colocated) GPU_CALL(aby3g_set_gemm_sharing(colocatedGemmSharing()));
                p.rt.gpu().aux();
            });
            // (only for parties sharing this process: one party per process
            // with a second stream each put six queues on the device, measured
            // 5x slower on C3)
            {
                std::shared_ptr<Gpu::SharedStream> ds;
                {
                    std::unique_lock<std::mutex> lk(turnMu);
                    turnCv.wait(lk, [&] { return turnNext > locals.back(); });
                    if (colocated && (locals.size() > 1 || partyDrawStream())) {
                        auto& slot = drawStreams[device];
                        if (!slot) slot = std::make_shared<Gpu::SharedStream>(device);
                        ds = slot;
                    }
                }
                if (ds) p.rt.gpu().setDrawStream(ds);
                // The null stream's hardware queue comes after every stream of
                // the process (the draw stream too: its creation is ordered
                // before this under turnMu), before any work. Measured: one
                // party per process without a null-stream queue ran C2 at
                // 0.59-0.74 against 0.30-0.35 ms and C4 at 0.086-0.11 against
                // 0.046 ms; three parties in a process with it created ahead
                // of theirs ran C3 at 0.41 against 0.334 ms.
                GPU_CALL(aby3g_set_device(device));
                GPU_CALL(aby3g_null_queue_init());
            }
            if (job->mlSeeds()) {
                const MlSeeds ms = mlSeeds(i);
                p.enc.init(i, ms.encPrev, ms.encNext);
                p.eval.init(i, ms.evalPrev, ms.evalNext);
            } else {
                p.enc.init(i, toBlock(0, i), toBlock(0, (i + 1) % 3));
                p.eval.init(i, toBlock(1, i), toBlock(1, (i + 1) % 3));
            }
            if (probe) GPU_CALL(aby3g_probe_enable_mask((u32)probe));
            p.ownProcess = locals.size() == 1;
            // one party per process: its AND-mask draws run on its own stream
            // in front of its first level, so they take more of the chip
            if (p.ownProcess) GPU_CALL(aby3g_set_draw_workgroups(partyDrawWorkgroups()));
            job->setup(p);
            p.checkpoint("the job's setup");
            p.rt.gpu().sync();
        } catch (const std::exception& e) {
            std::lock_guard<std::mutex> lk(mu);
            err = std::string("party ") + std::to_string(i) + " setup: " + e.what();
            // one party per process: the peers stop waiting for it now
            if (locals.size() == 1) LinkEnd::abortAll(err);
        }
        {
            std::lock_guard<std::mutex> lk(mu);
            ++finished;
            done.notify_all();
        }
        for (;;) {
            int c;
            u64 n;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return gen != seen; });
                seen = gen;
                c = cmd;
                n = steps;
            }
            if (c == 2) {
                if (locals.size() == 1) leaveTogether(p);
                return;
            }
            try {
                if (!err.empty()) throw std::runtime_error("session failed earlier");
                if (c == 1) {
                    const double dw0 = p.rt.gpu().waitUs();
                    const auto t0 = std::chrono::steady_clock::now();
                    const double w0 = recvWaitUs();
                    double a0 = 0, a1 = 0;
                    uint64_t c0 = 0, c1 = 0;
                    aby3g_api_time(&a0, &c0);
                    for (u64 s = 0; s < n; ++s) job->step(p);
                    job->drain(p);
                    aby3g_api_time(&a1, &c1);
                    hostRecvWaitUs[i] = n ? (recvWaitUs() - w0) / n : 0;
                    hostApiUs[i] = n ? (a1 - a0) / n : 0;
                    hostApiCalls[i] = n ? (double)(c1 - c0) / n : 0;
                    const auto t1 = std::chrono::steady_clock::now();
                    p.rt.gpu().sync();
                    const auto t2 = std::chrono::steady_clock::now();
                    hostEnqueueUs[i] = n ? std::chrono::duration<double, std::micro>(t1 - t0).count() / n : 0;
                    hostDrainUs[i] = std::chrono::duration<double, std::micro>(t2 - t1).count();
                    poolCached[i] = p.rt.gpu().cachedBytes();
                    deviceWaitUs[i] = n ? (p.rt.gpu().waitUs() - dw0) / n : 0;
                } else if (c == 3) {
                    double ms = 0;
                    uint64_t cnt = 0;
                    GPU_CALL(aby3g_probe_read(probeFamily, &ms, &cnt));
                    std::lock_guard<std::mutex> lk(mu);
                    probeMs[0] += ms;
                    probeN[0] += cnt;
                } else if (c == 4) {
                    GPU_CALL(aby3g_probe_reset());
                } else if (c == 7) {
                    // every local party is between runs with its streams
                    // drained (aby3h_session_run): nothing of this process can
                    // wait on a peer, so trim's device-wide wait cannot block
                    p.rt.gpu().trim();
                    poolCached[i] = 0;
                } else if (c == 8) {
                    const SharedMat* r = job->result(i);
                    std::vector<i64> v[2];
                    if (r && !r->empty())
                        for (int sh = 0; sh < 2; ++sh) v[sh] = r->shareToHost(sh);
                    std::lock_guard<std::mutex> lk(mu);
                    for (int sh = 0; sh < 2; ++sh) results[i][sh] = std::move(v[sh]);
                } else if (c == 6) {
                    const SharedMat* r = job->result(i);
                    u64 h = 0xcbf29ce484222325ull;  // FNV-1a over both shares' bytes
                    if (r && !r->empty())
                        for (int sh = 0; sh < 2; ++sh) {
                            const std::vector<i64> v = r->shareToHost(sh);
                            const u8* b = (const u8*)v.data();
                            for (size_t k = 0; k < v.size() * 8; ++k) h = (h ^ b[k]) * 0x100000001b3ull;
                        }
                    std::lock_guard<std::mutex> lk(mu);
                    digests[i] = h;
                } else if (c == 5) {
                    bool ok = job->check(p);
                    p.rt.gpu().sync();
                    std::lock_guard<std::mutex> lk(mu);
                    checkOk = checkOk && ok;
                }
            } catch (const std::exception& e) {
                std::lock_guard<std::mutex> lk(mu);
                if (err.empty()) err = std::string("party ") + std::to_string(i) + ": " + e.what();
                if (locals.size() == 1) LinkEnd::abortAll(err);
            }
            std::lock_guard<std::mutex> lk(mu);
            ++finished;
            done.notify_all();
        }
    }

    void command(int c, u64 n = 0) {
        std::unique_lock<std::mutex> lk(mu);
        cmd = c;
        steps = n;
        finished = 0;
        ++gen;
        cv.notify_all();
        done.wait(lk, [&] { return finished == (int)locals.size(); });
    }
};

// cached pool bytes per party above which a run's end trims the pools
// (ABY3_POOL_TRIM_MB, default 32 GiB of the 288 GB of HBM per MI355X)
static size_t poolTrimBytes() {
    static const size_t b = [] {
        const char* e = getenv("ABY3_POOL_TRIM_MB");
        return (e && *e ? (size_t)atoll(e) : (size_t)32 << 10) << 20;
    }();
    return b;
}

std::unique_ptr<Job> makeJob(int job, const uint64_t* params, int nparams) {
    auto P = [&](int i, u64 def) { return i < nparams ? params[i] : def; };
    switch (job) {
        case ABY3H_JOB_MUL_TRUNC:
            return std::make_unique<MulJob>(P(0, 1024), P(1, 1024), P(2, 1024), P(3, 16),
                                            P(4, 1) ? MulMode::Gemm : MulMode::Hadamard, true, P(5, 1), P(6, 0),
                                            P(7, 1));
        case ABY3H_JOB_MUL:
            return std::make_unique<MulJob>(P(0, 128), P(1, 128), P(2, 128), 0, P(3, 0) ? MulMode::Gemm : MulMode::Hadamard,
                                            false);
        case ABY3H_JOB_MSB: return std::make_unique<MsbJob>(P(0, 1 << 20), P(1, 0), P(2, 1));
        case ABY3H_JOB_LR:
            return std::make_unique<LrJob>(P(0, 1000000), P(1, 128), P(2, 256), P(3, 16), P(4, 11), P(5, 0));
        case ABY3H_JOB_SORT: return std::make_unique<SortJob>(P(0, 1 << 20), P(1, 0));
        case ABY3H_JOB_A2B: return std::make_unique<A2bJob>(P(0, 1 << 20));
        case ABY3H_JOB_BITINJ: return std::make_unique<BitInjJob>(P(0, 1 << 16), P(1, 64));
        default: throw std::runtime_error("unknown job");
    }
}

}  // namespace aby3

using namespace aby3;

struct aby3h_session {
    Session s;
};

extern "C" {

const char* aby3h_last_error(void) { return t_err.c_str(); }

aby3h_session* aby3h_session_create(int job, const uint64_t* params, int nparams, const int* devices, int probe) {
    try {
        // destroyed (threads joined) on any failure below
        std::unique_ptr<aby3h_session, void (*)(aby3h_session*)> guard(new aby3h_session, aby3h_session_destroy);
        aby3h_session* h = guard.get();
        Session& s = h->s;
        s.job = makeJob(job, params, nparams);
        s.locals = {0, 1, 2};
        {
            int dv[3] = {0, 0, 0};
            if (devices)
                for (int i = 0; i < 3; ++i) dv[i] = devices[i];
            for (int i = 0; i < 3; ++i) s.devices[i] = dv[i];
            // all three parties on one device: one stream each (aux aliased)
            // plus the shared draw stream, each with a hardware queue of its
            // own, so their kernels may hand messages over on the device
            // (and only while no other live stream of this process on the
            // device, e.g. another open session, could take one of the queues)
            const bool oneDevice = dv[0] == dv[1] && dv[1] == dv[2];
            s.comms = makeLocalRing(dv, oneDevice && liveStreams(dv[0]) + 4 <= hwQueuesPerDevice());
        }
        s.colocated = !devices || devices[0] == devices[1] || devices[1] == devices[2] || devices[0] == devices[2];
        {
            std::unique_lock<std::mutex> lk(s.mu);
            s.finished = 0;
        }
        for (int i = 0; i < 3; ++i) s.th[i] = std::thread([&s, i, devices, probe] {
            s.worker(i, devices ? devices[i] : 0, probe);
        });
        {
            std::unique_lock<std::mutex> lk(s.mu);
            s.done.wait(lk, [&] { return s.finished == 3; });
        }
        if (!s.err.empty()) throw std::runtime_error(s.err);
        return guard.release();
    } catch (const std::exception& e) {
        t_err = e.what();
        return nullptr;
    }
}

aby3h_session* aby3h_party_create(int job, const uint64_t* params, int nparams, int party, int device,
                                  const char* link, int colocated, int probe) {
    try {
        if (party < 0 || party > 2) throw std::runtime_error("party must be 0, 1 or 2");
        if (!link) throw std::runtime_error("null link name");
        // destroyed (thread joined, links closed) on any failure below
        std::unique_ptr<aby3h_session, void (*)(aby3h_session*)> guard(new aby3h_session, aby3h_session_destroy);
        aby3h_session* h = guard.get();
        Session& s = h->s;
        s.job = makeJob(job, params, nparams);
        s.locals = {party};
        s.comms.resize(3);
        if (colocated < 0 || colocated > 2) throw std::runtime_error("colocated must be 0, 1 or 2");
        s.comms[(size_t)party] = makeProcessRing(party, link, device, colocated == 1, colocated == 2);
        s.devices[party] = device;
        s.colocated = colocated != 0;
        s.turnNext = party;  // stream-creation turns: only this party's here
        {
            std::unique_lock<std::mutex> lk(s.mu);
            s.finished = 0;
        }
        s.th[party] = std::thread([&s, party, device, probe] { s.worker(party, device, probe); });
        {
            std::unique_lock<std::mutex> lk(s.mu);
            s.done.wait(lk, [&] { return s.finished == 1; });
        }
        if (!s.err.empty()) throw std::runtime_error(s.err);
        return guard.release();
    } catch (const std::exception& e) {
        t_err = e.what();
        return nullptr;
    }
}

int aby3h_session_run(aby3h_session* h, uint64_t steps) {
    Session& s = h->s;
    // an in-kernel hand-off that gave up during the run invalidates it
    // (common.h): the device's timeout count before and after
    u32 before[3] = {0, 0, 0};
    try {
        for (int q : s.locals) before[q] = handoffTimeouts(s.devices[q]);
    } catch (const std::exception& e) {
        t_err = e.what();
        return 1;
    }
    s.command(1, steps);
    if (s.err.empty()) {
        // The pools keep every freed block cached for reuse (a mid-run free
        // could wait on a peer, Device.cpp Gpu::alloc); past a bound, give the
        // cache back here, between runs, where every local party is idle.
        size_t most = 0;
        for (int q : s.locals) most = std::max(most, s.poolCached[q]);
        if (most > poolTrimBytes()) s.command(7);
    }
    if (s.err.empty()) {
        try {
            for (int q : s.locals) {
                const u32 n = handoffTimeouts(s.devices[q]) - before[q];
                if (n)
                    throw std::runtime_error(std::to_string(n) +
                                             " in-kernel hand-off wait(s) timed out: a party stream without a "
                                             "hardware queue of its own?");
            }
        } catch (const std::exception& e) {
            s.err = e.what();
        }
    }
    if (!s.err.empty()) {
        t_err = s.err;
        return 1;
    }
    return 0;
}

int aby3h_session_probe(aby3h_session* h, int family, double* ms, uint64_t* launches) {
    Session& s = h->s;
    s.probeFamily = family;
    s.probeMs[0] = 0;
    s.probeN[0] = 0;
    s.command(3);
    *ms = s.probeMs[0];
    *launches = s.probeN[0];
    if (!s.err.empty()) {
        t_err = s.err;
        return 1;
    }
    return 0;
}

int aby3h_session_probe_reset(aby3h_session* h) {
    h->s.command(4);
    return h->s.err.empty() ? 0 : 1;
}

int aby3h_session_info(aby3h_session* h, double* out, int n) {
    double tmp[ABY3H_INFO_COUNT] = {0};
    h->s.job->info(tmp);
    const int q = h->s.locals[0];  // party 0, or this process's party
    tmp[ABY3H_INFO_HOST_ENQUEUE_US] = *std::max_element(h->s.hostEnqueueUs, h->s.hostEnqueueUs + 3);
    tmp[ABY3H_INFO_HOST_DRAIN_US] = h->s.hostDrainUs[q];
    tmp[ABY3H_INFO_HOST_RECV_WAIT_US] = h->s.hostRecvWaitUs[q];
    tmp[ABY3H_INFO_HOST_API_US] = h->s.hostApiUs[q];
    tmp[ABY3H_INFO_HOST_API_CALLS] = h->s.hostApiCalls[q];
    double dw = 0;
    for (int l : h->s.locals) dw += h->s.deviceWaitUs[l];
    tmp[ABY3H_INFO_DEVICE_WAIT_US] = dw / (double)h->s.locals.size();
    for (int i = 0; i < n && i < ABY3H_INFO_COUNT; ++i) out[i] = tmp[i];
    return 0;
}

int aby3h_session_result(aby3h_session* h, int party, int share, int64_t* out, uint64_t count,
                         uint64_t* elements) {
    Session& s = h->s;
    if (std::find(s.locals.begin(), s.locals.end(), party) == s.locals.end()) {
        t_err = "result: party " + std::to_string(party) + " is not run by this session";
        return 1;
    }
    if (share < 0 || share > 1 || !elements || (count && !out)) {
        t_err = "result: share must be 0 or 1, elements and (for count > 0) out non-null";
        return 1;
    }
    s.command(8);
    if (!s.err.empty()) {
        t_err = s.err;
        return 1;
    }
    const std::vector<i64>& v = s.results[party][share];
    *elements = v.size();
    if (count) std::memcpy(out, v.data(), std::min<u64>(count, v.size()) * sizeof(i64));
    return 0;
}

int aby3h_session_digest(aby3h_session* h, int party, uint64_t* out) {
    Session& s = h->s;
    if (std::find(s.locals.begin(), s.locals.end(), party) == s.locals.end()) {
        t_err = "digest: party " + std::to_string(party) + " is not run by this session";
        return 1;
    }
    s.command(6);
    if (!s.err.empty()) {
        t_err = s.err;
        return 1;
    }
    *out = s.digests[party];
    return 0;
}

int aby3h_session_check(aby3h_session* h) {
    Session& s = h->s;
    s.checkOk = true;
    s.command(5);
    if (!s.err.empty()) {
        t_err = s.err;
        return 2;
    }
    return s.checkOk ? 0 : 1;
}

void aby3h_session_destroy(aby3h_session* h) {
    if (!h) return;
    Session& s = h->s;
    {
        std::lock_guard<std::mutex> lk(s.mu);
        s.cmd = 2;
        ++s.gen;
        s.cv.notify_all();
    }
    for (auto& t : s.th)
        if (t.joinable()) t.join();
    delete h;
}

int aby3h_circuit_write(const char* name, uint64_t size, uint64_t param, const char* path) {
    try {
        CircuitLibrary lib;
        BetaCircuit* c = lib.byName(name, size, param);
        std::ofstream f(path, std::ios::binary | std::ios::trunc);
        if (!f) throw std::runtime_error(std::string("cannot write ") + path);
        c->writeBin(f);
        return 0;
    } catch (const std::exception& e) {
        t_err = e.what();
        return 1;
    }
}

int aby3h_circuit(const char* name, uint64_t size, uint64_t param, uint64_t counts[6], uint32_t* gates,
                  uint32_t* level_counts, uint32_t* in_sizes, uint32_t* in_wires, uint32_t* out_sizes,
                  uint32_t* out_wires) {
    try {
        CircuitLibrary lib;
        BetaCircuit* c = lib.byName(name, size, param);
        u64 inW = 0, outW = 0;
        for (auto& b : c->mInputs) inW += b.size();
        for (auto& b : c->mOutputs) outW += b.size();
        counts[0] = c->mWireCount;
        counts[1] = c->mLevelGates.size();
        counts[2] = c->mLevelCounts.size();
        counts[3] = c->mInputs.size();
        counts[4] = c->mOutputs.size();
        counts[5] = inW + outW;
        if (gates)
            for (size_t i = 0; i < c->mLevelGates.size(); ++i) {
                const auto& g = c->mLevelGates[i];
                gates[4 * i] = g.in0;
                gates[4 * i + 1] = g.in1;
                gates[4 * i + 2] = g.out;
                gates[4 * i + 3] = (u32)g.type;
            }
        if (level_counts) std::copy(c->mLevelCounts.begin(), c->mLevelCounts.end(), level_counts);
        u64 o = 0;
        for (size_t b = 0; b < c->mInputs.size(); ++b) {
            if (in_sizes) in_sizes[b] = (u32)c->mInputs[b].size();
            if (in_wires) std::copy(c->mInputs[b].begin(), c->mInputs[b].end(), in_wires + o);
            o += c->mInputs[b].size();
        }
        o = 0;
        for (size_t b = 0; b < c->mOutputs.size(); ++b) {
            if (out_sizes) out_sizes[b] = (u32)c->mOutputs[b].size();
            if (out_wires) std::copy(c->mOutputs[b].begin(), c->mOutputs[b].end(), out_wires + o);
            o += c->mOutputs[b].size();
        }
        return 0;
    } catch (const std::exception& e) {
        t_err = e.what();
        return 1;
    }
}

}  // extern "C"
