#include "Basic.h"
#include <cmath>
#include <cstring>
#include <random>

namespace aby3 {

CircuitLibrary& basicLibrary() {
    thread_local CircuitLibrary lib;
    return lib;
}

void evalCircuit(BetaCircuit* cir, const std::vector<const sbMatrix*>& in, const std::vector<sbMatrix*>& out,
                 Sh3Evaluator& eval, Sh3Runtime& runtime) {
    Sh3BinaryEvaluator binEng;
    binEng.setCir(cir, in[0]->rows(), eval.mShareGen);
    for (size_t i = 0; i < in.size(); ++i) binEng.setInput(i, *in[i]);
    binEng.asyncEvaluate(runtime.noDependencies())
        .then([&](Sh3Task&) {
            for (size_t i = 0; i < out.size(); ++i) binEng.getOutput(i, *out[i]);
        })
        .get();
}

// Binary two-input sharing of an arithmetic value x = sum of coef * X over
// `x`'s terms, c0 = (sign * (x0 + x2), 0, 0) reshared by P0 and c1 =
// (0, x1, 0) (BuildingBlocks.cpp:475-502, :709-735), fed straight into the
// circuit's input wires (setTwoInputSharing: one launch, one message), then
// the circuit (inputs c0, c1; output 0) evaluated into `res`.
// (totalRows != 0: rows from rowOffset of a totalRows-row evaluation, setCirRows)
static void evalTwoInput(BetaCircuit* cir, int pIdx, const std::vector<std::pair<const si64Matrix*, i64>>& x, i64 sign,
                         sbMatrix& res, Sh3Evaluator& eval, Sh3Runtime& rt, u64 rowOffset = 0, u64 totalRows = 0) {
    Sh3BinaryEvaluator binEng;
    if (totalRows)
        binEng.setCirRows(cir, x[0].first->size(), eval.mShareGen, rowOffset, totalRows);
    else
        binEng.setCir(cir, x[0].first->size(), eval.mShareGen);
    setTwoInputSharing(binEng, pIdx, x, sign, {0}, {0}, 1, rt.mComm, rt.gpu());
    binEng.asyncEvaluate(rt.noDependencies())
        .then([&](Sh3Task&) { binEng.getOutput(0, res); })
        .get();
}

int fetch_msb(int pIdx, const si64Matrix& diffAB, sbMatrix& res, Sh3Evaluator& eval, Sh3Runtime& runtime) {
    evalTwoInput(basicLibrary().int_comp_helper(64), pIdx, {{&diffAB, 1}}, 1, res, eval, runtime);
    return 0;
}

static void checkShapes(const si64Matrix& a, const si64Matrix& b) {
    if (a.rows() != b.rows() || a.cols() != b.cols()) throw std::runtime_error("shape mismatch " LOCATION);
}

// cipher_gt(A, B) = MSB(B - A) (BuildingBlocks.cpp:525-532); the difference
// is folded into the input sharing
int cipher_gt(int pIdx, const si64Matrix& A, const si64Matrix& B, sbMatrix& res, Sh3Evaluator& eval,
              Sh3Runtime& runtime) {
    checkShapes(A, B);
    evalTwoInput(basicLibrary().int_comp_helper(64), pIdx, {{&B, 1}, {&A, -1}}, 1, res, eval, runtime);
    return 0;
}

int cipher_gt_rows(int pIdx, const si64Matrix& A, const si64Matrix& B, sbMatrix& res, Sh3Evaluator& eval,
                   Sh3Runtime& runtime, u64 rowOffset, u64 totalRows) {
    checkShapes(A, B);
    if (A.cols() != 1) throw std::invalid_argument("cipher_gt_rows: one value per row " LOCATION);
    if (!A.rows()) {  // an empty slice: the circuit's keys are still taken, as by the unsplit evaluation
        eval.mShareGen.getPrevBlock();
        eval.mShareGen.getNextBlock();
        res.resize(0, 1);
        return 0;
    }
    evalTwoInput(basicLibrary().int_comp_helper(64), pIdx, {{&B, 1}, {&A, -1}}, 1, res, eval, runtime, rowOffset,
                 totalRows);
    return 0;
}

int cipher_ge(int pIdx, const si64Matrix& A, const si64Matrix& B, sbMatrix& res, Sh3Evaluator& eval,
              Sh3Runtime& runtime) {
    checkShapes(A, B);
    evalTwoInput(basicLibrary().int_comp_helper(64), pIdx, {{&A, 1}, {&B, -1}}, 1, res, eval, runtime);
    // flip bit 0 of both shares of every party: all three shares flip
    Gpu& g = runtime.gpu();
    DeviceBuffer ones(g, res.size() * 2 * 8);
    std::vector<i64> h(res.size() * 2, 1);
    toDevice(ones.data(), h.data(), h.size() * 8, g);
    GPU_CALL(aby3g_u64_bitop(0, 2 * res.size(), (const u64*)res.data(), ones.as<u64>(), (u64*)res.data(), g.stream()));
    return 0;
}

int circuit_cipher_eq(int pIdx, const si64Matrix& A, const si64Matrix& B, sbMatrix& res, Sh3Evaluator& eval,
                      Sh3Runtime& runtime) {
    checkShapes(A, B);
    evalTwoInput(basicLibrary().int_eq(64), pIdx, {{&A, 1}, {&B, -1}}, -1, res, eval, runtime);
    return 0;
}

int cipher_mul(int, const si64Matrix& A, const si64Matrix& B, si64Matrix& res, Sh3Evaluator& eval,
               Sh3Runtime& runtime) {
    eval.asyncMul(runtime, A, B, res, MulMode::Hadamard).get();
    return 0;
}

int cipher_mul(int, const si64Matrix& A, const sbMatrix& B, si64Matrix& res, Sh3Evaluator& eval,
               Sh3Runtime& runtime) {
    eval.asyncMul(runtime, A, B, res).get();
    return 0;
}

void bool_cipher_lt(int, const sbMatrix& A, const sbMatrix& B, sbMatrix& res, Sh3Evaluator& eval,
                    Sh3Runtime& runtime) {
    evalCircuit(basicLibrary().int_int_lt(A.bitCount()), {&A, &B}, {&res}, eval, runtime);
}
void bool_cipher_eq(int, const sbMatrix& A, const sbMatrix& B, sbMatrix& res, Sh3Evaluator& eval,
                    Sh3Runtime& runtime) {
    evalCircuit(basicLibrary().int_eq(A.bitCount()), {&A, &B}, {&res}, eval, runtime);
}
void bool_cipher_and(int, const sbMatrix& A, const sbMatrix& B, sbMatrix& res, Sh3Evaluator& eval,
                     Sh3Runtime& runtime) {
    evalCircuit(basicLibrary().int_int_bitwiseAnd(A.bitCount()), {&A, &B}, {&res}, eval, runtime);
}
void bool_cipher_or(int, const sbMatrix& A, const sbMatrix& B, sbMatrix& res, Sh3Evaluator& eval,
                    Sh3Runtime& runtime) {
    evalCircuit(basicLibrary().int_int_bitwiseOr(A.bitCount()), {&A, &B}, {&res}, eval, runtime);
}
void bool_cipher_add(int, const sbMatrix& A, const sbMatrix& B, sbMatrix& res, Sh3Evaluator& eval,
                     Sh3Runtime& runtime) {
    evalCircuit(basicLibrary().int_int_add(A.bitCount()), {&A, &B}, {&res}, eval, runtime);
}
void bool_cipher_sub(int, const sbMatrix& A, const sbMatrix& B, sbMatrix& res, Sh3Evaluator& eval,
                     Sh3Runtime& runtime) {
    evalCircuit(basicLibrary().int_int_sub(A.bitCount()), {&A, &B}, {&res}, eval, runtime);
}

void bool_cipher_not(int pIdx, const sbMatrix& A, sbMatrix& res) {
    Gpu& g = A.gpu();
    const u64 n = A.size();
    if (&res != &A) {
        res.resize(A.rows(), A.bitCount());
        d2d(res.data(), A.data(), 2 * n * 8, g);
    }
    if (pIdx == 1) GPU_CALL(aby3g_u64_bitop(2, n, (const u64*)res.share(0), nullptr, (u64*)res.share(0), g.stream()));
    if (pIdx == 2) GPU_CALL(aby3g_u64_bitop(2, n, (const u64*)res.share(1), nullptr, (u64*)res.share(1), g.stream()));
}

void bool_cipher_max_min_split(int, const sbMatrix& A, const sbMatrix& B, sbMatrix& resMax, sbMatrix& resMin,
                               Sh3Evaluator& eval, Sh3Runtime& runtime) {
    evalCircuit(basicLibrary().cmp_swap(A.bitCount()), {&A, &B}, {&resMin, &resMax}, eval, runtime);
}
void bool_cipher_max(int pIdx, const sbMatrix& A, const sbMatrix& B, sbMatrix& res, Sh3Evaluator& eval,
                     Sh3Runtime& runtime) {
    sbMatrix mn;
    bool_cipher_max_min_split(pIdx, A, B, res, mn, eval, runtime);
}
void bool_cipher_min(int pIdx, const sbMatrix& A, const sbMatrix& B, sbMatrix& res, Sh3Evaluator& eval,
                     Sh3Runtime& runtime) {
    sbMatrix mx;
    bool_cipher_max_min_split(pIdx, A, B, mx, res, eval, runtime);
}

}  // namespace aby3

namespace aby3 {

void bool2arith(int pIdx, const sbMatrix& boolInput, si64Matrix& res, Sh3Encryptor& enc, Sh3Evaluator& eval,
                Sh3Runtime& runtime) {
    const u64 len = boolInput.rows(), bitSize = boolInput.bitCount();
    if (bitSize == 1) {  // pi_cb_mul(ones, boolInput) (:522-526)
        eval.asyncMul(runtime.noDependencies(), (i64)1, boolInput, res, enc.mShareGen).get();
        return;
    }
    // the reference copies `len` words per share (:538-545): one word per row
    if (boolInput.cols() != 1) throw std::runtime_error("bool2arith: at most 64 bits per row " LOCATION);
    Gpu& g = runtime.gpu();
    const u64 b8 = len * sizeof(i64);
    auto fresh = [](const block& seed) {  // PRNG prng(seed): a new generator, offset 0
        aby3g_stream_pos p;
        std::memcpy(p.seed, seed.data(), 16);
        p.off = 0;
        return p;
    };
    // 1) r, shared (r, 0, 0) by P0 (share 0) and P1 (share 1)
    sbMatrix r(len, bitSize);
    GPU_CALL(aby3g_memset(r.data(), 0, 2 * b8, g.stream()));
    aby3g_stream_pos rpos = fresh(pIdx == 0 ? enc.mShareGen.mNextSeed : enc.mShareGen.mPrevSeed);
    if (pIdx < 2 && len) GPU_CALL(aby3g_prng_i32(&rpos, len, 1, r.share(pIdx == 0 ? 0 : 1), g.stream()));
    // 2) c = x + r
    sbMatrix c;
    bool_cipher_add(pIdx, boolInput, r, c, eval, runtime);
    // 3) open c to P2, which reshares it
    si64Matrix out(len, 1);
    if (len)
        runtime.noDependencies()
            .then([&](CommPkg& comm, Sh3Task& self) {
                aby3g_stream st = g.stream();
                switch (pIdx) {
                    case 0: {  // (-r, c - t)
                        GPU_CALL(aby3g_prng_i32(&rpos, len, -1, out.share(0), st));
                        auto f = comm.mPrev.asyncRecvDevice(out.share(1), b8, g);
                        self.then([f](CommPkg&, Sh3Task&) { f.get(); });
                        break;
                    }
                    case 1: {  // (t, -r)
                        comm.mNext.asyncSendDevice(c.share(1), b8, g);
                        GPU_CALL(aby3g_prng_i32(&rpos, len, -1, out.share(1), st));
                        auto f = comm.mNext.asyncRecvDevice(out.share(0), b8, g);
                        self.then([f](CommPkg&, Sh3Task&) { f.get(); });
                        break;
                    }
                    case 2: {  // (c - t, t), t private to P2 (the reference's rand(), :580)
                        auto recv = std::make_shared<DeviceBuffer>(g, b8);
                        auto f = comm.mPrev.asyncRecvDevice(recv->data(), b8, g);
                        self.then([&, f, recv](CommPkg& comm2, Sh3Task&) {
                            f.get();
                            static thread_local std::random_device rd;
                            u8 seed[16];
                            for (int k = 0; k < 4; ++k) {
                                const u32 v = rd();
                                std::memcpy(seed + 4 * k, &v, 4);
                            }
                            aby3g_stream st2 = g.stream();
                            GPU_CALL(aby3g_prng_fill(seed, 0, b8, out.share(1), st2));
                            GPU_CALL(aby3g_b2a_open(c.share(0), c.share(1), recv->as<i64>(), out.share(1), len,
                                                    out.share(0), st2));
                            comm2.mNext.asyncSendDevice(out.share(0), b8, g);
                            comm2.mPrev.asyncSendDevice(out.share(1), b8, g);
                        });
                        break;
                    }
                    default:
                        throw RTE_LOC;
                }
            })
            .getClosure()
            .get();
    res = std::move(out);
}

// ---- large messages (Basic.cpp:3-62) --------------------------------------
namespace {
Channel& neighbour(Sh3Runtime& rt, bool next) { return next ? rt.mComm.mNext : rt.mComm.mPrev; }
void checkChunk(u64 chunk) {
    if (!chunk) throw std::runtime_error("large_data: chunk size must be positive");
}
}  // namespace

int large_data_sending(int, const i64Matrix& sharedA, Sh3Runtime& runtime, bool toNext, u64 chunk) {
    checkChunk(chunk);
    const u64 len = sharedA.mData.size();
    Channel& ch = neighbour(runtime, toNext);
    for (u64 o = 0; o < len; o += chunk) ch.asyncSendCopy(sharedA.mData.data() + o, 8 * std::min(chunk, len - o));
    return 0;
}

int large_data_receiving(int, i64Matrix& res, Sh3Runtime& runtime, bool fromPrev, u64 chunk) {
    checkChunk(chunk);
    const u64 len = res.mData.size();
    Channel& ch = neighbour(runtime, !fromPrev);
    for (u64 o = 0; o < len; o += chunk) ch.recv(res.mData.data() + o, 8 * std::min(chunk, len - o));
    return 0;
}

int large_data_sending(int, const i64* sharedA, u64 len, Sh3Runtime& runtime, bool toNext, u64 chunk) {
    checkChunk(chunk);
    Channel& ch = neighbour(runtime, toNext);
    for (u64 o = 0; o < len; o += chunk) ch.asyncSendDevice(sharedA + o, 8 * std::min(chunk, len - o), runtime.gpu());
    return 0;
}

int large_data_receiving(int, i64* res, u64 len, Sh3Runtime& runtime, bool fromPrev, u64 chunk) {
    checkChunk(chunk);
    Channel& ch = neighbour(runtime, !fromPrev);
    for (u64 o = 0; o < len; o += chunk) ch.asyncRecvDevice(res + o, 8 * std::min(chunk, len - o), runtime.gpu()).get();
    return 0;
}

}  // namespace aby3
