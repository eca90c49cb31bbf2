// Share-level parity of the SGD_Logistic iteration (aby3-ML/Regression.h:
// 249-293) in both of its GPU forms against the CPU oracle, on the aby3ML
// seeds (aby3ML.cpp:4-17):
//   * op by op: every step a C-ABI call, messages over the channels (the
//     parties' ring without kernel hand-offs: one party per process, or
//     parties on distinct devices, take this form);
//   * fused: one launch per party and iteration (aby3g_lr_iteration), the
//     three co-located parties exchanging their messages in-kernel.
// Both must leave every party's w shares equal to the oracle's after each
// iteration, and the fused form must actually have been taken.
#include <cstring>
#include "aby3ML.h"
#include "harness.h"

using namespace aby3;
using namespace harness;

static orc::Circuit toOrc(const BetaCircuit& c) {
    orc::Circuit o;
    o.wireCount = c.mWireCount;
    for (auto& g : c.mLevelGates) o.gates.push_back(orc::Gate{g.in0, g.in1, g.out, (u32)g.type});
    o.levelCounts = c.mLevelCounts;
    o.inputs = c.mInputs;
    o.outputs = c.mOutputs;
    return o;
}

// three party threads on `device`; fused: one stream each and a ring that
// allows in-kernel hand-offs (as aby3h_sim_* and the co-located sessions)
static void run3ml(bool fused, const std::function<void(Sh3Runtime&, Sh3Encryptor&, Sh3Evaluator&, int)>& f,
                   int device = 0) {
    const int dv[3] = {device, device, device};
    auto comms = fused ? makeLocalRing(dv, true) : makeLocalRing();
    const u32 timeouts0 = handoffTimeouts(device);
    std::exception_ptr err[3];
    std::thread th[3];
    for (int i = 0; i < 3; ++i)
        th[i] = std::thread([&, i] {
            try {
                Sh3Runtime rt;
                Sh3Encryptor enc;
                Sh3Evaluator eval;
                rt.init(i, comms[i], device);
                if (fused) rt.gpu().aliasAux();
                const MlSeeds ms = mlSeeds(i);
                enc.init(i, ms.encPrev, ms.encNext);
                eval.init(i, ms.evalPrev, ms.evalNext);
                f(rt, enc, eval, i);
                rt.gpu().sync();
            } catch (...) {
                err[i] = std::current_exception();
            }
        });
    for (auto& t : th) t.join();
    for (auto& e : err)
        if (e) std::rethrow_exception(e);
    check(handoffTimeouts(device) == timeouts0, "an in-kernel hand-off timed out");
}

static void lrParity(bool fused, u64 n, u64 d, u64 B, u64 iters) {
    const u64 D = 16, aB = 11;
    i64Matrix X, Y, w0(d, 1);
    logisticModelGen(logisticModel(d), n, D, X, Y);
    std::vector<u32> idx(iters * B);
    {
        BatchSampler s(n);
        std::vector<u64> b(B);
        for (u64 t = 0; t < iters; ++t) {
            s.next(b);
            for (u64 i = 0; i < B; ++i) idx[t * B + i] = (u32)b[i];
        }
    }
    std::vector<ShareSink> got(iters);
    bool tookFused[3] = {false, false, false};
    run3ml(fused, [&](Sh3Runtime& rt, Sh3Encryptor& enc, Sh3Evaluator& eval, int p) {
        si64Matrix sX(n, d), sY(n, 1), sW(d, 1);
        const std::pair<i64Matrix*, si64Matrix*> ins[3] = {{&X, &sX}, {&Y, &sY}, {&w0, &sW}};
        for (const auto& m : ins) {
            if (p == 0)
                enc.localIntMatrix(rt, *m.first, *m.second).get();
            else
                enc.remoteIntMatrix(rt, *m.second).get();
        }
        aby3ML ml(rt, enc, eval, D);
        SgdState st;
        for (u64 t = 0; t < iters; ++t) {
            sgdLogisticStep(ml, sX, sY, sW, std::vector<u32>(idx.begin() + t * B, idx.begin() + (t + 1) * B), aB, st);
            got[t].put(p, sW);
        }
        tookFused[p] = (bool)st.fused;
    });
    for (int p = 0; p < 3; ++p) check(tookFused[p] == fused, fused ? "fused form not taken" : "fused form taken");
    // the oracle, the same data and batches
    CircuitLibrary lib;
    BetaCircuit* cir = lib.int_Sh3Piecewise_helper(64, 2);
    if (!cir->levelized()) cir->levelByAndDepth();
    const orc::Circuit oc = toOrc(*cir);
    std::array<orc::Party, 3> enc, ev;
    orc::mlParties(enc, ev);
    orc::Shared oX = orc::shareInt(enc, 0, toOrc(X)), oY = orc::shareInt(enc, 0, toOrc(Y));
    orc::Shared oW = orc::shareInt(enc, 0, orc::Mat(d, 1));
    for (u64 t = 0; t < iters; ++t) {
        std::vector<u64> batch(idx.begin() + t * B, idx.begin() + (t + 1) * B);
        orc::sgdLogisticIteration(ev, oc, oX, oY, oW, batch, D, aB);
        got[t].expectEq(oW, "w after iteration " + std::to_string(t));
    }
}

int main() {
    test("sgd_logistic_op_by_op_3000x128_B64_x3", [] { lrParity(false, 3000, 128, 64, 3); });
    test("sgd_logistic_fused_3000x128_B64_x3", [] { lrParity(true, 3000, 128, 64, 3); });
    test("sgd_logistic_op_by_op_20000x128_B256_x4", [] { lrParity(false, 20000, 128, 256, 4); });
    test("sgd_logistic_fused_20000x128_B256_x4", [] { lrParity(true, 20000, 128, 256, 4); });
    // ragged shapes: a batch that is not a multiple of 64 rows, odd features
    test("sgd_logistic_fused_5000x37_B100_x3", [] { lrParity(true, 5000, 37, 100, 3); });
    test("sgd_logistic_op_by_op_5000x37_B100_x3", [] { lrParity(false, 5000, 37, 100, 3); });
    // more iterations than mailbox parities: reuse of both message regions
    test("sgd_logistic_fused_4096x128_B256_x7", [] { lrParity(true, 4096, 128, 256, 7); });
    return g_failures ? 1 : 0;
}
