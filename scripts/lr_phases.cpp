// Phase profile of the fused SGD_Logistic iteration (aby3g_lr_iteration):
// three co-located parties run `iters` iterations on a 10^6 x 128 dataset
// (B = 256), every launch stamping its phases (wall clock, 100 MHz); prints
// per party the median duration of each phase over the last half of the run.
// Build: scripts/lr_phases.sh
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <thread>
#include "aby3ML.h"

constexpr unsigned long long S = ABY3G_LR_PHASE_SLOTS;  // stamp slots per iteration

using namespace aby3;

int main(int argc, char** argv) {
    const u64 n = argc > 1 ? atoll(argv[1]) : 1000000, d = 128, B = 256, D = 16, aB = 11;
    const u64 iters = argc > 2 ? atoll(argv[2]) : 200;
    i64Matrix X, Y, w0(d, 1);
    logisticModelGen(logisticModel(d), n, D, X, Y);
    std::vector<u32> idx(iters * B);
    BatchSampler s(n);
    std::vector<u64> b(B);
    for (u64 t = 0; t < iters; ++t) {
        s.next(b);
        for (u64 i = 0; i < B; ++i) idx[t * B + i] = (u32)b[i];
    }
    const int dv[3] = {0, 0, 0};
    auto comms = makeLocalRing(dv, true);
    std::vector<std::vector<u64>> stamps(3);
    double wallUs = 0;
    std::thread th[3];
    for (int p = 0; p < 3; ++p)
        th[p] = std::thread([&, p] {
            Sh3Runtime rt;
            Sh3Encryptor enc;
            Sh3Evaluator ev;
            rt.init(p, comms[p], 0);
            rt.gpu().aliasAux();
            const MlSeeds ms = mlSeeds(p);
            enc.init(p, ms.encPrev, ms.encNext);
            ev.init(p, ms.evalPrev, ms.evalNext);
            si64Matrix sX(n, d), sY(n, 1), sW(d, 1);
            if (p == 0) {
                enc.localIntMatrix(rt, X, sX).get();
                enc.localIntMatrix(rt, Y, sY).get();
                enc.localIntMatrix(rt, w0, sW).get();
            } else {
                enc.remoteIntMatrix(rt, sX).get();
                enc.remoteIntMatrix(rt, sY).get();
                enc.remoteIntMatrix(rt, sW).get();
            }
            aby3ML ml(rt, enc, ev, D);
            SgdState st;
            DeviceBuffer dIdx(rt.gpu(), idx.size() * 4), ticks(rt.gpu(), iters * S * 8);
            toDevice(dIdx.data(), idx.data(), idx.size() * 4, rt.gpu());
            const std::vector<u64> zeros(iters * S, 0);  // unused slots read 0
            toDevice(ticks.data(), zeros.data(), iters * S * 8, rt.gpu());
            rt.gpu().sync();
            const auto t0 = std::chrono::steady_clock::now();
            for (u64 t = 0; t < iters; ++t) {
                st.phaseTicks = ticks.as<u64>() + S * t;
                sgdLogisticStep(ml, sX, sY, sW, dIdx.as<u32>() + t * B, B, aB, st);
            }
            rt.gpu().sync();
            if (p == 0)
                wallUs = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            stamps[p].resize(iters * S);
            toHost(stamps[p].data(), ticks.data(), iters * S * 8, rt.gpu());
            if (!st.fused) std::printf("party %d: fused form NOT taken\n", p);
        });
    for (auto& t : th) t.join();
    std::printf("wall %.1f us per iteration (%llu iterations)\n", wallUs / iters, (unsigned long long)iters);
    // interval i = stamps i -> i + 1 (lr.hip lr_stamp slots; slot 12 = after the table fill)
    const char* names[11] = {"aes table+masks", "xw product", "trunc pair+post", "z wait+finalize",
                             "reshare+inputs", "levels", "regions", "OT+public products", "err+XtE product",
                             "trunc pair 2", "finalize / w"};
    for (int p = 0; p < 3; ++p) {
        std::printf("party %d:", p);
        double tot = 0;
        for (int ph = 0; ph < 11; ++ph) {
            std::vector<double> v;
            for (u64 t = iters / 2; t < iters; ++t)
                v.push_back(0.01 * (double)(stamps[p][S * t + ph + 1] - stamps[p][S * t + ph]));
            std::sort(v.begin(), v.end());
            std::printf(" %s %.1f |", names[ph], v[v.size() / 2]);
            tot += v[v.size() / 2];
        }
        {
            std::vector<double> v;
            for (u64 t = iters / 2; t < iters; ++t) v.push_back(0.01 * (double)(stamps[p][S * t + 12] - stamps[p][S * t]));
            std::sort(v.begin(), v.end());
            std::printf(" (table fill %.1f)", v[v.size() / 2]);
            std::vector<double> f;
            for (u64 t = iters / 2; t < iters; ++t)
                f.push_back(100.0 * (double)(stamps[p][S * t + 14] - stamps[p][S * t + 13]) /
                            (double)(stamps[p][S * t + 11] - stamps[p][S * t]));
            std::sort(f.begin(), f.end());
            std::printf(" (shader clock %.0f MHz)", f[f.size() / 2]);
            std::vector<double> pr;  // slot 15: an optional probe stamp after slot 12
            for (u64 t = iters / 2; t < iters; ++t)
                if (stamps[p][S * t + 15]) pr.push_back(0.01 * (double)(stamps[p][S * t + 15] - stamps[p][S * t + 12]));
            if (!pr.empty()) {
                std::sort(pr.begin(), pr.end());
                std::printf(" (probe 12->15 %.1f)", pr[pr.size() / 2]);
            }
        }
        {
            // the circuit levels (slots 16 + lv: end of level lv; slot 5 = start of the levels)
            std::printf("\n   levels:");
            for (int lv = 0; lv < 8; ++lv) {
                std::vector<double> v;
                for (u64 t = iters / 2; t < iters; ++t) {
                    const u64 a = stamps[p][S * t + (lv ? 16 + lv - 1 : 5)], b = stamps[p][S * t + 16 + lv];
                    if (b) v.push_back(0.01 * (double)(b - a));
                }
                if (!v.empty()) {
                    std::sort(v.begin(), v.end());
                    std::printf(" L%d %.1f", lv, v[v.size() / 2]);
                }
            }
            // slots 96 + lv (lv = 1..7): level lv - 1's AND shares received and unpacked
            std::printf("\n   level lv: wait for lv-1's shares + unpack / gates:");
            for (int lv = 1; lv < 8; ++lv) {
                std::vector<double> a, b;
                for (u64 t = iters / 2; t < iters; ++t) {
                    const u64 e0 = stamps[p][S * t + 16 + lv - 1], r = stamps[p][S * t + 96 + lv],
                              e1 = stamps[p][S * t + 16 + lv];
                    if (r && e1) {
                        a.push_back(0.01 * (double)(r - e0));
                        b.push_back(0.01 * (double)(e1 - r));
                    }
                }
                if (!a.empty()) {
                    std::sort(a.begin(), a.end());
                    std::sort(b.begin(), b.end());
                    std::printf(" L%d %.2f/%.2f", lv, a[a.size() / 2], b[b.size() / 2]);
                }
            }
            // slots 32 + 4 lv + b: end of batch b of level lv (b < 4)
            std::printf("\n   batch ends after the shares (us):");
            for (int lv = 1; lv < 8; ++lv) {
                std::printf(" L%d", lv);
                for (int b = 0; b < 4; ++b) {
                    std::vector<double> v;
                    for (u64 t = iters / 2; t < iters; ++t) {
                        const u64 r = stamps[p][S * t + 96 + lv], e = stamps[p][S * t + 32 + 4 * lv + b];
                        if (r && e) v.push_back(0.01 * (double)(e - r));
                    }
                    if (v.empty()) break;
                    std::sort(v.begin(), v.end());
                    std::printf("%s%.2f", b ? "," : " ", v[v.size() / 2]);
                }
            }
            // slots 64 + 4 lv + b: thread 0 before batch b's barrier
            std::printf("\n   thread 0 before the barrier (us):");
            for (int lv = 1; lv < 8; ++lv) {
                std::printf(" L%d", lv);
                for (int b = 0; b < 4; ++b) {
                    std::vector<double> v;
                    for (u64 t = iters / 2; t < iters; ++t) {
                        const u64 r = stamps[p][S * t + 96 + lv], e = stamps[p][S * t + 64 + 4 * lv + b];
                        if (r && e) v.push_back(0.01 * (double)(e - r));
                    }
                    if (v.empty()) break;
                    std::sort(v.begin(), v.end());
                    std::printf("%s%.2f", b ? "," : " ", v[v.size() / 2]);
                }
            }
            std::printf("\n  ");
        }
        std::vector<double> gap;  // launch-to-launch gap: end of t-1 to start of t
        for (u64 t = iters / 2; t < iters; ++t) gap.push_back(0.01 * (double)(stamps[p][S * t] - stamps[p][S * (t - 1) + 11]));
        std::sort(gap.begin(), gap.end());
        std::printf(" total %.1f us, gap between launches %.1f us\n", tot, gap[gap.size() / 2]);
    }
    return 0;
}
