// aby3h_sim_* (include/aby3.h): one protocol call run by three in-process
// parties on one GPU, in the topology and with the seeds of the reference's
// unit tests (Sh3EvaluatorTests.cpp:23-131: encryptor toBlock(0, i),
// evaluator toBlock(1, i)), party 0 owning the inputs. Every party's two
// shares and the revealed result come back to the host, so a test can hold
// them against committed fixtures share by share.
#include <aby3.h>
#include <cstring>
#include <exception>
#include <thread>
#include "Basic.h"
#include "Sh3Piecewise.h"
#include "Shuffle.h"
#include "aby3ML.h"

namespace aby3 {
namespace {

thread_local std::string t_simErr;

struct SimParty {
    int idx = 0;
    Sh3Runtime rt;
    Sh3Encryptor enc;
    Sh3Evaluator eval;
};

void run3(int device, const std::function<void(SimParty&)>& f, bool mlSeeded = false) {
    // one stream per party (aux aliased below), so the parties' kernels hand
    // their messages over on the device (Channel::handoffPost)
    const int dv[3] = {device, device, device};
    // (only while every stream on the device can own a hardware queue: other
    // live streams of this process -- an open session -- count too)
    auto comms = makeLocalRing(dv, liveStreams(device) + 3 <= hwQueuesPerDevice());
    const u32 timeouts0 = handoffTimeouts(device);
    std::exception_ptr err[3];
    std::thread th[3];
    for (int i = 0; i < 3; ++i)
        th[i] = std::thread([&, i] {
            try {
                SimParty p;
                p.idx = i;
                p.rt.init(i, comms[i], device);
                p.rt.gpu().aliasAux();
                if (mlSeeded) {  // aby3ML::init (aby3ML.cpp:4-17)
                    const MlSeeds ms = mlSeeds(i);
                    p.enc.init(i, ms.encPrev, ms.encNext);
                    p.eval.init(i, ms.evalPrev, ms.evalNext);
                } else {
                    p.enc.init(i, toBlock(0, i), toBlock(0, (i + 1) % 3));
                    p.eval.init(i, toBlock(1, i), toBlock(1, (i + 1) % 3));
                }
                f(p);
                p.rt.gpu().sync();
            } catch (...) {
                err[i] = std::current_exception();
            }
        });
    for (auto& t : th) t.join();
    for (auto& e : err)
        if (e) std::rethrow_exception(e);
    // an in-kernel hand-off that gave up (here, or in a concurrent caller on
    // the device) invalidates the call
    if (handoffTimeouts(device) != timeouts0) throw std::runtime_error("in-kernel hand-off wait timed out");
}

i64Matrix hostMat(const int64_t* p, u64 r, u64 c) {
    i64Matrix m(r, c);
    std::memcpy(m.mData.data(), p, 8 * r * c);
    return m;
}

// out layout [party][share][n], as the oracle's putShared
void putShares(int party, const SharedMat& m, int64_t* out) {
    if (!out) return;
    const u64 n = m.size();
    for (int s = 0; s < 2; ++s) {
        auto v = m.shareToHost(s);
        std::memcpy(out + (2 * party + s) * n, v.data(), 8 * n);
    }
}

template <class T>
void shareIn(SimParty& p, const i64Matrix& m, T& dest) {
    if (p.idx == 0)
        p.enc.localIntMatrix(p.rt, m, dest).get();
    else
        p.enc.remoteIntMatrix(p.rt, dest).get();
}
void shareBinIn(SimParty& p, const i64Matrix& m, sbMatrix& dest) {
    if (p.idx == 0)
        p.enc.localBinMatrix(p.rt, m, dest).get();
    else
        p.enc.remoteBinMatrix(p.rt, dest).get();
}

template <class F>
int guarded(F&& f) {
    try {
        f();
        return 0;
    } catch (const std::exception& e) {
        t_simErr = e.what();
        return 1;
    }
}

}  // namespace
}  // namespace aby3

using namespace aby3;

extern "C" {

const char* aby3h_sim_last_error(void) { return t_simErr.c_str(); }

int aby3h_sim_mul(int device, int mode, int trunc, uint64_t d, const int64_t* a, const int64_t* b, uint64_t M,
                  uint64_t K, uint64_t N, int64_t* out_shares, int64_t* out_plain) {
    return guarded([&] {
        const MulMode mm = mode == 1 ? MulMode::Gemm : MulMode::Hadamard;
        const u64 br = mode == 1 ? K : M, bc = mode == 1 ? N : K;
        i64Matrix am = hostMat(a, M, K), bm = hostMat(b, br, bc);
        run3(device, [&](SimParty& p) {
            si64Matrix A(M, K), B(br, bc), C;
            shareIn(p, am, A);
            shareIn(p, bm, B);
            if (trunc)
                p.eval.asyncMul(p.rt, A, B, C, d, mm).get();
            else
                p.eval.asyncMul(p.rt, A, B, C, mm).get();
            putShares(p.idx, C, out_shares);
            i64Matrix r;
            p.enc.revealAll(p.rt, C, r).get();
            if (p.idx == 0 && out_plain) std::memcpy(out_plain, r.mData.data(), 8 * r.size());
        });
    });
}

int aby3h_sim_mul_bit(int device, int kind, const int64_t* a, int64_t apub, const int64_t* bits, uint64_t n,
                      int64_t* out_shares, int64_t* out_plain) {
    return guarded([&] {
        i64Matrix bm = hostMat(bits, n, 1);
        i64Matrix am = kind == 0 ? hostMat(a, n, 1) : i64Matrix();
        run3(device, [&](SimParty& p) {
            si64Matrix A(n, 1), C;
            sbMatrix B(n, 1);
            shareBinIn(p, bm, B);  // the oracle shares the bits first
            if (kind == 0) {
                shareIn(p, am, A);
                p.eval.asyncMul(p.rt, A, B, C).get();
            } else {
                p.eval.asyncMul(p.rt, apub, B, C).get();
            }
            putShares(p.idx, C, out_shares);
            i64Matrix r;
            p.enc.revealAll(p.rt, C, r).get();
            if (p.idx == 0 && out_plain) std::memcpy(out_plain, r.mData.data(), 8 * n);
        });
    });
}

int aby3h_sim_circuit(int device, const char* name, uint64_t size, uint64_t param, uint64_t rows, const int64_t* ins,
                      int64_t* outs, int64_t* out_shares) {
    return guarded([&] {
        CircuitLibrary lib;
        BetaCircuit* cir = lib.byName(name, size, param);
        std::vector<i64Matrix> inM;
        u64 off = 0;
        for (auto& b : cir->mInputs) {
            const u64 cols = (b.size() + 63) / 64;
            inM.push_back(hostMat(ins + off, rows, cols));
            off += rows * cols;
        }
        run3(device, [&](SimParty& p) {
            std::vector<sbMatrix> in(cir->mInputs.size()), out(cir->mOutputs.size());
            std::vector<const sbMatrix*> ip;
            std::vector<sbMatrix*> op;
            for (size_t b = 0; b < in.size(); ++b) {
                in[b].resize(rows, cir->mInputs[b].size());
                shareBinIn(p, inM[b], in[b]);
                ip.push_back(&in[b]);
            }
            for (auto& o : out) op.push_back(&o);
            CircuitLibrary local;
            evalCircuit(local.byName(name, size, param), ip, op, p.eval, p.rt);
            u64 o = 0, so = 0;
            for (auto& m : out) {
                if (out_shares) putShares(p.idx, m, out_shares + so);
                i64Matrix r;
                p.enc.revealAll(p.rt, m, r).get();
                if (p.idx == 0 && outs) std::memcpy(outs + o, r.mData.data(), 8 * r.size());
                o += m.size();
                so += 6 * m.size();
            }
        });
    });
}

int aby3h_sim_piecewise(int device, int kind, const int64_t* x, uint64_t n, uint64_t D, int64_t* out_shares,
                        int64_t* out_plain) {
    return guarded([&] {
        i64Matrix xm = hostMat(x, n, 1);
        run3(device, [&](SimParty& p) {
            si64Matrix X(n, 1), Y;
            shareIn(p, xm, X);
            Sh3Piecewise pw;
            if (kind == 0) {  // the reference's sigmoid (aby3ML.h:121-139)
                pw.mThresholds = {Sh3Piecewise::Coef(-0.5), Sh3Piecewise::Coef(0.5)};
                pw.mCoefficients.resize(3);
                pw.mCoefficients[1] = {Sh3Piecewise::Coef(0.5), Sh3Piecewise::Coef(1)};
                pw.mCoefficients[2] = {Sh3Piecewise::Coef(1)};
            } else {  // ReLU
                pw.mThresholds = {Sh3Piecewise::Coef(0)};
                pw.mCoefficients.resize(2);
                pw.mCoefficients[1] = {Sh3Piecewise::Coef(0), Sh3Piecewise::Coef(1)};
            }
            pw.eval(p.rt, X, Y, D, p.eval).get();
            putShares(p.idx, Y, out_shares);
            i64Matrix r;
            p.enc.revealAll(p.rt, Y, r).get();
            if (p.idx == 0 && out_plain) std::memcpy(out_plain, r.mData.data(), 8 * n);
        });
    });
}

int aby3h_sim_cipher_gt(int device, const int64_t* a, const int64_t* b, uint64_t n, int64_t* out_plain,
                        int64_t* out_shares) {
    return guarded([&] {
        i64Matrix am = hostMat(a, n, 1), bm = hostMat(b, n, 1);
        run3(device, [&](SimParty& p) {
            si64Matrix A(n, 1), B(n, 1);
            shareIn(p, am, A);
            shareIn(p, bm, B);
            sbMatrix g;
            cipher_gt(p.idx, A, B, g, p.eval, p.rt);
            putShares(p.idx, g, out_shares);
            i64Matrix r;
            p.enc.revealAll(p.rt, g, r).get();
            if (p.idx == 0 && out_plain) std::memcpy(out_plain, r.mData.data(), 8 * n);
        });
    });
}

int aby3h_sim_shuffle(int device, int mode, const int64_t* x, uint64_t len, uint64_t unit, int64_t* out_shares,
                      int64_t* out_pi_shares, int64_t* out_plain) {
    return guarded([&] {
        if (mode < 0 || mode > 3) throw std::runtime_error("unknown shuffle mode");
        if (mode == 1 && unit != 1) throw std::runtime_error("the sbMatrix form takes one word per row");
        if (!len || !unit) throw std::runtime_error("empty input");
        const u64 L = len * unit;
        run3(device, [&](SimParty& p) {
            // party 0 shares x [len][unit] as one binary matrix (row-major
            // draws: the same as sharing the units one after the other)
            sbMatrix X(len, 64 * unit), R(len, 64 * unit), Pi(len, 64);
            shareBinIn(p, hostMat(x, len, unit), X);
            Gpu& g = p.rt.gpu();
            if (mode == 1) {
                efficient_shuffle(X, p.idx, R, p.enc, p.eval, p.rt);
            } else if (mode == 3) {
                efficient_shuffle_units(reinterpret_cast<const u64*>(X.data()), len, unit, p.idx,
                                        reinterpret_cast<u64*>(R.data()), p.enc, p.rt);
            } else {
                // the reference's vector<sbMatrix> form: one unit per matrix
                std::vector<sbMatrix> T(len), Tres;
                for (u64 i = 0; i < len; ++i) {
                    T[i].resize(unit, 64);
                    for (int sh = 0; sh < 2; ++sh) d2d(T[i].share(sh), X.share(sh) + i * unit, 8 * unit, g);
                }
                std::vector<si64> pi;
                if (mode == 0)
                    efficient_shuffle(T, p.idx, Tres, p.enc, p.eval, p.rt);
                else
                    efficient_shuffle_with_random_permutation(T, p.idx, Tres, pi, p.enc, p.eval, p.rt);
                for (u64 i = 0; i < len; ++i)
                    for (int sh = 0; sh < 2; ++sh) d2d(R.share(sh) + i * unit, Tres[i].share(sh), 8 * unit, g);
                if (mode == 2) {
                    std::vector<i64> h(2 * len);
                    for (u64 i = 0; i < len; ++i) {
                        h[i] = pi[i].mData[0];
                        h[len + i] = pi[i].mData[1];
                    }
                    toDevice(Pi.data(), h.data(), 16 * len, g);
                }
            }
            putShares(p.idx, R, out_shares);
            if (mode == 2) putShares(p.idx, Pi, out_pi_shares);
            i64Matrix r;
            p.enc.revealAll(p.rt, R, r).get();
            if (p.idx == 0 && out_plain) std::memcpy(out_plain, r.mData.data(), 8 * L);
        });
    });
}

int aby3h_sim_merge(int device, int mode, const uint64_t* lens, uint64_t nlists, uint64_t dim, const int64_t* keys,
                    int64_t* out_sorted, int64_t* out_shares) {
    return guarded([&] {
        if (mode < 0 || mode > 5) throw std::runtime_error("unknown merge mode");
        if (!nlists) throw std::runtime_error("no lists");
        std::vector<i64Matrix> lists;
        u64 off = 0;
        for (u64 k = 0; k < nlists; ++k) {
            lists.push_back(hostMat(keys + off, lens[k], 1));
            off += lens[k];
        }
        const u64 total = off;
        if ((mode == 2 || mode == 3 || mode == 5) && (!dim || nlists % dim)) throw std::runtime_error("nlists must be a multiple of dim");
        if (mode == 3 && nlists != 2 * dim) throw std::runtime_error("high_dimensional_odd_even_merge: 2 lists per dim");
        run3(device, [&](SimParty& p) {
            sbMatrix sorted;
            if (mode == 0 || mode == 4) {
                std::vector<sbMatrix> data(nlists);
                for (u64 k = 0; k < nlists; ++k) {
                    data[k].resize(lens[k], 64);
                    shareBinIn(p, lists[k], data[k]);
                }
                odd_even_multi_merge(data, sorted, p.idx, p.eval, p.rt,
                                     mode == 4 ? MergeOrder::Sequential : MergeOrder::Batched);
            } else if (mode == 1) {
                sbMatrix flat(total, 64);
                shareBinIn(p, hostMat(keys, total, 1), flat);
                if (nlists == total)
                    odd_even_merge_sort(flat, sorted, p.idx, p.eval, p.rt);
                else
                    odd_even_multi_merge(flat, std::vector<u64>(lens, lens + nlists), sorted, p.idx, p.eval, p.rt);
            } else {
                const u64 k = nlists / dim;
                std::vector<std::vector<sbMatrix>> data(dim);
                for (u64 i = 0; i < dim; ++i) {
                    data[i].resize(k);
                    for (u64 j = 0; j < k; ++j) {
                        data[i][j].resize(lens[i * k + j], 64);
                        shareBinIn(p, lists[i * k + j], data[i][j]);
                    }
                }
                std::vector<sbMatrix> out;
                if (mode == 2 || mode == 5) {
                    high_dimensional_odd_even_multi_merge(data, out, p.idx, p.eval, p.rt,
                                                          mode == 5 ? MergeOrder::Sequential : MergeOrder::Batched);
                } else {
                    std::vector<sbMatrix> d1(dim), d2(dim);
                    for (u64 i = 0; i < dim; ++i) {
                        d1[i] = std::move(data[i][0]);
                        d2[i] = std::move(data[i][1]);
                    }
                    high_dimensional_odd_even_merge(d1, d2, out, p.idx, p.eval, p.rt);
                }
                sorted.resize(total, 64);
                u64 o = 0;
                for (auto& x : out) {
                    for (int s = 0; s < 2; ++s)
                        if (x.rows()) d2d(sorted.share(s) + o, x.share(s), x.rows() * 8, p.rt.gpu());
                    o += x.rows();
                }
            }
            putShares(p.idx, sorted, out_shares);
            i64Matrix r;
            p.enc.revealAll(p.rt, sorted, r).get();
            if (p.idx == 0 && out_sorted) std::memcpy(out_sorted, r.mData.data(), 8 * r.size());
        });
    });
}

int aby3h_sim_lr(int device, uint64_t n, uint64_t d, uint64_t B, uint64_t D, uint64_t aB, uint64_t iters,
                 const int64_t* X, const int64_t* Y, const uint64_t* batches, int64_t* out_w_shares,
                 int64_t* out_w_plain) {
    return guarded([&] {
        if (!n || !d || !B) throw std::runtime_error("empty LR shapes");
        i64Matrix xm = hostMat(X, n, d), ym = hostMat(Y, n, 1), w0(d, 1);
        std::vector<u32> idx(iters * B);
        for (u64 i = 0; i < idx.size(); ++i) {
            if (batches[i] >= n) throw std::runtime_error("batch index out of range");
            idx[i] = (u32)batches[i];
        }
        run3(
            device,
            [&](SimParty& p) {
                si64Matrix sX(n, d), sY(n, 1), sW(d, 1);
                shareIn(p, xm, sX);
                shareIn(p, ym, sY);
                shareIn(p, w0, sW);
                aby3ML ml(p.rt, p.enc, p.eval, D);
                SgdState st;
                for (u64 t = 0; t < iters; ++t)
                    sgdLogisticStep(ml, sX, sY, sW, std::vector<u32>(idx.begin() + t * B, idx.begin() + (t + 1) * B),
                                    aB, st);
                putShares(p.idx, sW, out_w_shares);
                i64Matrix r;
                p.enc.revealAll(p.rt, sW, r).get();
                if (p.idx == 0 && out_w_plain) std::memcpy(out_w_plain, r.mData.data(), 8 * d);
            },
            true);
    });
}

int aby3h_lr_dataset(uint64_t n, uint64_t dim, uint64_t D, int64_t* X, int64_t* Y, double* model) {
    return guarded([&] {
        auto m = logisticModel(dim);
        if (model) std::memcpy(model, m.data(), 8 * dim);
        if (!X && !Y) return;
        i64Matrix x, y;
        logisticModelGen(m, n, D, x, y);
        if (X) std::memcpy(X, x.data(), 8 * x.size());
        if (Y) std::memcpy(Y, y.data(), 8 * n);
    });
}

int aby3h_lr_batches(uint64_t n, uint64_t B, uint64_t iters, uint64_t* out) {
    return guarded([&] {
        BatchSampler s(n);
        std::vector<u64> b(B);
        for (u64 t = 0; t < iters; ++t) {
            s.next(b);
            std::memcpy(out + t * B, b.data(), 8 * B);
        }
    });
}

}  // extern "C"
