// TEST INFRASTRUCTURE ONLY -- C entry points of the CPU oracle for ctypes
// (tests/oracle.py). Plain pointers and sizes; errors return nonzero.
#include "orc_core.h"
#include <cstring>
#include <string>
#include <chrono>
#include <thread>

using namespace orc;

namespace {
thread_local std::string g_err;
template <class F>
int guard(F&& f) {
    try {
        f();
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return 1;
    }
}
Mat toMat(const int64_t* p, u64 r, u64 c) {
    Mat m(r, c);
    memcpy(m.v.data(), p, 8 * r * c);
    return m;
}
SMat toSMat(const int64_t* s0, const int64_t* s1, u64 r, u64 c) {
    SMat m;
    m.s[0] = toMat(s0, r, c);
    m.s[1] = toMat(s1, r, c);
    return m;
}
// shares layout for the 3-party outputs: [party][share][rows*cols]
void putShared(const Shared& x, int64_t* out) {
    u64 n = x[0].size();
    for (int p = 0; p < 3; ++p)
        for (int s = 0; s < 2; ++s) memcpy(out + (2 * p + s) * n, x[p].s[s].v.data(), 8 * n);
}
Circuit toCircuit(uint32_t wires, const uint32_t* gates, uint64_t ngates, const uint32_t* levels, uint64_t nlevels,
                  const uint32_t* inWires, const uint32_t* inSizes, uint64_t nin, const uint32_t* outWires,
                  const uint32_t* outSizes, uint64_t nout) {
    Circuit c;
    c.wireCount = wires;
    c.gates.resize(ngates);
    for (u64 g = 0; g < ngates; ++g) c.gates[g] = Gate{gates[4 * g], gates[4 * g + 1], gates[4 * g + 2], gates[4 * g + 3]};
    c.levelCounts.assign(levels, levels + nlevels);
    u64 o = 0;
    for (u64 b = 0; b < nin; ++b) {
        c.inputs.emplace_back(inWires + o, inWires + o + inSizes[b]);
        o += inSizes[b];
    }
    o = 0;
    for (u64 b = 0; b < nout; ++b) {
        c.outputs.emplace_back(outWires + o, outWires + o + outSizes[b]);
        o += outSizes[b];
    }
    return c;
}
}  // namespace

extern "C" {

const char* orc_last_error() { return g_err.c_str(); }
int orc_aesni_available() { return aesni_available() ? 1 : 0; }

int orc_aes_ref_encrypt(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]) {
    return guard([&] {
        AesRef a;
        a.setKey(key);
        a.encrypt(in, out);
    });
}

int orc_aes_ctr(const uint8_t key[16], uint64_t base, uint64_t n, uint8_t* out, int use_ref) {
    return guard([&] {
        if (use_ref) {
            AesRef a;
            a.setKey(key);
            for (u64 i = 0; i < n; ++i) {
                Block b = a.encrypt(toBlock(base + i));
                memcpy(out + 16 * i, &b, 16);
            }
        } else {
            AesNI a;
            a.setKey(key);
            a.ctr(base, n, (Block*)out);
        }
    });
}

int orc_prng_bytes(const uint8_t seed[16], uint64_t off, uint64_t n, uint8_t* out) {
    return guard([&] { prng_bytes(seed, off, n, out); });
}

// Sh3ShareGen draws j = base .. base+n-1 with keys (k_prev, k_next).
// kind 0: getShare, 1: getBinaryShare, 2: getRandIntShare (out0 = r[0], out1 = r[1])
int orc_share_draws(int kind, const uint8_t kprev[16], const uint8_t knext[16], uint64_t base, uint64_t n,
                    int64_t* out0, int64_t* out1) {
    return guard([&] {
        ShareGen g;
        g.key[0].setKey(kprev);
        g.key[1].setKey(knext);
        g.drawIdx = base;
        for (u64 i = 0; i < n; ++i) {
            if (kind == 0)
                out0[i] = g.getShare();
            else if (kind == 1)
                out0[i] = g.getBinaryShare();
            else {
                auto r = g.getRandIntShare();
                out0[i] = r[0];
                out1[i] = r[1];
            }
        }
    });
}

// Keys a party derives in Sh3ShareGen::init + Sh3Evaluator::init:
// out = [kSharePrev | kShareNext | kOtPrev | kOtNext] (4 x 16 bytes)
int orc_party_keys(const uint8_t prevSeed[16], const uint8_t nextSeed[16], uint8_t out[64]) {
    return guard([&] {
        Party p;
        Block ps, ns;
        memcpy(&ps, prevSeed, 16);
        memcpy(&ns, nextSeed, 16);
        p.initEvaluator(0, ps, ns);
        memcpy(out, p.gen.keyBytes[0], 16);
        memcpy(out + 16, p.gen.keyBytes[1], 16);
        prng_bytes(nextSeed, 16, 16, out + 32);
        prng_bytes(prevSeed, 16, 16, out + 48);
    });
}

int orc_local_product(int mode, const int64_t* A0, const int64_t* A1, const int64_t* B0, const int64_t* B1, uint64_t M,
                      uint64_t K, uint64_t N, int64_t* C0) {
    return guard([&] {
        SMat A = toSMat(A0, A1, M, K);
        SMat B = mode == MUL_GEMM ? toSMat(B0, B1, K, N) : toSMat(B0, B1, M, K);
        Mat c;
        localProduct((MulMode)mode, A, B, c);
        memcpy(C0, c.v.data(), 8 * c.size());
    });
}

// getTruncationTuple with the next/prev streams at the given byte offsets.
int orc_trunc_tuple(const uint8_t nextSeed[16], uint64_t nextOff, const uint8_t prevSeed[16], uint64_t prevOff,
                    uint64_t n, uint64_t d, int64_t* R, int64_t* RT0, int64_t* RT1) {
    return guard([&] {
        Party p;
        p.gen.next.init(nextSeed);
        p.gen.next.off = nextOff;
        p.gen.prev.init(prevSeed);
        p.gen.prev.off = prevOff;
        TruncPair t = truncationTuple(p, n, 1, d);
        memcpy(R, t.R.v.data(), 8 * n);
        memcpy(RT0, t.RT.s[0].v.data(), 8 * n);
        memcpy(RT1, t.RT.s[1].v.data(), 8 * n);
    });
}

// Full 3-party protocol simulations from plaintext inputs. Inputs are shared
// by party 0 with Encryptor seeds toBlock(0, i); the evaluator uses
// toBlock(1, i) (Sh3EvaluatorTests.cpp:617-623). out_shares: [3][2][n].
int orc_sim_mul(int mode, int trunc, uint64_t d, const int64_t* a, const int64_t* b, uint64_t M, uint64_t K,
                uint64_t N, int64_t* out_shares, int64_t* out_plain) {
    return guard([&] {
        auto enc = makeEncryptors(0);
        auto ev = makeEvaluators(1);
        Mat am = toMat(a, M, K);
        Mat bm = mode == MUL_GEMM ? toMat(b, K, N) : toMat(b, M, K);
        Shared A = shareInt(enc, 0, am), B = shareInt(enc, 0, bm);
        Shared C = trunc ? mulTrunc(ev, (MulMode)mode, A, B, d) : mul(ev, (MulMode)mode, A, B);
        if (!consistent(C)) throw std::runtime_error("inconsistent shares");
        putShared(C, out_shares);
        Mat r = revealInt(C);
        memcpy(out_plain, r.v.data(), 8 * r.size());
    });
}

// a * b for a shared i64 vector and a shared bit vector (kind 0, Sh3Evaluator.cpp:119-263)
// or public a * shared bit (kind 1, :418-501).
int orc_sim_mul_bit(int kind, const int64_t* a, int64_t apub, const int64_t* bits, uint64_t n, int64_t* out_shares,
                    int64_t* out_plain) {
    return guard([&] {
        auto enc = makeEncryptors(0);
        auto ev = makeEvaluators(1);
        Shared B = shareBin(enc, 0, toMat(bits, n, 1));
        Shared C;
        if (kind == 0) {
            Shared A = shareInt(enc, 0, toMat(a, n, 1));
            C = mulBit(ev, A, B);
        } else {
            C = mulPubBit(ev, apub, B);
        }
        if (!consistent(C)) throw std::runtime_error("inconsistent shares");
        putShared(C, out_shares);
        Mat r = revealInt(C);
        memcpy(out_plain, r.v.data(), 8 * n);
    });
}

// Evaluate a serialized circuit on binary-shared 64-bit inputs (one i64 column
// per 64 input wires). ins: [nin][rows*inCols[b]]; outs: revealed [nout][rows*outCols].
int orc_sim_circuit(uint32_t wires, const uint32_t* gates, uint64_t ngates, const uint32_t* levels, uint64_t nlevels,
                    const uint32_t* inWires, const uint32_t* inSizes, uint64_t nin, const uint32_t* outWires,
                    const uint32_t* outSizes, uint64_t nout, uint64_t rows, const int64_t* ins, int64_t* outs,
                    int64_t* out_shares) {
    return guard([&] {
        Circuit c = toCircuit(wires, gates, ngates, levels, nlevels, inWires, inSizes, nin, outWires, outSizes, nout);
        auto enc = makeEncryptors(0);
        auto ev = makeEvaluators(1);
        std::vector<Shared> sh(nin);
        u64 off = 0;
        std::vector<const Shared*> ptrs;
        for (u64 b = 0; b < nin; ++b) {
            u64 cols = (inSizes[b] + 63) / 64;
            sh[b] = shareBin(enc, 0, toMat(ins + off, rows, cols));
            off += rows * cols;
        }
        for (auto& s : sh) ptrs.push_back(&s);
        auto o = evalCircuit(ev, c, ptrs);
        off = 0;
        u64 soff = 0;
        for (u64 b = 0; b < nout; ++b) {
            if (!consistent(o[b])) throw std::runtime_error("inconsistent shares");
            Mat r = revealBin(o[b]);
            memcpy(outs + off, r.v.data(), 8 * r.size());
            off += r.size();
            if (out_shares) {
                putShared(o[b], out_shares + soff);
                soff += 6 * r.size();
            }
        }
    });
}

// Piecewise eval (3PC) with the reference's sigmoid (aby3ML.h:121-139) or a
// ReLU-like (thresholds {0}, coefs {{}, {0, 1}}): kind 0 sigmoid, 1 relu.
int orc_sim_piecewise(int kind, uint32_t wires, const uint32_t* gates, uint64_t ngates, const uint32_t* levels,
                      uint64_t nlevels, const uint32_t* inWires, const uint32_t* inSizes, uint64_t nin,
                      const uint32_t* outWires, const uint32_t* outSizes, uint64_t nout, const int64_t* x, uint64_t n,
                      uint64_t D, int64_t* out_shares, int64_t* out_plain) {
    return guard([&] {
        Circuit c = toCircuit(wires, gates, ngates, levels, nlevels, inWires, inSizes, nin, outWires, outSizes, nout);
        Piecewise pw;
        if (kind == 0) {
            pw.thresholds = {Coef{false, 0, -0.5}, Coef{false, 0, 0.5}};
            pw.coefs = {{}, {Coef{false, 0, 0.5}, Coef{true, 1, 0}}, {Coef{true, 1, 0}}};
        } else {
            pw.thresholds = {Coef{true, 0, 0}};
            pw.coefs = {{}, {Coef{true, 0, 0}, Coef{true, 1, 0}}};
        }
        auto enc = makeEncryptors(0);
        auto ev = makeEvaluators(1);
        Shared X = shareInt(enc, 0, toMat(x, n, 1));
        Shared Y = piecewiseEval(ev, pw, c, X, D);
        if (!consistent(Y)) throw std::runtime_error("inconsistent shares");
        putShared(Y, out_shares);
        Mat r = revealInt(Y);
        memcpy(out_plain, r.v.data(), 8 * n);
    });
}

int orc_sim_fetch_msb(uint32_t wires, const uint32_t* gates, uint64_t ngates, const uint32_t* levels,
                      uint64_t nlevels, const uint32_t* inWires, const uint32_t* inSizes, uint64_t nin,
                      const uint32_t* outWires, const uint32_t* outSizes, uint64_t nout, const int64_t* a,
                      const int64_t* b, uint64_t n, int64_t* out_plain, int64_t* out_shares) {
    return guard([&] {
        Circuit c = toCircuit(wires, gates, ngates, levels, nlevels, inWires, inSizes, nin, outWires, outSizes, nout);
        auto enc = makeEncryptors(0);
        auto ev = makeEvaluators(1);
        Shared A = shareInt(enc, 0, toMat(a, n, 1));
        Shared B = shareInt(enc, 0, toMat(b, n, 1));
        // cipher_gt: diff = B - A (BuildingBlocks.cpp:525-532)
        Shared diff = A;
        for (int p = 0; p < 3; ++p)
            for (int s = 0; s < 2; ++s)
                for (u64 k = 0; k < n; ++k)
                    diff[p].s[s].v[k] = (i64)((u64)B[p].s[s].v[k] - (u64)A[p].s[s].v[k]);
        Shared r = fetchMsb(ev, c, diff);
        if (out_shares) putShared(r, out_shares);
        Mat m = revealBin(r);
        memcpy(out_plain, m.v.data(), 8 * n);
    });
}

// The merge network (Sort.cpp:327-628) on binary-shared 64-bit keys, with the
// supplied cmp_swap circuit. mode 0: odd_even_multi_merge, each of the nlists
// lists shared on its own; 1: the same over all keys shared as one matrix;
// 2: high_dimensional_odd_even_multi_merge, lists [dim][nlists / dim] shared
// in that order; 3: high_dimensional_odd_even_merge (nlists = 2 * dim);
// 4 / 5: mode 0 / 2 with the reference's sequential merge order.
// out_sorted / out_shares: the merged list(s) back to back.
int orc_sim_merge(uint32_t wires, const uint32_t* gates, uint64_t ngates, const uint32_t* levels, uint64_t nlevels,
                  const uint32_t* inWires, const uint32_t* inSizes, uint64_t nin, const uint32_t* outWires,
                  const uint32_t* outSizes, uint64_t nout, int mode, const uint64_t* lens, uint64_t nlists,
                  uint64_t dim, const int64_t* keys, int64_t* out_sorted, int64_t* out_shares) {
    return guard([&] {
        Circuit c = toCircuit(wires, gates, ngates, levels, nlevels, inWires, inSizes, nin, outWires, outSizes, nout);
        auto enc = makeEncryptors(0);
        auto ev = makeEvaluators(1);
        u64 total = 0;
        for (u64 k = 0; k < nlists; ++k) total += lens[k];
        Shared res;
        if (mode == 0 || mode == 1 || mode == 4) {
            Shared flat;
            if (mode == 1) {
                flat = shareBin(enc, 0, toMat(keys, total, 1));
            } else {
                for (int p = 0; p < 3; ++p) flat[p] = SMat(total, 1);
                u64 off = 0;
                for (u64 k = 0; k < nlists; ++k) {
                    Shared x = shareBin(enc, 0, toMat(keys + off, lens[k], 1));
                    for (int p = 0; p < 3; ++p)
                        for (int s = 0; s < 2; ++s)
                            std::copy(x[p].s[s].v.begin(), x[p].s[s].v.end(), flat[p].s[s].v.begin() + off);
                    off += lens[k];
                }
            }
            res = multiMerge(ev, c, flat, std::vector<u64>(lens, lens + nlists), mode == 4);
        } else if (mode == 2 || mode == 3 || mode == 5) {
            if (!dim || nlists % dim) throw std::runtime_error("nlists must be a multiple of dim");
            const u64 k = nlists / dim;
            if (mode == 3 && k != 2) throw std::runtime_error("high_dimensional_odd_even_merge takes two lists per dim");
            std::vector<std::vector<Shared>> data(dim, std::vector<Shared>(k));
            u64 off = 0, li = 0;
            for (u64 i = 0; i < dim; ++i)
                for (u64 j = 0; j < k; ++j, ++li) {
                    data[i][j] = shareBin(enc, 0, toMat(keys + off, lens[li], 1));
                    off += lens[li];
                }
            auto sorted = hdMultiMerge(ev, c, data, mode == 5);
            for (int p = 0; p < 3; ++p) res[p] = SMat(total, 1);
            off = 0;
            for (auto& x : sorted) {
                for (int p = 0; p < 3; ++p)
                    for (int s = 0; s < 2; ++s)
                        std::copy(x[p].s[s].v.begin(), x[p].s[s].v.end(), res[p].s[s].v.begin() + off);
                off += x[0].rows();
            }
        } else {
            throw std::runtime_error("unknown merge mode");
        }
        if (!consistent(res)) throw std::runtime_error("inconsistent shares");
        Mat m = revealBin(res);
        if (out_sorted) memcpy(out_sorted, m.v.data(), 8 * total);
        if (out_shares) putShared(res, out_shares);
    });
}

// CPU baseline of asyncMul + truncation (bench.py cpu_baseline): the three
// parties' round-1 local compute (three scalar i64 GEMMs as Eigen evaluates
// A0*B0 + A0*B1 + A1*B0, Sh3Evaluator.cpp:662-665, plus the truncation tuple
// from AES-NI PRNG streams) run concurrently, one thread per party like the
// reference's one compute thread per party process, followed by the round-2
// finalize of P0/P1. Returns wall seconds for `reps` multiplications.
double orc_bench_mul_trunc(int mode, uint64_t M, uint64_t K, uint64_t N, uint64_t d, int reps) {
    try {
        auto ev = makeEvaluators(1);
        std::array<SMat, 3> A, B;
        u64 x = 42;
        auto rnd = [&](SMat& m, u64 r, u64 c) {
            m = SMat(r, c);
            for (int s = 0; s < 2; ++s)
                for (auto& v : m.s[s].v) {
                    x ^= x << 13;
                    x ^= x >> 7;
                    x ^= x << 17;
                    v = (i64)x;
                }
        };
        for (int p = 0; p < 3; ++p) {
            rnd(A[p], M, K);
            rnd(B[p], mode == MUL_GEMM ? K : M, mode == MUL_GEMM ? N : K);
        }
        auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < reps; ++r) {
            std::array<Mat, 3> z;
            std::array<SMat, 3> C;
            std::vector<std::thread> th;
            for (int p = 0; p < 3; ++p)
                th.emplace_back([&, p] { mulTruncLocal(ev[p], (MulMode)mode, A[p], B[p], d, z[p], C[p]); });
            for (auto& t : th) t.join();
            Mat s = z[0];
            for (u64 k = 0; k < s.size(); ++k) s.v[k] = (i64)((u64)z[0].v[k] + (u64)z[1].v[k] + (u64)z[2].v[k]);
            for (int p = 0; p < 2; ++p) truncFinalize(p, s, d, C[p]);
        }
        auto t1 = std::chrono::steady_clock::now();
        return std::chrono::duration<double>(t1 - t0).count();
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}


// The shuffles of aby3-Basic/Shuffle.cpp by three parties with the
// encryptor seeds toBlock(0, i): x [len][unit] shared by party 0 as one
// binary matrix. mode 0 efficient_shuffle(vector<sbMatrix>), 1
// efficient_shuffle(sbMatrix) (unit 1), 2 efficient_shuffle_with_random_
// permutation. out_shares [3][2][len*unit], out_pi_shares [3][2][len] (mode 2),
// out_plain [len*unit]; any may be NULL.
int orc_sim_shuffle(int mode, const int64_t* x, uint64_t len, uint64_t unit, int64_t* out_shares,
                    int64_t* out_pi_shares, int64_t* out_plain) {
    return guard([&] {
        if (mode < 0 || mode > 2) throw std::runtime_error("unknown shuffle mode");
        if (mode == 1 && unit != 1) throw std::runtime_error("the sbMatrix form takes one word per row");
        auto enc = makeEncryptors(0);
        Shared T = shareBin(enc, 0, toMat(x, len, unit));
        Shared pi, out;
        if (mode == 0)
            out = shuffleUnits(enc, T);
        else if (mode == 1)
            out = shuffleRows(enc, T);
        else
            out = shuffleWithPermutation(enc, T, pi);
        if (!consistent(out) || (mode == 2 && !consistent(pi))) throw std::runtime_error("inconsistent shares");
        if (out_shares) putShared(out, out_shares);
        if (out_pi_shares && mode == 2) putShared(pi, out_pi_shares);
        if (out_plain) {
            Mat r = revealBin(out);
            memcpy(out_plain, r.v.data(), 8 * r.size());
        }
    });
}

// get_permutation(len, seed) (BoolBasic.cpp:925-934)
int orc_shuffle_permutation(uint64_t len, const uint8_t seed[16], uint64_t* out) {
    return guard([&] {
        auto p = shufflePermutation(len, seed);
        memcpy(out, p.data(), 8 * len);
    });
}

// CPU baseline of C1: asyncMul without truncation
// (Sh3Evaluator.cpp:92-116), one thread per party: each party's local share
// product as Eigen evaluates it (three i64 products, or the fork's
// element-wise loop) plus its zero-share, then the ring reshare (a copy of
// C0 to the next party). Seconds for `reps` multiplications.
double orc_bench_mul(int mode, uint64_t M, uint64_t K, uint64_t N, int reps) {
    try {
        auto ev = makeEvaluators(1);
        std::array<SMat, 3> A, B;
        u64 x = 43;
        auto rnd = [&](SMat& m, u64 r, u64 c) {
            m = SMat(r, c);
            for (int s = 0; s < 2; ++s)
                for (auto& v : m.s[s].v) {
                    x ^= x << 13;
                    x ^= x >> 7;
                    x ^= x << 17;
                    v = (i64)x;
                }
        };
        for (int p = 0; p < 3; ++p) {
            rnd(A[p], M, K);
            rnd(B[p], mode == MUL_GEMM ? K : M, mode == MUL_GEMM ? N : K);
        }
        auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < reps; ++r) {
            std::array<SMat, 3> C;
            std::vector<std::thread> th;
            for (int p = 0; p < 3; ++p)
                th.emplace_back([&, p] {
                    Mat c0;
                    localProduct((MulMode)mode, A[p], B[p], c0);
                    for (u64 k = 0; k < c0.size(); ++k) c0.v[k] = (i64)((u64)c0.v[k] + (u64)ev[p].gen.getShare());
                    C[p].s[0] = std::move(c0);
                });
            for (auto& t : th) t.join();
            for (int p = 0; p < 3; ++p) C[(p + 1) % 3].s[1] = C[p].s[0];
        }
        auto t1 = std::chrono::steady_clock::now();
        return std::chrono::duration<double>(t1 - t0).count();
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

// CPU baseline of cipher_gt / fetch_msb (bench.py binary cpu_baseline for C3,
// BuildingBlocks.cpp:464-532): diff = B - A, the two-input binary resharing,
// and the 64-bit MSB circuit evaluated by the three parties (bit-sliced u64
// gate loops, AES-NI z masks, Sh3BinaryEvaluator.cpp:539-1464), simulated in
// sequence on one thread (no network). Inputs: n random 62-bit pairs shared
// by party 0 (untimed). Returns wall seconds for `reps` evaluations.
double orc_bench_fetch_msb(uint32_t wires, const uint32_t* gates, uint64_t ngates, const uint32_t* levels,
                           uint64_t nlevels, const uint32_t* inWires, const uint32_t* inSizes, uint64_t nin,
                           const uint32_t* outWires, const uint32_t* outSizes, uint64_t nout, uint64_t n, int reps) {
    try {
        Circuit c = toCircuit(wires, gates, ngates, levels, nlevels, inWires, inSizes, nin, outWires, outSizes, nout);
        auto enc = makeEncryptors(0);
        auto ev = makeEvaluators(1);
        Mat a(n, 1), b(n, 1);
        u64 x = 88172645463325252ull;
        for (u64 k = 0; k < n; ++k) {
            x ^= x << 13, x ^= x >> 7, x ^= x << 17;
            a.v[k] = (i64)(x >> 2);
            x ^= x << 13, x ^= x >> 7, x ^= x << 17;
            b.v[k] = (i64)(x >> 2);
        }
        Shared A = shareInt(enc, 0, a), B = shareInt(enc, 0, b);
        auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < reps; ++r) {
            Shared diff = A;
            for (int p = 0; p < 3; ++p)
                for (int s = 0; s < 2; ++s)
                    for (u64 k = 0; k < n; ++k)
                        diff[p].s[s].v[k] = (i64)((u64)B[p].s[s].v[k] - (u64)A[p].s[s].v[k]);
            Shared res = fetchMsb(ev, c, diff);
            if (res[0].s[0].v.empty()) throw std::runtime_error("empty result");
        }
        auto t1 = std::chrono::steady_clock::now();
        return std::chrono::duration<double>(t1 - t0).count();
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

// CPU baseline of one SGD_Logistic iteration (bench.py cpu_baseline for C4,
// Regression.h:249-293) on the LogisticModelGen dataset (n x d, fixed point
// D) with aby3ML's seeds and getSubset's batches: batch gather, xw = X_B w
// (GEMM + truncation D), sigmoid piecewise (2 MSB circuits + OT products),
// err = f - Y_B, X_B^T err >> (D + aB), w -= update. Three parties simulated in
// sequence on one thread (no network). Returns wall seconds for `iters`
// iterations (after one untimed iteration).
double orc_bench_lr(uint32_t wires, const uint32_t* gates, uint64_t ngates, const uint32_t* levels, uint64_t nlevels,
                    const uint32_t* inWires, const uint32_t* inSizes, uint64_t nin, const uint32_t* outWires,
                    const uint32_t* outSizes, uint64_t nout, uint64_t n, uint64_t d, uint64_t B, uint64_t D,
                    uint64_t aB, int iters) {
    try {
        Circuit c = toCircuit(wires, gates, ngates, levels, nlevels, inWires, inSizes, nin, outWires, outSizes, nout);
        std::array<Party, 3> enc, ev;
        mlParties(enc, ev);
        Mat X, Y, w0(d, 1);
        logisticModelGen(logisticModel(d), n, D, X, Y);
        Shared sX = shareInt(enc, 0, X), sY = shareInt(enc, 0, Y), sW = shareInt(enc, 0, w0);
        BatchSampler sampler(n);
        std::vector<u64> batch(B);
        sampler.next(batch);
        sgdLogisticIteration(ev, c, sX, sY, sW, batch, D, aB);
        auto t0 = std::chrono::steady_clock::now();
        for (int t = 0; t < iters; ++t) {
            sampler.next(batch);
            sgdLogisticIteration(ev, c, sX, sY, sW, batch, D, aB);
        }
        auto t1 = std::chrono::steady_clock::now();
        return std::chrono::duration<double>(t1 - t0).count();
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

// The C4 dataset (LogisticModelGen, fixed point D): X [n][dim], Y [n],
// model [dim] (any output may be NULL).
int orc_lr_dataset(uint64_t n, uint64_t dim, uint64_t D, int64_t* X, int64_t* Y, double* model) {
    return guard([&] {
        auto m = logisticModel(dim);
        if (model) memcpy(model, m.data(), 8 * dim);
        if (!X && !Y) return;
        Mat x, y;
        logisticModelGen(m, n, D, x, y);
        if (X) memcpy(X, x.v.data(), 8 * x.size());
        if (Y) memcpy(Y, y.v.data(), 8 * n);
    });
}

// logisticLabelMargin of the C4 dataset's first n rows (orc_ml.cpp)
int orc_lr_label_margin(uint64_t n, uint64_t dim, double* margin) {
    return guard([&] { *margin = logisticLabelMargin(logisticModel(dim), n); });
}

// getSubset's first `iters` mini-batches of B indices over n rows: out [iters][B]
int orc_lr_batches(uint64_t n, uint64_t B, uint64_t iters, uint64_t* out) {
    return guard([&] {
        BatchSampler s(n);
        std::vector<u64> b(B);
        for (u64 t = 0; t < iters; ++t) {
            s.next(b);
            memcpy(out + t * B, b.data(), 8 * B);
        }
    });
}

// `iters` SGD_Logistic iterations, 3 parties with aby3ML's seeds: party 0
// shares X [n][d], Y [n], w = 0 [d] (localFixedMatrix, in that order), then
// iteration t uses batch [t][B]. out_w_shares [3][2][d], out_w_plain [d].
int orc_sim_lr(uint32_t wires, const uint32_t* gates, uint64_t ngates, const uint32_t* levels, uint64_t nlevels,
               const uint32_t* inWires, const uint32_t* inSizes, uint64_t nin, const uint32_t* outWires,
               const uint32_t* outSizes, uint64_t nout, uint64_t n, uint64_t d, uint64_t B, uint64_t D, uint64_t aB,
               uint64_t iters, const int64_t* X, const int64_t* Y, const uint64_t* batches, int64_t* out_w_shares,
               int64_t* out_w_plain) {
    return guard([&] {
        Circuit c = toCircuit(wires, gates, ngates, levels, nlevels, inWires, inSizes, nin, outWires, outSizes, nout);
        std::array<Party, 3> enc, ev;
        mlParties(enc, ev);
        Shared sX = shareInt(enc, 0, toMat(X, n, d)), sY = shareInt(enc, 0, toMat(Y, n, 1));
        Shared sW = shareInt(enc, 0, Mat(d, 1));
        for (u64 t = 0; t < iters; ++t) {
            std::vector<u64> batch(batches + t * B, batches + (t + 1) * B);
            for (u64 r : batch)
                if (r >= n) throw std::runtime_error("batch index out of range");
            sgdLogisticIteration(ev, c, sX, sY, sW, batch, D, aB);
        }
        if (!consistent(sW)) throw std::runtime_error("inconsistent shares");
        if (out_w_shares) putShared(sW, out_w_shares);
        Mat w = revealInt(sW);
        if (out_w_plain) memcpy(out_w_plain, w.v.data(), 8 * d);
    });
}

}  // extern "C"

// CPU baselines of the share conversions (bench.py cpu_baseline legs for the
// Sh3Converter lines): n random 64-bit values shared by party 0 (untimed),
// then `reps` toBinaryMatrix calls (Sh3Converter.cpp:61-207, the adder circuit
// passed in) / bitInjection calls (:209-370) of the three parties simulated in
// sequence on one thread (no network). Return wall seconds.
extern "C" double orc_bench_a2b(uint32_t wires, const uint32_t* gates, uint64_t ngates, const uint32_t* levels,
                                uint64_t nlevels, const uint32_t* inWires, const uint32_t* inSizes, uint64_t nin,
                                const uint32_t* outWires, const uint32_t* outSizes, uint64_t nout, uint64_t n,
                                int reps) {
    try {
        Circuit c = toCircuit(wires, gates, ngates, levels, nlevels, inWires, inSizes, nin, outWires, outSizes, nout);
        auto enc = makeEncryptors(0);
        auto ev = makeEvaluators(1);
        Mat a(n, 1);
        u64 x = 0x2545F4914F6CDD1Dull;
        for (u64 k = 0; k < n; ++k) {
            x ^= x << 13, x ^= x >> 7, x ^= x << 17;
            a.v[k] = (i64)x;
        }
        Shared A = shareInt(enc, 0, a);
        auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < reps; ++r) {
            Shared res = toBinaryMatrix(ev, c, A, 64);
            if (res[0].s[0].v.size() != n) throw std::runtime_error("a2b: result size");
        }
        auto t1 = std::chrono::steady_clock::now();
        return std::chrono::duration<double>(t1 - t0).count();
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

extern "C" double orc_bench_bitinj(uint64_t rows, uint64_t bits, int reps) {
    try {
        if (!bits || bits > 64) throw std::runtime_error("bitinj: 1..64 bits");
        auto enc = makeEncryptors(0);
        auto ev = makeEvaluators(1);
        Mat a(rows, 1);
        u64 x = 0x9E3779B97F4A7C15ull;
        for (u64 k = 0; k < rows; ++k) {
            x ^= x << 13, x ^= x >> 7, x ^= x << 17;
            a.v[k] = bits < 64 ? (i64)(x & ((1ull << bits) - 1)) : (i64)x;
        }
        Shared A = shareBin(enc, 0, a);
        auto cv = converterInit(ev);
        auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < reps; ++r) {
            Shared res = bitInjection(ev, cv, A, bits, false);
            if (res[0].s[0].v.size() != rows * bits) throw std::runtime_error("bitinj: result size");
        }
        auto t1 = std::chrono::steady_clock::now();
        return std::chrono::duration<double>(t1 - t0).count();
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

// CPU baseline of the C5 sort: the oracle's batched odd-even merge sort of n
// distinct keys ((x mod 2^43) << 20 | i), three parties simulated in sequence
// on one thread. Returns seconds, -1 on error.
extern "C" double orc_bench_sort(uint32_t wires, const uint32_t* gates, uint64_t ngates, const uint32_t* levels,
                                 uint64_t nlevels, const uint32_t* inWires, const uint32_t* inSizes, uint64_t nin,
                                 const uint32_t* outWires, const uint32_t* outSizes, uint64_t nout, uint64_t n) {
    try {
        Circuit c = toCircuit(wires, gates, ngates, levels, nlevels, inWires, inSizes, nin, outWires, outSizes, nout);
        auto enc = makeEncryptors(0);
        auto ev = makeEvaluators(1);
        Mat a(n, 1);
        u64 x = 7;
        for (u64 k = 0; k < n; ++k) {
            x ^= x << 13, x ^= x >> 7, x ^= x << 17;
            a.v[k] = (i64)(((x % (1ull << 43)) << 20) | k);
        }
        Shared A = shareBin(enc, 0, a);
        auto t0 = std::chrono::steady_clock::now();
        Shared res = multiMerge(ev, c, A, std::vector<u64>(n, 1));
        auto t1 = std::chrono::steady_clock::now();
        Mat r = revealBin(res);
        for (u64 k = 1; k < n; ++k)
            if (r.v[k - 1] > r.v[k]) throw std::runtime_error("sort baseline: output not sorted");
        return std::chrono::duration<double>(t1 - t0).count();
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}
