// The aby3-ML engine wrapper (aby3-ML/aby3ML.h:103-139) and one iteration of
// SGD_Logistic (aby3-ML/Regression.h:218-295) on device shares.
#pragma once
#include "Sh3Encryptor.h"
#include "Sh3Evaluator.h"
#include "Sh3Piecewise.h"
#include <algorithm>
#include <vector>

namespace aby3 {

class aby3ML {
public:
    aby3ML(Sh3Runtime& rt, Sh3Encryptor& enc, Sh3Evaluator& eval, u64 D) : mRt(rt), mEnc(enc), mEval(eval), mD(D) {}

    // mul: asyncMul(left, right, dest) with shift D (aby3ML.h:103-108), matrix product
    void mul(const si64Matrix& left, const si64Matrix& right, si64Matrix& dest);
    // mulTruncate: shift D + shift (aby3ML.h:110-116)
    void mulTruncate(const si64Matrix& left, const si64Matrix& right, si64Matrix& dest, u64 shift);
    // logisticFunc: piecewise sigmoid, thresholds -0.5 / 0.5, f = 0 | 0.5 + x | 1 (aby3ML.h:121-139)
    void logisticFunc(const si64Matrix& Y, si64Matrix& out);
    // the sigmoid's piecewise description (set up on first use)
    Sh3Piecewise& logistic();

    Sh3Runtime& mRt;
    Sh3Encryptor& mEnc;
    Sh3Evaluator& mEval;
    u64 mD;
    Sh3Piecewise mLogistic;
};

struct FusedLr;
struct SgdState {
    si64Matrix XX, YY, XXt, xw, fxw, err, update;
    DeviceBuffer idx;
    // The fused iteration (aby3g_lr_iteration): one launch per party and
    // iteration when the three parties share a device and process (their ring
    // allows kernel hand-offs); set up by the first step, which all three
    // parties take together.
    std::shared_ptr<FusedLr> fused;
    bool fusedChecked = false;
    bool fusedSysScope = false;  // the fused iteration's messages are system-scope (parties on other GPUs)
    u64* phaseTicks = nullptr;  // optional device [ABY3G_LR_PHASE_SLOTS]: the fused launch's phase stamps (profiling)
    const u32* nextBatch = nullptr;  // optional: the next iteration's batch (its rows prefetched into L2)
};

// One SGD_Logistic iteration on the batch of B row indices at device pointer
// `batchIdx` (e.g. a slice of a device-resident permutation, so no host
// upload or stream sync sits in the iteration) of (X, Y):
//   XX, YY = extractBatch; xw = mul(XX, w); fxw = logistic(xw);
//   err = fxw - YY; update = mulTruncate(XX^T, err, aB); w = w - update
// (Regression.h:252-287).
void sgdLogisticStep(aby3ML& ml, const si64Matrix& X, const si64Matrix& Y, si64Matrix& w,
                     const u32* batchIdx, u64 B, u64 aB, SgdState& st);
// Host-index convenience form: uploads the indices (and waits for the upload).
void sgdLogisticStep(aby3ML& ml, const si64Matrix& X, const si64Matrix& Y, si64Matrix& w,
                     const std::vector<u32>& batchIdx, u64 aB, SgdState& st);

// ---- the C4 driver around the iteration (host side) -----------------------

// oc::PRNG(seed) on the host: the AES-CTR byte stream under `seed`, consumed
// contiguously, refilled 256 blocks at a time (cryptoTools PRNG.cpp) through
// aby3g_aes_ctr_host.
class HostPrng {
public:
    explicit HostPrng(block seed) : mSeed(seed) {}
    void get(void* dst, u64 nbytes);
    template <class T>
    T get() {
        T v;
        get(&v, sizeof(T));
        return v;
    }

private:
    block mSeed;
    u64 mOff = 0;          // bytes consumed
    u64 mBufBlock = ~0ull;  // first block held in mBuf
    std::vector<u8> mBuf;
};

// main-logistic.cpp:82-92: model(i) = PRNG(toBlock(1)).get<int>() % 10 for
// i < min(dim, 10); the reference leaves the rest uninitialized (0 here).
std::vector<double> logisticModel(u64 dim);
// LogisticModelGen::sample (LinearModelGen.cpp:49-93) with setModel's
// defaults noise = sd = 1 (LinearModelGen.h:36): libstdc++
// default_random_engine(234345) and normal_distribution(1, 1), row-major
// feature draws then one noise draw per row, Y = [X model + noise > 0];
// stored as fixed point D (fp<i64, D> = i64(v * 2^D), Sh3FixedPoint.h:94-97).
void logisticModelGen(const std::vector<double>& model, u64 n, u64 D, i64Matrix& X, i64Matrix& Y);
// getSubset (Regression.h:24-40): mini-batches without replacement from the
// pool 0..n-1, reshuffled with std::random_shuffle (for i = 1..n-1: swap with
// j = r(i + 1)) when exhausted, r(m) = PRNG(toBlock(234543234)).get<u64>() % m
// (checked against libstdc++'s std::random_shuffle on the same stream by
// tests/cpp/test_random_shuffle.cpp; the functor's get<u64>() % m is
// cryptoTools' PRNG::operator()(R), not vendored in the reference).
class BatchSampler {
public:
    explicit BatchSampler(u64 n);
    void next(std::vector<u64>& dest);

private:
    std::vector<u64> mPool;
    u64 mIter;
    HostPrng mPrng;
};

// getSubset's pool shuffle (std::random_shuffle(pool, prng), Regression.h:36):
// for i = 1..n-1 swap pool[i] with pool[prng.get<u64>() % (i + 1)].
template <class T>
void randomShuffle(T* pool, u64 n, HostPrng& prng) {
    for (u64 i = 1; i < n; ++i) {
        const u64 j = prng.get<u64>() % (i + 1);
        if (i != j) std::swap(pool[i], pool[j]);
    }
}

// getSubset (Regression.h:24-40) for iterations that run on the device: the
// same mini-batches as BatchSampler, the pool resident in HBM. next() returns
// the next B row indices as a device pointer, usable by work enqueued on the
// party's stream before the following call: a slice of the device pool when
// the batch lies inside one pool, else (a batch across a reshuffle) the batch
// assembled on the host and uploaded into a small slot. The reshuffle for the
// next epoch -- std::random_shuffle of the current pool, the PRNG advanced
// exactly as the reference advances it -- runs on a host thread during the
// current epoch and is uploaded asynchronously when the pool runs out, so no
// iteration waits for it or synchronises the stream.
class DeviceBatchSampler {
public:
    DeviceBatchSampler(Gpu& g, u64 n, u64 B);
    ~DeviceBatchSampler();
    DeviceBatchSampler(const DeviceBatchSampler&) = delete;
    DeviceBatchSampler& operator=(const DeviceBatchSampler&) = delete;
    const u32* next();
    u64 reshuffles() const;  // pools started so far (the first getSubset reshuffles at once)

private:
    struct Impl;
    std::unique_ptr<Impl> mImpl;
};

// RegressionParam / SGD_Logistic (Regression.h:15-20, 216-295): the whole
// training loop on device shares -- getSubset, extractBatch, xw = XX w,
// logistic, err, w -= XX^T err >> (D + aB) with aB = log2(B / rate) -- each
// iteration one sgdLogisticStep on a DeviceBatchSampler batch.
struct RegressionParam {
    u64 mIterations = 0;
    u64 mBatchSize = 0;
    double mLearningRate = 0;
};
void SGD_Logistic(RegressionParam& params, aby3ML& engine, const si64Matrix& X, const si64Matrix& Y, si64Matrix& w);
// aby3ML::init (aby3ML.cpp:4-17): party i's seed toBlock(i); PRNG(seed)'s
// first block is its Sh3Encryptor seed, the second its Sh3Evaluator seed,
// each exchanged with the neighbours (Sh3ShareGen.h:25-31): returns the
// (prevSeed, nextSeed) pairs {enc, eval} party pIdx initialises with.
struct MlSeeds {
    block encPrev, encNext, evalPrev, evalNext;
};
MlSeeds mlSeeds(int pIdx);

}  // namespace aby3
