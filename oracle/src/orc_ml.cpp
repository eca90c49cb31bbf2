// TEST INFRASTRUCTURE ONLY -- CPU oracle. Only tests/, __graft_entry__.smoke()
// and bench.py's cpu_baseline leg may use anything under oracle/.
//
// Restatement of aby3-ML's logistic-regression driver: the synthetic data
// (LinearModelGen.cpp:49-93, main-logistic.cpp:82-100), the mini-batch
// sampler (Regression.h:24-58), aby3ML::init's seeds (aby3ML.cpp:4-17) and
// one SGD_Logistic iteration (Regression.h:249-293).
#include "orc_core.h"
#include <algorithm>
#include <random>
#include <cmath>
#include <limits>

namespace orc {

std::vector<double> logisticModel(u64 dim) {
    Stream prng;
    Block seed = toBlock(1);
    prng.init((const u8*)&seed);
    std::vector<double> model(dim, 0.0);
    for (u64 i = 0; i < std::min<u64>(dim, 10); ++i) {
        int v;
        prng.get(&v, sizeof(v));
        model[i] = v % 10;
    }
    return model;
}

void logisticModelGen(const std::vector<double>& model, u64 n, u64 D, Mat& X, Mat& Y) {
    const u64 dim = model.size();
    std::default_random_engine generator(234345);
    std::normal_distribution<double> distribution(1.0, 1.0);
    X = Mat(n, dim);
    Y = Mat(n, 1);
    std::vector<double> row(dim);
    for (u64 i = 0; i < n; ++i) {
        for (u64 j = 0; j < dim; ++j) row[j] = distribution(generator);
        const double noise = distribution(generator);
        double y = 0;
        for (u64 j = 0; j < dim; ++j) y += row[j] * model[j];
        y += noise;
        for (u64 j = 0; j < dim; ++j) X.v[i * dim + j] = (i64)(row[j] * (double)(1ull << D));
        Y.v[i] = (i64)((y > 0 ? 1.0 : 0.0) * (double)(1ull << D));
    }
}

// How far every label of logisticModelGen is from flipping under another
// summation order of X * mModel (the reference's Eigen GEMV,
// LinearModelGen.cpp:75, sums in its own blocked / FMA order; this
// restatement sums left to right). Any order's sum of the dim products lies
// within E = gamma_dim * sum_j |x_j m_j| of the exact one (gamma_n = n u /
// (1 - n u), u = 2^-53), so two orders can disagree on the sign of
// sum + noise only where |sum + noise| <= 2E (the final add rounds to
// nearest and keeps the sign). Returns min over rows of |sum + noise| / 2E
// (infinity when no row has a non-zero product): > 1 means the labels are
// the same under every summation order.
double logisticLabelMargin(const std::vector<double>& model, u64 n) {
    const u64 dim = model.size();
    std::default_random_engine generator(234345);
    std::normal_distribution<double> distribution(1.0, 1.0);
    const double u = std::ldexp(1.0, -53), gamma = dim * u / (1 - dim * u);
    double worst = std::numeric_limits<double>::infinity();
    std::vector<double> row(dim);
    for (u64 i = 0; i < n; ++i) {
        for (u64 j = 0; j < dim; ++j) row[j] = distribution(generator);
        const double noise = distribution(generator);
        double y = 0, a = 0;
        for (u64 j = 0; j < dim; ++j) {
            y += row[j] * model[j];
            a += std::fabs(row[j] * model[j]);
        }
        // E itself is computed in floating point: inflate it by 1 %
        const double E = 1.01 * gamma * a;
        if (E > 0) worst = std::min(worst, std::fabs(y + noise) / (2 * E));
    }
    return worst;
}

BatchSampler::BatchSampler(u64 n) : pool(n), iter(n) {
    for (u64 i = 0; i < n; ++i) pool[i] = i;
    Block seed = toBlock(234543234);
    prng.init((const u8*)&seed);
}

void BatchSampler::next(std::vector<u64>& dest) {
    u64 d = 0;
    while (d != dest.size()) {
        const u64 step = std::min<u64>(pool.size() - iter, dest.size() - d);
        std::copy(pool.begin() + iter, pool.begin() + iter + step, dest.begin() + d);
        iter += step;
        d += step;
        if (iter == pool.size()) {
            // std::random_shuffle(pool.begin(), pool.end(), prng)
            for (u64 i = 1; i < pool.size(); ++i) {
                u64 r;
                prng.get(&r, sizeof(r));
                const u64 j = r % (i + 1);
                if (i != j) std::swap(pool[i], pool[j]);
            }
            iter = 0;
        }
    }
}

void mlParties(std::array<Party, 3>& enc, std::array<Party, 3>& ev) {
    Block es[3], vs[3];
    for (u64 i = 0; i < 3; ++i) {
        Stream prng;
        Block seed = toBlock(i);
        prng.init((const u8*)&seed);
        es[i] = prng.getBlock();
        vs[i] = prng.getBlock();
    }
    for (int i = 0; i < 3; ++i) {
        enc[i].initEncryptor(i, es[(i + 2) % 3], es[i]);
        ev[i].initEvaluator(i, vs[(i + 2) % 3], vs[i]);
    }
}

void sgdLogisticIteration(std::array<Party, 3>& ev, const Circuit& pwHelper, const Shared& sX, const Shared& sY,
                          Shared& sW, const std::vector<u64>& batch, u64 D, u64 aB) {
    Piecewise pw;  // aby3ML.h:121-139
    pw.thresholds = {Coef{false, 0, -0.5}, Coef{false, 0, 0.5}};
    pw.coefs = {{}, {Coef{false, 0, 0.5}, Coef{true, 1, 0}}, {Coef{true, 1, 0}}};
    const u64 B = batch.size(), d = sX[0].cols();
    Shared XX, YY, XXt;
    for (int p = 0; p < 3; ++p) {
        XX[p] = SMat(B, d);
        YY[p] = SMat(B, 1);
        XXt[p] = SMat(d, B);
        for (int s = 0; s < 2; ++s)
            for (u64 i = 0; i < B; ++i) {  // extractBatch (Regression.h:42-58)
                const u64 r = batch[i];
                for (u64 j = 0; j < d; ++j) {
                    XX[p].s[s].v[i * d + j] = sX[p].s[s].v[r * d + j];
                    XXt[p].s[s].v[j * B + i] = sX[p].s[s].v[r * d + j];
                }
                YY[p].s[s].v[i] = sY[p].s[s].v[r];
            }
    }
    Shared xw = mulTrunc(ev, MUL_GEMM, XX, sW, D);
    Shared f = piecewiseEval(ev, pw, pwHelper, xw, D);
    for (int p = 0; p < 3; ++p)  // error = fxw - YY
        for (int s = 0; s < 2; ++s)
            for (u64 i = 0; i < B; ++i) f[p].s[s].v[i] = (i64)((u64)f[p].s[s].v[i] - (u64)YY[p].s[s].v[i]);
    Shared upd = mulTrunc(ev, MUL_GEMM, XXt, f, D + aB);
    for (int p = 0; p < 3; ++p)  // w = w - update
        for (int s = 0; s < 2; ++s)
            for (u64 j = 0; j < d; ++j) sW[p].s[s].v[j] = (i64)((u64)sW[p].s[s].v[j] - (u64)upd[p].s[s].v[j]);
}

}  // namespace orc
