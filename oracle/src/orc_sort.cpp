// TEST INFRASTRUCTURE ONLY -- CPU oracle. Only tests/, __graft_entry__.smoke()
// and bench.py's cpu_baseline leg may use anything under oracle/.
//
// Restatement of the merge network of aby3-Basic/Sort.cpp:327-628 (batched,
// see orc_core.h), written the reference's way: gather the round's x_mask /
// y_mask rows, compare-and-swap, write min / max back.
#include "orc_core.h"
#include <algorithm>
#include <cmath>

namespace orc {

std::vector<std::pair<u64, u64>> mergeRounds(u64 length) {
    if (!length) throw std::runtime_error("merge of an empty list");
    // Sort.cpp:361-363: t = ceil(log2(length) + 1), q = 2^(t-1), d = 1, r = 0
    size_t t = (size_t)std::ceil(std::log2((double)length) + 1);
    size_t q = (size_t)std::pow(2, t - 1);
    size_t d = 1, r = 0;
    std::vector<std::pair<u64, u64>> out;
    while (d > 0) {  // :365-398
        out.push_back({d, r});
        d = q - 1;
        q = q >> 1;
        r = 1;
    }
    return out;
}

namespace {

Shared gatherRows(const Shared& x, const std::vector<u64>& idx) {
    Shared o;
    for (int p = 0; p < 3; ++p) {
        o[p] = SMat(idx.size(), 1);
        for (int s = 0; s < 2; ++s)
            for (size_t i = 0; i < idx.size(); ++i) o[p].s[s].v[i] = x[p].s[s].v[idx[i]];
    }
    return o;
}
void scatterRows(const Shared& src, const std::vector<u64>& idx, Shared& dst) {
    for (int p = 0; p < 3; ++p)
        for (int s = 0; s < 2; ++s)
            for (size_t i = 0; i < idx.size(); ++i) dst[p].s[s].v[idx[i]] = src[p].s[s].v[i];
}
Shared sliceRows(const Shared& x, u64 off, u64 n) {
    std::vector<u64> idx(n);
    for (u64 i = 0; i < n; ++i) idx[i] = off + i;
    return gatherRows(x, idx);
}

// bool_cipher_max_min_split over the rows (x[i], y[i]), one cmp_swap
// evaluation per MAX_SENDING_SIZE rows (Sort.cpp:522-543)
void maxMinSplit(std::array<Party, 3>& ev, const Circuit& cir, const Shared& x, const Shared& y, Shared& mn,
                 Shared& mx) {
    const u64 MAX_SENDING_SIZE = 1ull << 25;
    const u64 n = x[0].rows();
    for (int p = 0; p < 3; ++p) {
        mn[p] = SMat(n, 1);
        mx[p] = SMat(n, 1);
    }
    for (u64 c = 0; c < n; c += MAX_SENDING_SIZE) {
        const u64 len = std::min(MAX_SENDING_SIZE, n - c);
        Shared xp = sliceRows(x, c, len), yp = sliceRows(y, c, len);
        auto o = evalCircuit(ev, cir, {&xp, &yp});
        for (int p = 0; p < 3; ++p)
            for (int s = 0; s < 2; ++s) {
                std::copy(o[0][p].s[s].v.begin(), o[0][p].s[s].v.end(), mn[p].s[s].v.begin() + c);
                std::copy(o[1][p].s[s].v.begin(), o[1][p].s[s].v.end(), mx[p].s[s].v.begin() + c);
            }
    }
}

}  // namespace

void mergeBatch(std::array<Party, 3>& ev, const Circuit& cir, Shared& data, const std::vector<MergeSpec>& ms) {
    const u64 M = ms.size(), N = data[0].rows();
    if (!M) return;
    std::vector<u64> len(M), base(M);
    u64 slots = 0;
    bool pad = false;
    for (u64 m = 0; m < M; ++m) {
        if (!ms[m].lenA || !ms[m].lenB || ms[m].offA + ms[m].lenA + ms[m].lenB > N)
            throw std::runtime_error("merge list out of range");
        len[m] = std::max(ms[m].lenA, ms[m].lenB);  // Sort.cpp:331
        base[m] = slots;
        slots += 2 * len[m];
        pad = pad || ms[m].lenA != ms[m].lenB;
    }
    // max(last1, last2) per merge (Sort.cpp:335-347)
    Shared maxEle;
    if (pad) {
        std::vector<u64> ia(M), ib(M);
        for (u64 m = 0; m < M; ++m) {
            ia[m] = ms[m].offA + ms[m].lenA - 1;
            ib[m] = ms[m].offA + ms[m].lenA + ms[m].lenB - 1;
        }
        Shared mn;
        maxMinSplit(ev, cir, gatherRows(data, ia), gatherRows(data, ib), mn, maxEle);
    }
    // result = padding, list 1 at even slots, list 2 at odd slots (:349-358)
    Shared res;
    for (int p = 0; p < 3; ++p) res[p] = SMat(slots, 1);
    for (u64 m = 0; m < M; ++m)
        for (int p = 0; p < 3; ++p)
            for (int s = 0; s < 2; ++s) {
                auto& out = res[p].s[s].v;
                const auto& in = data[p].s[s].v;
                for (u64 i = 0; i < 2 * len[m]; ++i) out[base[m] + i] = pad ? maxEle[p].s[s].v[m] : 0;
                for (u64 i = 0; i < ms[m].lenA; ++i) out[base[m] + 2 * i] = in[ms[m].offA + i];
                for (u64 i = 0; i < ms[m].lenB; ++i) out[base[m] + 2 * i + 1] = in[ms[m].offA + ms[m].lenA + i];
            }
    // the rounds (:365-398), all merges' round j in one evaluation
    std::vector<std::vector<std::pair<u64, u64>>> sched(M);
    size_t rounds = 0;
    for (u64 m = 0; m < M; ++m) {
        sched[m] = mergeRounds(len[m]);
        rounds = std::max(rounds, sched[m].size());
    }
    for (size_t j = 0; j < rounds; ++j) {
        std::vector<u64> xm, ym;
        for (u64 m = 0; m < M; ++m) {
            if (j >= sched[m].size()) continue;
            const u64 d = sched[m][j].first, r = sched[m][j].second;
            for (u64 i = r; i + d < 2 * len[m]; i += 2) {  // for(i = r; i < length*2 - d; i += 2)
                xm.push_back(base[m] + i);
                ym.push_back(base[m] + i + d);
            }
        }
        if (xm.empty()) continue;
        Shared mn, mx;
        maxMinSplit(ev, cir, gatherRows(res, xm), gatherRows(res, ym), mn, mx);
        scatterRows(mn, xm, res);
        scatterRows(mx, ym, res);
    }
    // res.resize(arr1_length + arr2_length) per merge (:400-404), back in place
    for (u64 m = 0; m < M; ++m)
        for (int p = 0; p < 3; ++p)
            for (int s = 0; s < 2; ++s)
                for (u64 i = 0; i < ms[m].lenA + ms[m].lenB; ++i)
                    data[p].s[s].v[ms[m].offA + i] = res[p].s[s].v[base[m] + i];
}

Shared multiMerge(std::array<Party, 3>& ev, const Circuit& cir, const Shared& flat, std::vector<u64> lens,
                  bool sequential) {
    Shared cur = flat;
    // Sort.cpp:413-437
    while (lens.size() != 1) {
        const size_t k = lens.size();
        std::vector<u64> off(k, 0);
        for (size_t i = 1; i < k; ++i) off[i] = off[i - 1] + lens[i - 1];
        if (k % 2 != 0) {
            mergeBatch(ev, cir, cur, {MergeSpec{off[k - 2], lens[k - 2], lens[k - 1]}});
            lens[k - 2] += lens[k - 1];
            lens.pop_back();
        } else {
            std::vector<MergeSpec> ms;
            std::vector<u64> next;
            for (size_t i = 0; i < k; i += 2) {
                ms.push_back(MergeSpec{off[i], lens[i], lens[i + 1]});
                next.push_back(lens[i] + lens[i + 1]);
            }
            if (sequential)
                for (const MergeSpec& m : ms) mergeBatch(ev, cir, cur, {m});
            else
                mergeBatch(ev, cir, cur, ms);
            lens = next;
        }
    }
    return cur;
}

std::vector<Shared> hdMultiMerge(std::array<Party, 3>& ev, const Circuit& cir, std::vector<std::vector<Shared>> data,
                                 bool sequential) {
    const size_t dim = data.size();
    size_t k = data[0].size();
    // one level: merges (data[i][a], data[i][a + 1]), pair-major then dimension
    auto level = [&](const std::vector<size_t>& firsts, const std::vector<size_t>& dsts) {
        Shared flat;
        for (int p = 0; p < 3; ++p) flat[p] = SMat(0, 1);
        std::vector<MergeSpec> ms;
        u64 off = 0;
        auto append = [&](const Shared& x) {
            for (int p = 0; p < 3; ++p)
                for (int s = 0; s < 2; ++s) {
                    auto& v = flat[p].s[s].v;
                    v.insert(v.end(), x[p].s[s].v.begin(), x[p].s[s].v.end());
                    flat[p].s[s].rows = v.size();
                }
        };
        for (size_t a : firsts)
            for (size_t i = 0; i < dim; ++i) {
                append(data[i][a]);
                append(data[i][a + 1]);
                ms.push_back(MergeSpec{off, data[i][a][0].rows(), data[i][a + 1][0].rows()});
                off += data[i][a][0].rows() + data[i][a + 1][0].rows();
            }
        mergeBatch(ev, cir, flat, ms);
        size_t m = 0;
        for (size_t p = 0; p < firsts.size(); ++p)
            for (size_t i = 0; i < dim; ++i, ++m) data[i][dsts[p]] = sliceRows(flat, ms[m].offA, ms[m].lenA + ms[m].lenB);
    };
    while (k != 1) {  // Sort.cpp:590-621
        if (k % 2 != 0) {
            level({k - 2}, {k - 2});
            k -= 1;
        } else {
            std::vector<size_t> firsts, dsts;
            for (size_t i = 0; i < k; i += 2) {
                firsts.push_back(i);
                dsts.push_back(i / 2);
            }
            if (sequential)
                for (size_t p = 0; p < firsts.size(); ++p) level({firsts[p]}, {dsts[p]});
            else
                level(firsts, dsts);
            k >>= 1;
        }
    }
    std::vector<Shared> out(dim);
    for (size_t i = 0; i < dim; ++i) out[i] = data[i][0];
    return out;
}

}  // namespace orc
