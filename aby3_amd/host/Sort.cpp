// aby3-Basic/Sort.cpp:327-628 on the GPU engine; see Sort.h for the batched
// semantics and the round schedule.
#include "Sort.h"
#include <algorithm>
#include <cmath>
#include "Basic.h"

namespace aby3 {

std::vector<std::pair<u64, u64>> mergeSchedule(u64 length) {
    if (!length) throw std::invalid_argument("merge of an empty list " LOCATION);
    std::vector<std::pair<u64, u64>> s;
    // Sort.cpp:361-398
    const u64 t = (u64)std::ceil(std::log2((double)length) + 1);
    u64 q = (u64)1 << (t - 1);
    u64 d = 1, r = 0;
    while (d > 0) {
        s.push_back({d, r});
        d = q - 1;
        q >>= 1;
        r = 1;
    }
    return s;
}

namespace {

// pairs (i, i + d) for i = r, r + 2, ... < slots - d
u64 pairCount(u64 slots, u64 d, u64 r) { return slots > d + r ? (slots - d - r + 1) / 2 : 0; }

aby3g_rowmap affine(u64 start, u64 step, u64 perRep, u64 repStride) {
    return aby3g_rowmap{0, start, step, perRep, repStride, nullptr};
}
aby3g_rowmap byIndex(const DeviceBuffer& idx) { return aby3g_rowmap{0, 0, 0, 1, 0, idx.as<u32>()}; }

DeviceBuffer upload32(const std::vector<u32>& v, Gpu& g) {
    DeviceBuffer b(g, std::max<size_t>(v.size() * 4, 4));
    if (!v.empty()) toDevice(b.data(), v.data(), v.size() * 4, g);
    return b;
}

// cmp_swap over `rows` pairs, one evaluation per kMaxSendingSize rows
// (Sort.cpp:522-543): circuit row p compares rows gx(p) and gy(p) of src;
// its min goes to row sx(p) of dst, its max to row sy(p) (either may be
// skipped). The gathers read src before any scatter of the same chunk writes
// dst; chunks of one round touch disjoint pairs.
void compareExchange(Sh3BinaryEvaluator& eng, const sbMatrix& src, sbMatrix& dst, const aby3g_rowmap& gx,
                     const aby3g_rowmap& gy, const aby3g_rowmap* sx, const aby3g_rowmap* sy, u64 rows,
                     Sh3Evaluator& eval, Sh3Runtime& rt) {
    BetaCircuit* cir = basicLibrary().cmp_swap(64);
    for (u64 c = 0; c < rows; c += kMaxSendingSize) {
        const u64 n = std::min(kMaxSendingSize, rows - c);
        aby3g_rowmap m[4] = {gx, gy, sx ? *sx : gx, sy ? *sy : gy};
        for (auto& x : m) x.first += c;
        eng.setCir(cir, n, eval.mShareGen);
        eng.setInputs(0, m[0], 1, m[1], src);  // both gathers in one launch
        eng.asyncEvaluate(rt.noDependencies())
            .then([&](Sh3Task&) {
                if (sx && sy)
                    eng.getOutputs(0, m[2], 1, m[3], dst);  // both scatters in one launch
                else if (sx)
                    eng.getOutput(0, dst, m[2]);
                else if (sy)
                    eng.getOutput(1, dst, m[3]);
            })
            .get();
    }
}

void concatRows(const std::vector<const sbMatrix*>& parts, sbMatrix& out, Gpu& g) {
    u64 n = 0;
    for (auto* p : parts) {
        if (p->bitCount() != 64 || p->cols() != 1) throw std::runtime_error("64-bit keys expected " LOCATION);
        n += p->rows();
    }
    out.resize(n, 64);
    for (int s = 0; s < 2; ++s) {
        u64 o = 0;
        for (auto* p : parts) {
            if (p->rows()) d2d(out.share(s) + o, p->share(s), p->rows() * 8, g);
            o += p->rows();
        }
    }
}

void sliceRows(const sbMatrix& in, u64 off, u64 n, sbMatrix& out, Gpu& g) {
    out.resize(n, 64);
    for (int s = 0; s < 2; ++s)
        if (n) d2d(out.share(s), in.share(s) + off, n * 8, g);
}

}  // namespace

std::vector<u64> mergeBatchEvalRows(const std::vector<MergeSpec>& ms) {
    std::vector<u64> rows;
    auto add = [&](u64 n) {
        for (u64 c = 0; c < n; c += kMaxSendingSize) rows.push_back(std::min(kMaxSendingSize, n - c));
    };
    bool pad = false;
    std::vector<std::vector<std::pair<u64, u64>>> sched;
    size_t rounds = 0;
    for (auto& m : ms) {
        pad = pad || m.lenA != m.lenB;
        sched.push_back(mergeSchedule(std::max(m.lenA, m.lenB)));
        rounds = std::max(rounds, sched.back().size());
    }
    if (pad) add(ms.size());
    for (size_t j = 0; j < rounds; ++j) {
        u64 n = 0;
        for (size_t m = 0; m < ms.size(); ++m)
            if (j < sched[m].size())
                n += pairCount(2 * std::max(ms[m].lenA, ms[m].lenB), sched[m][j].first, sched[m][j].second);
        if (n) add(n);
    }
    return rows;
}

std::vector<u64> multiMergeEvalRows(std::vector<u64> lens, bool sequential) {
    std::vector<u64> rows;
    while (lens.size() > 1) {
        const size_t k = lens.size();
        std::vector<u64> off(k, 0);
        for (size_t i = 1; i < k; ++i) off[i] = off[i - 1] + lens[i - 1];
        std::vector<MergeSpec> ms;
        if (k % 2) {
            ms.push_back(MergeSpec{off[k - 2], lens[k - 2], lens[k - 1]});
            lens[k - 2] += lens[k - 1];
            lens.pop_back();
        } else {
            std::vector<u64> next;
            for (size_t i = 0; i < k; i += 2) {
                ms.push_back(MergeSpec{off[i], lens[i], lens[i + 1]});
                next.push_back(lens[i] + lens[i + 1]);
            }
            lens = std::move(next);
        }
        if (sequential)  // one merge after the other: each its own evaluations
            for (const MergeSpec& m : ms)
                for (u64 r : mergeBatchEvalRows({m})) rows.push_back(r);
        else
            for (u64 r : mergeBatchEvalRows(ms)) rows.push_back(r);
    }
    return rows;
}

void mergeBatch(sbMatrix& data, const std::vector<MergeSpec>& ms, int, Sh3Evaluator& eval, Sh3Runtime& rt) {
    if (ms.empty()) return;
    if (data.bitCount() != 64) throw std::runtime_error("64-bit keys expected " LOCATION);
    Gpu& g = rt.gpu();
    const u64 N = data.rows(), M = ms.size();
    for (auto& m : ms)
        if (!m.lenA || !m.lenB || m.offA + m.lenA + m.lenB > N)
            throw std::invalid_argument("mergeBatch: empty list or list out of range " LOCATION);
    Sh3BinaryEvaluator eng;

    // Equal lengths L, merges back to back over the whole array: affine maps,
    // and round 0 (d = 1, r = 0: slot pairs (2i, 2i + 1) = (A_m[i], B_m[i]))
    // reads the lists where they lie and writes the interleaved slots.
    const u64 L = ms[0].lenA;
    bool uniform = M * 2 * L == N;
    for (u64 m = 0; m < M && uniform; ++m)
        uniform = ms[m].lenA == L && ms[m].lenB == L && ms[m].offA == m * 2 * L;
    if (uniform) {
        const auto sched = mergeSchedule(L);
        const u64 S = 2 * L;
        sbMatrix res(N, 64);
        const aby3g_rowmap mn = affine(0, 2, L, S), mx = affine(1, 2, L, S);
        compareExchange(eng, data, res, affine(0, 1, L, S), affine(L, 1, L, S), &mn, &mx, M * L, eval, rt);
        for (size_t j = 1; j < sched.size(); ++j) {
            const u64 d = sched[j].first, r = sched[j].second, cnt = pairCount(S, d, r);
            const aby3g_rowmap x = affine(r, 2, cnt, S), y = affine(r + d, 2, cnt, S);
            if (cnt) compareExchange(eng, res, res, x, y, &x, &y, M * cnt, eval, rt);
        }
        data = std::move(res);
        return;
    }

    // General shapes: explicit row lists.
    std::vector<u64> len(M), slot0(M);
    u64 slots = 0;
    bool pad = false;
    for (u64 m = 0; m < M; ++m) {
        len[m] = std::max(ms[m].lenA, ms[m].lenB);
        slot0[m] = slots;
        slots += 2 * len[m];
        pad = pad || ms[m].lenA != ms[m].lenB;
    }
    if (slots + N + M >= (1ull << 32)) throw std::runtime_error("mergeBatch: too many rows for u32 row lists");
    // padding maxima max(last_A, last_B) (Sort.cpp:335-347, :447-485) into rows N.. of src
    sbMatrix withPad;
    const sbMatrix* src = &data;
    if (pad) {
        withPad.resize(N + M, 64);
        for (int s = 0; s < 2; ++s) d2d(withPad.share(s), data.share(s), N * 8, g);
        std::vector<u32> lx(M), ly(M);
        for (u64 m = 0; m < M; ++m) {
            lx[m] = (u32)(ms[m].offA + ms[m].lenA - 1);
            ly[m] = (u32)(ms[m].offA + ms[m].lenA + ms[m].lenB - 1);
        }
        DeviceBuffer dx = upload32(lx, g), dy = upload32(ly, g);
        const aby3g_rowmap to = affine(N, 1, M, 0);
        compareExchange(eng, data, withPad, byIndex(dx), byIndex(dy), nullptr, &to, M, eval, rt);
        src = &withPad;
    }
    // interleave: list A at even slots, list B at odd slots, the rest padding
    sbMatrix res(slots, 64);
    {
        std::vector<u32> il(slots);
        for (u64 m = 0; m < M; ++m)
            for (u64 i = 0; i < len[m]; ++i) {
                il[slot0[m] + 2 * i] = (u32)(i < ms[m].lenA ? ms[m].offA + i : N + m);
                il[slot0[m] + 2 * i + 1] = (u32)(i < ms[m].lenB ? ms[m].offA + ms[m].lenA + i : N + m);
            }
        DeviceBuffer di = upload32(il, g);
        for (int s = 0; s < 2; ++s)
            GPU_CALL(aby3g_u64_gather(slots, di.as<u32>(), (const u64*)src->share(s), (u64*)res.share(s), g.stream()));
    }
    std::vector<std::vector<std::pair<u64, u64>>> sched(M);
    size_t rounds = 0;
    for (u64 m = 0; m < M; ++m) {
        sched[m] = mergeSchedule(len[m]);
        rounds = std::max(rounds, sched[m].size());
    }
    for (size_t j = 0; j < rounds; ++j) {
        std::vector<u32> ix, iy;
        for (u64 m = 0; m < M; ++m) {
            if (j >= sched[m].size()) continue;
            const u64 d = sched[m][j].first, r = sched[m][j].second, cnt = pairCount(2 * len[m], d, r);
            for (u64 k = 0; k < cnt; ++k) {
                ix.push_back((u32)(slot0[m] + r + 2 * k));
                iy.push_back((u32)(slot0[m] + r + 2 * k + d));
            }
        }
        if (ix.empty()) continue;
        DeviceBuffer dx = upload32(ix, g), dy = upload32(iy, g);
        const aby3g_rowmap x = byIndex(dx), y = byIndex(dy);
        compareExchange(eng, res, res, x, y, &x, &y, ix.size(), eval, rt);
    }
    // the first lenA + lenB slots of each merge back over its two lists
    std::vector<u32> from, to;
    for (u64 m = 0; m < M; ++m)
        for (u64 i = 0; i < ms[m].lenA + ms[m].lenB; ++i) {
            from.push_back((u32)(slot0[m] + i));
            to.push_back((u32)(ms[m].offA + i));
        }
    DeviceBuffer df = upload32(from, g), dt = upload32(to, g);
    sbMatrix packed(from.size(), 64);
    for (int s = 0; s < 2; ++s) {
        GPU_CALL(aby3g_u64_gather(from.size(), df.as<u32>(), (const u64*)res.share(s), (u64*)packed.share(s),
                                  g.stream()));
        GPU_CALL(aby3g_u64_scatter(to.size(), dt.as<u32>(), (const u64*)packed.share(s), (u64*)data.share(s),
                                   g.stream()));
    }
}

int odd_even_merge(const sbMatrix& data1, const sbMatrix& data2, sbMatrix& res, int pIdx, Sh3Evaluator& eval,
                   Sh3Runtime& runtime) {
    Gpu& g = runtime.gpu();
    sbMatrix flat;
    concatRows({&data1, &data2}, flat, g);
    mergeBatch(flat, {MergeSpec{0, data1.rows(), data2.rows()}}, pIdx, eval, runtime);
    res = std::move(flat);
    return 0;
}

int odd_even_multi_merge(const sbMatrix& flat, const std::vector<u64>& lensIn, sbMatrix& sorted, int pIdx,
                         Sh3Evaluator& eval, Sh3Runtime& runtime, MergeOrder order) {
    if (lensIn.empty()) throw std::invalid_argument("odd_even_multi_merge: no lists " LOCATION);
    u64 total = 0;
    for (u64 l : lensIn) total += l;
    if (total != flat.rows()) throw std::invalid_argument("odd_even_multi_merge: list lengths do not sum to rows");
    Gpu& g = runtime.gpu();
    sbMatrix cur;
    cur.resize(flat.rows(), 64);
    for (int s = 0; s < 2; ++s)
        if (flat.rows()) d2d(cur.share(s), flat.share(s), flat.rows() * 8, g);
    std::vector<u64> lens(lensIn);
    // Sort.cpp:413-437
    while (lens.size() != 1) {
        const size_t k = lens.size();
        std::vector<u64> off(k, 0);
        for (size_t i = 1; i < k; ++i) off[i] = off[i - 1] + lens[i - 1];
        if (k % 2) {
            mergeBatch(cur, {MergeSpec{off[k - 2], lens[k - 2], lens[k - 1]}}, pIdx, eval, runtime);
            lens[k - 2] += lens[k - 1];
            lens.pop_back();
        } else {
            std::vector<MergeSpec> ms;
            std::vector<u64> next;
            for (size_t i = 0; i < k; i += 2) {
                ms.push_back(MergeSpec{off[i], lens[i], lens[i + 1]});
                next.push_back(lens[i] + lens[i + 1]);
            }
            if (order == MergeOrder::Sequential)
                for (const MergeSpec& m : ms) mergeBatch(cur, {m}, pIdx, eval, runtime);
            else
                mergeBatch(cur, ms, pIdx, eval, runtime);
            lens = std::move(next);
        }
    }
    sorted = std::move(cur);
    return 0;
}

int odd_even_multi_merge(std::vector<sbMatrix>& data, sbMatrix& sorted, int pIdx, Sh3Evaluator& eval,
                         Sh3Runtime& runtime, MergeOrder order) {
    std::vector<const sbMatrix*> parts;
    std::vector<u64> lens;
    for (auto& d : data) {
        parts.push_back(&d);
        lens.push_back(d.rows());
    }
    sbMatrix flat;
    concatRows(parts, flat, runtime.gpu());
    return odd_even_multi_merge(flat, lens, sorted, pIdx, eval, runtime, order);
}

int odd_even_merge_sort(const sbMatrix& keys, sbMatrix& sorted, int pIdx, Sh3Evaluator& eval, Sh3Runtime& runtime) {
    if (!keys.rows()) throw std::invalid_argument("odd_even_merge_sort: no keys " LOCATION);
    return odd_even_multi_merge(keys, std::vector<u64>(keys.rows(), 1), sorted, pIdx, eval, runtime);
}

int high_dimensional_odd_even_merge(std::vector<sbMatrix>& data1, std::vector<sbMatrix>& data2,
                                    std::vector<sbMatrix>& sorted, int pIdx, Sh3Evaluator& eval, Sh3Runtime& runtime) {
    const size_t dim = data1.size();
    if (dim != data2.size()) throw std::runtime_error("The dimensions of the two data sets are not equal! " LOCATION);
    if (!dim) {
        sorted.clear();
        return 0;
    }
    Gpu& g = runtime.gpu();
    std::vector<const sbMatrix*> parts;
    std::vector<MergeSpec> ms;
    u64 off = 0;
    for (size_t i = 0; i < dim; ++i) {
        parts.push_back(&data1[i]);
        parts.push_back(&data2[i]);
        ms.push_back(MergeSpec{off, data1[i].rows(), data2[i].rows()});
        off += data1[i].rows() + data2[i].rows();
    }
    sbMatrix flat;
    concatRows(parts, flat, g);
    mergeBatch(flat, ms, pIdx, eval, runtime);
    sorted.resize(dim);
    for (size_t i = 0; i < dim; ++i) sliceRows(flat, ms[i].offA, ms[i].lenA + ms[i].lenB, sorted[i], g);
    return 0;
}

int high_dimensional_odd_even_multi_merge(std::vector<std::vector<sbMatrix>>& data, std::vector<sbMatrix>& sorted,
                                          int pIdx, Sh3Evaluator& eval, Sh3Runtime& runtime, MergeOrder order) {
    const size_t dim = data.size();
    if (!dim) {
        sorted.clear();
        return 0;
    }
    size_t k = data[0].size();
    for (auto& d : data)
        if (d.size() != k || !k) throw std::runtime_error("every dimension needs the same number of lists " LOCATION);
    Gpu& g = runtime.gpu();
    // one level: merges (data[i][a_p], data[i][a_p + 1]) for the given a_p,
    // pair-major then dimension, results into data[i][dst_p]
    auto level = [&](const std::vector<size_t>& firsts, const std::vector<size_t>& dsts) {
        std::vector<const sbMatrix*> parts;
        std::vector<MergeSpec> ms;
        u64 off = 0;
        for (size_t a : firsts)
            for (size_t i = 0; i < dim; ++i) {
                parts.push_back(&data[i][a]);
                parts.push_back(&data[i][a + 1]);
                ms.push_back(MergeSpec{off, data[i][a].rows(), data[i][a + 1].rows()});
                off += data[i][a].rows() + data[i][a + 1].rows();
            }
        sbMatrix flat;
        concatRows(parts, flat, g);
        mergeBatch(flat, ms, pIdx, eval, runtime);
        size_t m = 0;
        for (size_t p = 0; p < firsts.size(); ++p)
            for (size_t i = 0; i < dim; ++i, ++m) sliceRows(flat, ms[m].offA, ms[m].lenA + ms[m].lenB, data[i][dsts[p]], g);
    };
    // Sort.cpp:585-628
    while (k != 1) {
        if (k % 2) {
            level({k - 2}, {k - 2});
            k -= 1;
        } else {
            std::vector<size_t> firsts, dsts;
            for (size_t i = 0; i < k; i += 2) {
                firsts.push_back(i);
                dsts.push_back(i / 2);
            }
            if (order == MergeOrder::Sequential)
                for (size_t p = 0; p < firsts.size(); ++p) level({firsts[p]}, {dsts[p]});
            else
                level(firsts, dsts);
            k >>= 1;
        }
    }
    sorted.resize(dim);
    for (size_t i = 0; i < dim; ++i) sorted[i] = std::move(data[i][0]);
    return 0;
}

}  // namespace aby3
