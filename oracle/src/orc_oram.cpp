// TEST INFRASTRUCTURE ONLY -- CPU oracle. Only tests/, __graft_entry__.smoke()
// and bench.py's cpu_baseline leg may use anything under oracle/.
//
// Restatement of the square-root ORAM of aby3-Basic (SqrtOram.h:63-450 over
// the base classes of Oram/include/oram.h:90-275) and the BoolBasic helpers
// it is built from (BoolBasic.cpp:42-141, 373-515, 596-710, 732-783, 895-904),
// the three parties simulated together. Every bool_cipher_* call is a fresh
// Sh3BinaryEvaluator in the reference (setCir on the evaluator's ShareGen), so
// each is one evalCircuit here, in the reference's call order; the plain
// steps (share-wise NOT, the boolShare OR / AND with its reshare to next, the
// -1/0 expansions, back2plain's opening) are written out per party.
#include "orc_core.h"
#include <cmath>
#include <functional>
#include <memory>

namespace orc {

namespace {
using Row = std::array<i64, 2>;

// one column of 64-bit words: party p's shares of row i are v[i][p]
Shared column(u64 rows, const std::function<Row(int, u64)>& f) {
    Shared x;
    for (int p = 0; p < 3; ++p) {
        x[p] = SMat(rows, 1);
        for (u64 i = 0; i < rows; ++i) {
            const Row r = f(p, i);
            x[p].s[0].v[i] = r[0];
            x[p].s[1].v[i] = r[1];
        }
    }
    return x;
}
Shared indexColumn(const std::vector<Index3>& v) {  // vecBoolIndices::to_matrix (Basics.h:165-175)
    return column(v.size(), [&](int p, u64 i) { return Row{v[i].s[p][0], v[i].s[p][1]}; });
}
Shared repeatIndex(const Index3& x, u64 rows) {
    return column(rows, [&](int p, u64) { return Row{x.s[p][0], x.s[p][1]}; });
}
// (x == 1) ? -1 : 0 per share word (SqrtOram.h:160-169, 266-278, BoolBasic.cpp:476-483)
Shared expandBit(const Shared& x) {
    Shared y = x;
    for (auto& sm : y)
        for (auto& m : sm.s)
            for (auto& v : m.v) v = v == 1 ? -1 : 0;
    return y;
}
Index3 indexOf(const Shared& x, u64 row) {
    Index3 r;
    for (int p = 0; p < 3; ++p) r.s[p] = {x[p].s[0].v[row], x[p].s[1].v[row]};
    return r;
}
}  // namespace

Index3 Index3::pub(i64 plain) {  // boolIndex(plain, pIdx) (Basics.h:124-141)
    Index3 r;
    r.s[0] = {0, 0};
    r.s[1] = {plain, 0};
    r.s[2] = {0, plain};
    return r;
}
Bool3 Bool3::pub(bool plain) {  // boolShare(plain, pIdx) (Basics.h:39-56)
    Bool3 r;
    r.s[0] = {false, false};
    r.s[1] = {plain, false};
    r.s[2] = {false, plain};
    return r;
}
Bool3 Bool3::initFalse() {  // bool_init_false(boolShare) (BoolBasic.cpp:692-710)
    Bool3 r;
    r.s[0] = {true, false};
    r.s[1] = {true, true};
    r.s[2] = {false, true};
    return r;
}

// ---------------------------------------------------------------------------
// BoolBasic helpers
// ---------------------------------------------------------------------------
Shared OramOps::eq(const Shared& A, const Shared& B) {  // BoolBasic.cpp:42-62 (int_eq)
    return evalCircuit(*ev, cir->eq64, {&A, &B})[0];
}
Shared OramOps::eqPlain(const Shared& A, const std::vector<i64>& b) {  // :64-100
    Shared B = column(A[0].rows(), [&](int p, u64 i) {
        return p == 1 ? Row{b[i], 0} : p == 2 ? Row{0, b[i]} : Row{0, 0};
    });
    return eq(A, B);
}
Shared OramOps::and64(const Shared& A, const Shared& B) {  // :187-209 (int_int_bitwiseAnd)
    return evalCircuit(*ev, cir->and64, {&A, &B})[0];
}
Shared OramOps::or1(const Shared& A, const Shared& B) {  // :102-122 (int_int_bitwiseOr, 1 bit here)
    return evalCircuit(*ev, cir->or1, {&A, &B})[0];
}
Bool3 OramOps::orBool(const Bool3& a, const Bool3& b) {  // :124-141
    // each party's local AND share, XORed with its share-0 inputs, sent to next
    std::array<bool, 3> sh;
    for (int p = 0; p < 3; ++p) {
        const bool c = (a.s[p][0] && b.s[p][0]) ^ (a.s[p][0] && b.s[p][1]) ^ (a.s[p][1] && b.s[p][0]);
        sh[p] = c ^ a.s[p][0] ^ b.s[p][0];
    }
    Bool3 r;
    for (int p = 0; p < 3; ++p) r.s[p] = {sh[p], sh[(p + 2) % 3]};
    return r;
}
Bool3 OramOps::notBool(const Bool3& a) {  // :373-391
    Bool3 r = a;
    r.s[1][0] = !a.s[1][0];
    r.s[2][1] = !a.s[2][1];
    return r;
}
Shared OramOps::dotRows(const Shared& A, const Shared& B) {  // :393-423
    const Shared m = and64(A, B);
    return column(1, [&](int p, u64) {
        Row r{0, 0};
        for (u64 i = 0; i < m[p].rows(); ++i) {
            r[0] ^= m[p].s[0].v[i];
            r[1] ^= m[p].s[1].v[i];
        }
        return r;
    });
}
Shared OramOps::dotUnits(const std::vector<Shared>& A, Shared B, bool bOneBit) {  // :463-515
    const u64 n = A.size();
    if (n != B[0].rows()) throw std::runtime_error("dotUnits: sizes");
    const u64 block = A[0][0].size();
    if (bOneBit) B = expandBit(B);  // sharedB.bitCount() == 1
    Shared eA, eB;
    for (int p = 0; p < 3; ++p) {
        eA[p] = SMat(n * block, 1);
        eB[p] = SMat(n * block, 1);
        for (u64 i = 0; i < n; ++i)
            for (u64 j = 0; j < block; ++j)
                for (int s = 0; s < 2; ++s) {
                    eA[p].s[s].v[i * block + j] = A[i][p].s[s].v[j];
                    eB[p].s[s].v[i * block + j] = B[p].s[s].v[i];
                }
    }
    const Shared m = and64(eA, eB);
    Shared r;
    for (int p = 0; p < 3; ++p) {
        r[p] = SMat(block, 1);
        for (u64 j = 0; j < block; ++j)
            for (int s = 0; s < 2; ++s) {
                i64 v = m[p].s[s].v[j];
                for (u64 i = 1; i < n; ++i) v ^= m[p].s[s].v[i * block + j];
                r[p].s[s].v[j] = v;
            }
    }
    return r;
}
Shared OramOps::selector(const Bool3& flag, const Shared& t, const Shared& f) {  // :425-461
    const Bool3 nf = notBool(flag);
    const u64 n = t[0].size();
    auto fill = [&](const Bool3& b) {
        return column(n, [&](int p, u64) { return Row{b.s[p][0] ? -1 : 0, b.s[p][1] ? -1 : 0}; });
    };
    const Shared a = and64(fill(flag), t);
    const Shared b = and64(fill(nf), f);
    Shared r = a;
    for (int p = 0; p < 3; ++p)
        for (int s = 0; s < 2; ++s)
            for (u64 i = 0; i < n; ++i) r[p].s[s].v[i] = a[p].s[s].v[i] ^ b[p].s[s].v[i];
    return r;
}
Shared OramOps::firstZeroMask(const std::vector<Bool3>& A) {  // :596-640
    const u64 len = A.size();
    const u64 rounds = (u64)std::floor(std::log2((double)len));
    // not(A) rotated right by one, entry 0 = (0, 0) (vecBoolShares::to_matrix)
    Shared m = column(len, [&](int p, u64 i) {
        if (i == 0) return Row{0, 0};
        const Bool3 na = notBool(A[i - 1]);
        return Row{na.s[p][0], na.s[p][1]};
    });
    for (u64 r = 0; r < rounds; ++r) {
        const u64 stride = 1ull << r, k = len - stride;
        const Shared x = column(k, [&](int p, u64 j) { return Row{m[p].s[0].v[j + stride], m[p].s[1].v[j + stride]}; });
        const Shared y = column(k, [&](int p, u64 j) { return Row{m[p].s[0].v[j], m[p].s[1].v[j]}; });
        const Shared o = or1(x, y);
        for (int p = 0; p < 3; ++p)
            for (int s = 0; s < 2; ++s)
                for (u64 j = stride; j < len; ++j) m[p].s[s].v[j] = o[p].s[s].v[j - stride];
    }
    return column(len, [&](int p, u64 i) {
        if (i + 1 < len) return Row{m[p].s[0].v[i] ^ m[p].s[0].v[i + 1], m[p].s[1].v[i] ^ m[p].s[1].v[i + 1]};
        return Row{m[p].s[0].v[i] ^ 1, m[p].s[1].v[i] ^ 1};
    });
}
i64 OramOps::back2plain(const Index3& x) {  // :895-904: send share 0 to prev, receive next's
    i64 out = 0;
    for (int p = 0; p < 3; ++p) {
        const i64 v = x.s[(p + 1) % 3][0] ^ x.s[p][1] ^ x.s[p][0];
        if (p == 0)
            out = v;
        else if (v != out)
            throw std::runtime_error("back2plain: parties disagree (inconsistent shares)");
    }
    return out;
}

// ---------------------------------------------------------------------------
// ABY3PosMap (SqrtOram.h:63-369; PosMap, oram.h:90-119)
// ---------------------------------------------------------------------------
namespace {
// pack_to_single_matrix (SqrtOram.h:22-35): [logical, packed 0 .. pack-1]
std::vector<i64> packUnit(const PackedIndex3& q, int p, int s) {
    std::vector<i64> u{q.logical.s[p][s]};
    for (auto& x : q.packed) u.push_back(x.s[p][s]);
    return u;
}
}  // namespace

PosMap3::PosMap3(std::array<Party, 3>& enc_, OramOps& ops_, u64 n_, u64 pack_, u64 S_,
                 const std::vector<Index3>& perm)
    : n(n_), pack(pack_), S(S_), enc(&enc_), ops(&ops_) {
    if (!pack || (pack & (pack - 1))) throw std::runtime_error("pack must be a power of 2");  // :83-85
    map_len = n / pack;
    linear = map_len < S;  // oram.h:106-111
    if (linear) {          // SqrtOram.h:87-91
        usage_map.assign(n, Bool3::initFalse());
        permutation = perm;
        return;
    }
    // 1. the packed map (:94-104)
    for (u64 i = 0; i < map_len; ++i) {
        PackedIndex3 q;
        q.logical = Index3::pub((i64)i);
        q.packed.assign(perm.begin() + i * pack, perm.begin() + (i + 1) * pack);
        packed_index.push_back(q);
    }
    // 2. shuffle it, keeping the shares of the permutation (:106-120)
    Shared T;
    for (int p = 0; p < 3; ++p) {
        T[p] = SMat(map_len, pack + 1);
        for (u64 i = 0; i < map_len; ++i)
            for (int s = 0; s < 2; ++s) {
                const std::vector<i64> u = packUnit(packed_index[i], p, s);
                std::copy(u.begin(), u.end(), T[p].s[s].v.begin() + i * (pack + 1));
            }
    }
    Shared Pi;
    const Shared U = shuffleWithPermutation(*enc, T, Pi);
    for (u64 i = 0; i < map_len; ++i)  // unpack_from_single_matrix (:37-49)
        for (int p = 0; p < 3; ++p)
            for (int s = 0; s < 2; ++s) {
                packed_index[i].logical.s[p][s] = U[p].s[s].v[i * (pack + 1)];
                for (u64 j = 0; j < pack; ++j) packed_index[i].packed[j].s[p][s] = U[p].s[s].v[i * (pack + 1) + 1 + j];
            }
    // 3. the sub-map (:122-129)
    std::vector<Index3> sub(map_len);
    for (u64 i = 0; i < map_len; ++i) sub[i] = indexOf(Pi, i);
    subPosMap = std::make_unique<PosMap3>(*enc, *ops, map_len, pack, S, sub);
}

Shared PosMap3::linearRam(const std::vector<Shared>& data, const Index3& index) {  // :345-368
    std::vector<i64> range(data.size());
    for (u64 i = 0; i < data.size(); ++i) range[i] = (i64)i;
    const Shared s1 = ops->eqPlain(repeatIndex(index, data.size()), range);
    return ops->dotUnits(data, s1, true);  // s1: int_eq's 1-bit output
}

i64 PosMap3::access(const Index3& index, const Bool3& fake) {  // :133-343
    Index3 physical;
    if (linear) {
        std::vector<i64> range(n);
        for (u64 i = 0; i < n; ++i) range[i] = (i64)i;
        const Shared s1 = ops->eqPlain(repeatIndex(index, n), range);  // :137-149
        const Shared s2 = ops->firstZeroMask(usage_map);                // :151-154
        const Shared s1m = expandBit(s1), s2m = expandBit(s2);          // :156-169
        const Shared perm = indexColumn(permutation);                   // :171-172
        const Shared r1 = ops->dotRows(perm, s1m);                      // :174-182
        const Shared r2 = ops->dotRows(perm, s2m);
        const Shared r = ops->selector(fake, r2, r1);  // :184-189
        physical = indexOf(r, 0);
        // usage_map = s1 OR usage_map, 1 bit (:191-203)
        const Shared used = column(n, [&](int p, u64 i) { return Row{usage_map[i].s[p][0], usage_map[i].s[p][1]}; });
        const Shared o = ops->or1(s1m, used);
        for (u64 i = 0; i < n; ++i)
            for (int p = 0; p < 3; ++p) usage_map[i].s[p] = {(o[p].s[0].v[i] & 1) != 0, (o[p].s[1].v[i] & 1) != 0};
    } else {
        // h = index >> log2(pack), l = index & (pack - 1), share-wise (:206-207,
        // BoolBasic.cpp:732-783)
        const u64 k = (u64)std::log2((double)pack);
        const i64 mask = (i64)((1 << k) - 1);
        Index3 h, l;
        for (int p = 0; p < 3; ++p)
            for (int s = 0; s < 2; ++s) {
                h.s[p][s] = index.s[p][s] >> k;
                l.s[p][s] = index.s[p][s] & mask;
            }
        Bool3 found = fake;                             // :209-210
        Shared inStash = indexColumn({Index3::pub(-1)});  // :211-212
        if (t > 0) {
            // 1. is h in the stash? (:214-244)
            std::vector<Index3> si(t);
            for (u64 i = 0; i < t; ++i) si[i] = stash[i].logical;
            const Shared hit = ops->eq(repeatIndex(h, t), indexColumn(si));
            Bool3 tmp;
            for (int p = 0; p < 3; ++p)
                for (int s = 0; s < 2; ++s) {
                    bool b = hit[p].s[s].v[0] & 1;
                    for (u64 i = 1; i < t; ++i) b ^= (hit[p].s[s].v[i] & 1) != 0;
                    tmp.s[p][s] = b;
                }
            found = ops->orBool(found, tmp);
            // 2. its l-th packed index (:246-299)
            std::vector<i64> range(pack);
            for (u64 i = 0; i < pack; ++i) range[i] = (i64)i;
            const Shared per = ops->eqPlain(repeatIndex(l, pack), range);
            const u64 tp = t * pack;
            const Shared eh = column(tp, [&](int p, u64 k2) {
                const u64 i = k2 / pack;
                return Row{hit[p].s[0].v[i] == 1 ? -1 : 0, hit[p].s[1].v[i] == 1 ? -1 : 0};
            });
            const Shared el = column(tp, [&](int p, u64 k2) {
                const u64 j = k2 % pack;
                return Row{per[p].s[0].v[j] == 1 ? -1 : 0, per[p].s[1].v[j] == 1 ? -1 : 0};
            });
            const Shared sx = column(tp, [&](int p, u64 k2) {
                const Index3& x = stash[k2 / pack].packed[k2 % pack];
                return Row{x.s[p][0], x.s[p][1]};
            });
            const Shared target = ops->and64(eh, el);
            inStash = ops->dotRows(target, sx);
        }
        // 3. the packed entry's position from the sub-map (:302-303)
        const i64 next = subPosMap->access(h, found);
        if (next < 0 || (u64)next >= packed_index.size()) throw std::runtime_error("posMap: sub-map index out of range");
        // 4. stash hit -> the stashed index, else (or fake) the fetched entry's (:305-337)
        Bool3 mainFlag = ops->notBool(found);
        mainFlag = ops->orBool(mainFlag, fake);
        stash.push_back(packed_index[(u64)next]);
        ++t;
        std::vector<Shared> elems;
        for (u64 i = 0; i < pack; ++i) elems.push_back(indexColumn({packed_index[(u64)next].packed[i]}));
        const Shared fetched = linearRam(elems, l);
        const Shared r = ops->selector(mainFlag, fetched, inStash);
        physical = indexOf(r, 0);
    }
    last_physical = physical;
    return ops->back2plain(physical);  // :339-342
}

// ---------------------------------------------------------------------------
// ABY3SqrtOram (SqrtOram.h:371-450; SqrtOram, oram.h:203-275)
// ---------------------------------------------------------------------------
SqrtOram3::SqrtOram3(std::array<Party, 3>& enc_, OramOps& ops_, u64 n_, u64 S_, u64 pack_)
    : n(n_), S(S_), pack(pack_), enc(&enc_), ops(&ops_) {}
// (the reference clamps its constructor argument S, not the member, :387-388)

void SqrtOram3::initiate(const std::vector<Shared>& data) {  // :391-403
    if (data.size() != n) throw std::runtime_error("SqrtOram3::initiate: data size");
    const u64 unit = data[0][0].size();
    Shared T;
    for (int p = 0; p < 3; ++p) {
        T[p] = SMat(n, unit);
        for (u64 i = 0; i < n; ++i)
            for (int s = 0; s < 2; ++s)
                std::copy(data[i][p].s[s].v.begin(), data[i][p].s[s].v.end(), T[p].s[s].v.begin() + i * unit);
    }
    Shared Pi;
    const Shared U = shuffleWithPermutation(*enc, T, Pi);
    shuffle_mem.assign(n, Shared{});
    for (u64 i = 0; i < n; ++i)
        for (int p = 0; p < 3; ++p) {
            shuffle_mem[i][p] = SMat(data[i][p].rows(), data[i][p].cols());
            for (int s = 0; s < 2; ++s)
                std::copy(U[p].s[s].v.begin() + i * unit, U[p].s[s].v.begin() + (i + 1) * unit,
                          shuffle_mem[i][p].s[s].v.begin());
        }
    std::vector<Index3> perm(n);
    for (u64 i = 0; i < n; ++i) perm[i] = indexOf(Pi, i);
    posMap = std::make_unique<PosMap3>(*enc, *ops, n, pack, S, perm);
}

Shared SqrtOram3::access(const Index3& index) {  // :405-450
    // the base class's t is never advanced by the derived access (its own stash
    // vector grows, t stays 0), so the stash branches never run and found is
    // boolShare(false, pIdx) on every access
    const Bool3 found = Bool3::pub(false);
    const i64 phy = posMap->access(index, found);
    if (phy < 0 || (u64)phy >= n) throw std::runtime_error("sqrt-ORAM: physical index out of range");
    return shuffle_mem[(u64)phy];
}

// party p's view of the state, in the order tests/cpp/test_oram.cpp dumps the
// product's: per level [linear, t, last physical, usage map, permutation,
// packed map (logical, packed), stash (logical, packed)], then the sub-map
std::vector<i64> PosMap3::dump(int p) const {
    std::vector<i64> d{(i64)linear, (i64)t, last_physical.s[p][0], last_physical.s[p][1]};
    for (auto& u : usage_map) d.insert(d.end(), {(i64)u.s[p][0], (i64)u.s[p][1]});
    for (auto& x : permutation) d.insert(d.end(), {x.s[p][0], x.s[p][1]});
    for (auto* v : {&packed_index, &stash})
        for (auto& q : *v) {
            d.insert(d.end(), {q.logical.s[p][0], q.logical.s[p][1]});
            for (auto& x : q.packed) d.insert(d.end(), {x.s[p][0], x.s[p][1]});
        }
    if (subPosMap) {
        const std::vector<i64> s = subPosMap->dump(p);
        d.insert(d.end(), s.begin(), s.end());
    }
    return d;
}

}  // namespace orc
