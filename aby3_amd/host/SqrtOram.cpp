#include "SqrtOram.h"
#include <cmath>

namespace aby3 {

boolShare::boolShare(bool plain, int pIdx) {
    bshares[0] = pIdx == 1 ? plain : false;
    bshares[1] = pIdx == 2 ? plain : false;
    if (pIdx < 0 || pIdx > 2) throw std::runtime_error("boolShare: invalid pIdx");
}

boolIndex::boolIndex(i64 plain, int pIdx) {
    indexShares[0] = pIdx == 1 ? plain : 0;
    indexShares[1] = pIdx == 2 ? plain : 0;
    if (pIdx < 0 || pIdx > 2) throw std::runtime_error("boolIndex: invalid pIdx");
}

namespace {
// a device sbMatrix from host share words (the reference fills mShares(i, 0))
sbMatrix mat(u64 rows, u64 bits, const std::vector<i64>& s0, const std::vector<i64>& s1) {
    sbMatrix m(rows, bits);
    if (rows) {
        m.shareFromHost(0, s0.data());
        m.shareFromHost(1, s1.data());
    }
    return m;
}
sbMatrix indexColumn(const std::vector<boolIndex>& v) {  // vecBoolIndices::to_matrix
    std::vector<i64> a(v.size()), b(v.size());
    for (size_t i = 0; i < v.size(); ++i) {
        a[i] = v[i].indexShares[0];
        b[i] = v[i].indexShares[1];
    }
    return mat(v.size(), BITSIZE, a, b);
}
sbMatrix repeatIndex(const boolIndex& x, u64 rows) {
    return mat(rows, BITSIZE, std::vector<i64>(rows, x.indexShares[0]), std::vector<i64>(rows, x.indexShares[1]));
}
// share words (i, 0) == 1 ? -1 : 0 (the 1-bit results expanded to masks)
std::vector<i64> expandBit(const std::vector<i64>& v) {
    std::vector<i64> o(v.size());
    for (size_t i = 0; i < v.size(); ++i) o[i] = v[i] == 1 ? -1 : 0;
    return o;
}
i64Matrix range(u64 n) {
    i64Matrix r(n, 1);
    for (u64 i = 0; i < n; ++i) r(i, 0) = (i64)i;
    return r;
}
}  // namespace

void bool_cipher_eq(int pIdx, const sbMatrix& A, const i64Matrix& plainB, sbMatrix& res, Sh3Evaluator& eval,
                    Sh3Runtime& runtime) {
    const u64 n = A.i64Size();
    if (plainB.mData.size() < n) throw std::invalid_argument("bool_cipher_eq: plainB too short");
    std::vector<i64> b0(n, 0), b1(n, 0);
    for (u64 i = 0; i < n; ++i) {
        if (pIdx == 1) b0[i] = plainB.mData[i];
        if (pIdx == 2) b1[i] = plainB.mData[i];
    }
    sbMatrix B = mat(n, A.bitCount(), b0, b1);
    bool_cipher_eq(pIdx, A, B, res, eval, runtime);
}

void bool_cipher_or(int, const boolShare& A, const boolShare& B, boolShare& res, Sh3Runtime& runtime) {
    const bool cross = (A.bshares[0] && B.bshares[0]) ^ (A.bshares[0] && B.bshares[1]) ^ (A.bshares[1] && B.bshares[0]);
    const u8 share = (u8)(cross ^ A.bshares[0] ^ B.bshares[0]);
    runtime.mComm.mNext.asyncSendCopy(share);
    u8 other = 0;
    runtime.mComm.mPrev.recv(other);
    res = boolShare(share != 0, other != 0);
}

void bool_cipher_not(int pIdx, const boolShare& A, boolShare& res) {
    res = A;
    if (pIdx == 1) res.bshares[0] = !A.bshares[0];
    if (pIdx == 2) res.bshares[1] = !A.bshares[1];
}

void bool_init_false(int pIdx, boolShare& res) {
    // (1, 0), (1, 1), (0, 1): x0 = 1, x1 = 1, x2 = 0
    res = boolShare(pIdx != 2, pIdx != 0);
}

void bool_cipher_dot(int pIdx, const sbMatrix& A, const sbMatrix& B, sbMatrix& res, Sh3Evaluator& eval,
                     Sh3Runtime& runtime) {
    sbMatrix prod;
    bool_cipher_and(pIdx, A, B, prod, eval, runtime);
    const std::vector<i64> p0 = prod.shareToHost(0), p1 = prod.shareToHost(1);
    std::vector<i64> r0(1, 0), r1(1, 0);
    for (u64 i = 0; i < A.i64Size(); ++i) {
        r0[0] ^= p0[i];
        r1[0] ^= p1[i];
    }
    res = mat(1, A.bitCount(), r0, r1);
}

void bool_cipher_dot(int pIdx, const std::vector<sbMatrix>& A, const sbMatrix& B, sbMatrix& res, Sh3Evaluator& eval,
                     Sh3Runtime& runtime) {
    const u64 n = A.size();
    if (n != B.rows()) throw std::invalid_argument("The size of sharedA and sharedB does not match!");
    const u64 block = A[0].i64Size(), bits = A[0].bitCount();
    std::vector<i64> b0 = B.shareToHost(0), b1 = B.shareToHost(1);
    if (B.bitCount() == 1) {
        b0 = expandBit(b0);
        b1 = expandBit(b1);
    }
    std::vector<i64> a0(n * block), a1(n * block), e0(n * block), e1(n * block);
    for (u64 i = 0; i < n; ++i) {
        const std::vector<i64> x0 = A[i].shareToHost(0), x1 = A[i].shareToHost(1);
        for (u64 j = 0; j < block; ++j) {
            a0[i * block + j] = x0[j];
            a1[i * block + j] = x1[j];
            e0[i * block + j] = b0[i];
            e1[i * block + j] = b1[i];
        }
    }
    sbMatrix prod;
    bool_cipher_and(pIdx, mat(n * block, bits, a0, a1), mat(n * block, bits, e0, e1), prod, eval, runtime);
    const std::vector<i64> p0 = prod.shareToHost(0), p1 = prod.shareToHost(1);
    std::vector<i64> r0(block, 0), r1(block, 0);
    for (u64 i = 0; i < n; ++i)
        for (u64 j = 0; j < block; ++j) {
            r0[j] ^= p0[i * block + j];
            r1[j] ^= p1[i * block + j];
        }
    res = mat(block, bits, r0, r1);
}

void bool_cipher_selector(int pIdx, const boolShare& flag, const sbMatrix& trueVal, const sbMatrix& falseVal,
                          sbMatrix& res, Sh3Evaluator& eval, Sh3Runtime& runtime) {
    if (trueVal.bitCount() != 64) throw std::runtime_error("The bitsize must be 64!");
    const u64 n = trueVal.i64Size();
    boolShare nFlag;
    bool_cipher_not(pIdx, flag, nFlag);
    auto fill = [&](const boolShare& f) {
        return mat(n, 64, std::vector<i64>(n, f.bshares[0] ? -1 : 0), std::vector<i64>(n, f.bshares[1] ? -1 : 0));
    };
    sbMatrix t, f;
    bool_cipher_and(pIdx, fill(flag), trueVal, t, eval, runtime);
    bool_cipher_and(pIdx, fill(nFlag), falseVal, f, eval, runtime);
    const std::vector<i64> t0 = t.shareToHost(0), t1 = t.shareToHost(1), f0 = f.shareToHost(0), f1 = f.shareToHost(1);
    std::vector<i64> r0(n), r1(n);
    for (u64 i = 0; i < n; ++i) {
        r0[i] = t0[i] ^ f0[i];
        r1[i] = t1[i] ^ f1[i];
    }
    res = mat(n, 64, r0, r1);
}

void bool_get_first_zero_mask(int pIdx, const std::vector<boolShare>& A, sbMatrix& res, Sh3Evaluator& eval,
                              Sh3Runtime& runtime) {
    const u64 len = A.size();
    const u64 rounds = (u64)std::floor(std::log2((double)len));
    // not(A), rotated right by one, first entry (0, 0)
    std::vector<i64> m0(len, 0), m1(len, 0);
    for (u64 i = 1; i < len; ++i) {
        boolShare nA;
        bool_cipher_not(pIdx, A[i - 1], nA);
        m0[i] = nA.bshares[0];
        m1[i] = nA.bshares[1];
    }
    // log-round prefix OR
    for (u64 r = 0; r < rounds; ++r) {
        const u64 stride = 1ull << r, k = len - stride;
        std::vector<i64> x0(m0.begin() + stride, m0.end()), x1(m1.begin() + stride, m1.end());
        std::vector<i64> y0(m0.begin(), m0.begin() + k), y1(m1.begin(), m1.begin() + k);
        sbMatrix o;
        bool_cipher_or(pIdx, mat(k, 1, x0, x1), mat(k, 1, y0, y1), o, eval, runtime);
        const std::vector<i64> o0 = o.shareToHost(0), o1 = o.shareToHost(1);
        for (u64 j = stride; j < len; ++j) {
            m0[j] = o0[j - stride];
            m1[j] = o1[j - stride];
        }
    }
    std::vector<i64> r0(len), r1(len);
    for (u64 i = 0; i + 1 < len; ++i) {
        r0[i] = m0[i] ^ m0[i + 1];
        r1[i] = m1[i] ^ m1[i + 1];
    }
    r0[len - 1] = m0[len - 1] ^ 1;
    r1[len - 1] = m1[len - 1] ^ 1;
    res = mat(len, 1, r0, r1);
}

void bool_shift_and_left(int, const boolIndex& A, u64 k, boolIndex& shifted, boolIndex& left) {
    const i64 mask = (i64)((1 << k) - 1);  // int arithmetic, as the reference
    shifted = boolIndex(A.indexShares[0] >> k, A.indexShares[1] >> k);
    left = boolIndex(A.indexShares[0] & mask, A.indexShares[1] & mask);
}

i64 back2plain(int, const boolIndex& x, Sh3Runtime& runtime) {
    runtime.mComm.mPrev.asyncSendCopy(x.indexShares[0]);
    i64 other = 0;
    runtime.mComm.mNext.recv(other);
    return other ^ x.indexShares[1] ^ x.indexShares[0];
}

// ---- position map (SqrtOram.h:60-387) ---------------------------------------

namespace {
// pack_to_single_matrix / unpack_from_single_matrix (SqrtOram.h:22-48)
sbMatrix packIndex(const ABY3PackedIndex& p) {
    std::vector<boolIndex> v{p.logicalIndex};
    v.insert(v.end(), p.packedIndices.begin(), p.packedIndices.end());
    return indexColumn(v);
}
void unpackIndex(const sbMatrix& m, ABY3PackedIndex& p) {
    const std::vector<i64> s0 = m.shareToHost(0), s1 = m.shareToHost(1);
    p.pack = m.rows() - 1;
    p.logicalIndex = boolIndex(s0[0], s1[0]);
    p.packedIndices.resize(p.pack);
    for (u64 i = 0; i < p.pack; ++i) p.packedIndices[i] = boolIndex(s0[i + 1], s1[i + 1]);
}
}  // namespace

ABY3PosMap::ABY3PosMap(u64 n_, u64 pack_, u64 S_, const std::vector<boolIndex>& perm, int p, Sh3Encryptor& e,
                       Sh3Evaluator& ev, Sh3Runtime& rt)
    : n(n_), pack(pack_), S(S_), pIdx(p), enc(&e), eval(&ev), runtime(&rt) {
    if (!pack || (pack & (pack - 1))) throw std::runtime_error("pack = " + std::to_string(pack) + " must be a power of 2.");
    map_len = n / pack;
    mLinear = map_len < S;  // oram.h:106-111
    if (mLinear) {
        usage_map.resize(n);
        for (auto& u : usage_map) bool_init_false(pIdx, u);
        permutation = perm;
        return;
    }
    // 1. the packed map: entry i holds the physical indices of logical i*pack .. i*pack+pack-1
    for (u64 i = 0; i < map_len; ++i) {
        ABY3PackedIndex q;
        q.pack = pack;
        q.logicalIndex = boolIndex((i64)i, pIdx);
        q.packedIndices.assign(perm.begin() + i * pack, perm.begin() + (i + 1) * pack);
        packed_index.push_back(q);
    }
    // 2. shuffle it, keeping the shares of the permutation (Pi)
    std::vector<sbMatrix> mats(map_len);
    for (u64 i = 0; i < map_len; ++i) mats[i] = packIndex(packed_index[i]);
    std::vector<si64> Pi;
    efficient_shuffle_with_random_permutation(mats, pIdx, mats, Pi, *enc, *eval, *runtime);
    for (u64 i = 0; i < map_len; ++i) unpackIndex(mats[i], packed_index[i]);
    // 3. the sub-map over the packed entries' positions
    std::vector<boolIndex> sub(map_len);
    for (u64 i = 0; i < map_len; ++i) sub[i] = boolIndex(Pi[i].mData[0], Pi[i].mData[1]);
    subPosMap = std::make_unique<ABY3PosMap>(map_len, pack, S, sub, pIdx, *enc, *eval, *runtime);
}

void ABY3PosMap::linear_ram(const std::vector<sbMatrix>& data, const boolIndex& index, sbMatrix& res) {
    sbMatrix s1;
    bool_cipher_eq(pIdx, repeatIndex(index, data.size()), range(data.size()), s1, *eval, *runtime);
    bool_cipher_dot(pIdx, data, s1, res, *eval, *runtime);
}

i64 ABY3PosMap::access(const boolIndex& index, const boolShare& fake) {
    boolIndex physical;
    if (mLinear) {
        // s1: the entry of `index`; s2: the first unused entry (SqrtOram.h:136-160)
        sbMatrix s1, s2;
        bool_cipher_eq(pIdx, repeatIndex(index, n), range(n), s1, *eval, *runtime);
        bool_get_first_zero_mask(pIdx, usage_map, s2, *eval, *runtime);
        const std::vector<i64> s10 = s1.shareToHost(0), s11 = s1.shareToHost(1);
        const sbMatrix s1m = mat(n, BITSIZE, expandBit(s10), expandBit(s11));
        const sbMatrix s2m = mat(n, BITSIZE, expandBit(s2.shareToHost(0)), expandBit(s2.shareToHost(1)));
        // the physical index: dot products with the permutation, selected by `fake` (:174-191)
        const sbMatrix perm = indexColumn(permutation);
        sbMatrix r1, r2, r;
        bool_cipher_dot(pIdx, perm, s1m, r1, *eval, *runtime);
        bool_cipher_dot(pIdx, perm, s2m, r2, *eval, *runtime);
        bool_cipher_selector(pIdx, fake, r2, r1, r, *eval, *runtime);
        physical = boolIndex(r.shareToHost(0)[0], r.shareToHost(1)[0]);
        // usage_map |= s1 (bit 0 of the expanded masks) (:193-205)
        std::vector<i64> u0(n), u1(n);
        for (u64 i = 0; i < n; ++i) {
            u0[i] = usage_map[i].bshares[0];
            u1[i] = usage_map[i].bshares[1];
        }
        sbMatrix used;
        bool_cipher_or(pIdx, mat(n, 1, expandBit(s10), expandBit(s11)), mat(n, 1, u0, u1), used, *eval, *runtime);
        const std::vector<i64> o0 = used.shareToHost(0), o1 = used.shareToHost(1);
        for (u64 i = 0; i < n; ++i) usage_map[i] = boolShare((o0[i] & 1) != 0, (o1[i] & 1) != 0);
    } else {
        boolIndex h, l;
        bool_shift_and_left(pIdx, index, (u64)std::log2((double)pack), h, l);
        boolShare found = fake;
        sbMatrix inStash = indexColumn({boolIndex(-1, pIdx)});
        if (t > 0) {
            // 1. is h in the stash? (:216-247)
            std::vector<boolIndex> si(t);
            for (u64 i = 0; i < t; ++i) si[i] = stash[i].logicalIndex;
            sbMatrix hit;
            bool_cipher_eq(pIdx, repeatIndex(h, t), indexColumn(si), hit, *eval, *runtime);
            const std::vector<i64> hit0 = hit.shareToHost(0), hit1 = hit.shareToHost(1);
            boolShare tmp((hit0[0] & 1) != 0, (hit1[0] & 1) != 0);
            for (u64 i = 1; i < t; ++i) {
                tmp.bshares[0] ^= (hit0[i] & 1);
                tmp.bshares[1] ^= (hit1[i] & 1);
            }
            bool_cipher_or(pIdx, found, tmp, found, *runtime);
            // 2. its l-th packed index (:249-304)
            sbMatrix perStash;
            bool_cipher_eq(pIdx, repeatIndex(l, pack), range(pack), perStash, *eval, *runtime);
            const std::vector<i64> ps0 = perStash.shareToHost(0), ps1 = perStash.shareToHost(1);
            std::vector<i64> eh0(t * pack), eh1(t * pack), el0(t * pack), el1(t * pack), sx0(t * pack), sx1(t * pack);
            for (u64 i = 0; i < t; ++i)
                for (u64 j = 0; j < pack; ++j) {
                    const u64 k = i * pack + j;
                    eh0[k] = hit0[i] == 1 ? -1 : 0;
                    eh1[k] = hit1[i] == 1 ? -1 : 0;
                    el0[k] = ps0[j] == 1 ? -1 : 0;
                    el1[k] = ps1[j] == 1 ? -1 : 0;
                    sx0[k] = stash[i].packedIndices[j].indexShares[0];
                    sx1[k] = stash[i].packedIndices[j].indexShares[1];
                }
            sbMatrix target;
            bool_cipher_and(pIdx, mat(t * pack, BITSIZE, eh0, eh1), mat(t * pack, BITSIZE, el0, el1), target, *eval,
                            *runtime);
            bool_cipher_dot(pIdx, target, mat(t * pack, BITSIZE, sx0, sx1), inStash, *eval, *runtime);
        }
        // 3. the packed entry's position from the sub-map (:307)
        const i64 next = subPosMap->access(h, found);
        if (next < 0 || (u64)next >= packed_index.size()) throw std::runtime_error("posMap: sub-map index out of range");
        // 4. stash hit -> the stashed index, else (or fake) the fetched entry's (:310-347)
        boolShare mainFlag;
        bool_cipher_not(pIdx, found, mainFlag);
        bool_cipher_or(pIdx, mainFlag, fake, mainFlag, *runtime);
        stash.push_back(packed_index[(u64)next]);
        ++t;
        std::vector<sbMatrix> elems;
        for (u64 i = 0; i < pack; ++i) elems.push_back(indexColumn({packed_index[(u64)next].packedIndices[i]}));
        sbMatrix fetched, r;
        linear_ram(elems, l, fetched);
        bool_cipher_selector(pIdx, mainFlag, fetched, inStash, r, *eval, *runtime);
        physical = boolIndex(r.shareToHost(0)[0], r.shareToHost(1)[0]);
    }
    last_physical_index = physical;
    return back2plain(pIdx, physical, *runtime);
}

// ---- the ORAM (SqrtOram.h:389-450) -----------------------------------------

ABY3SqrtOram::ABY3SqrtOram(int n_, int S_, int pack_, int p, Sh3Encryptor& e, Sh3Evaluator& ev, Sh3Runtime& rt)
    : n(n_), S(S_), pack(pack_), pIdx(p), enc(&e), eval(&ev), runtime(&rt) {
    // the reference clamps its constructor argument, not the member (:400-401): S is kept
    shuffle_mem.resize((size_t)n);
}

void ABY3SqrtOram::initiate(std::vector<sbMatrix>& data) {
    std::vector<si64> Pi;
    efficient_shuffle_with_random_permutation(data, pIdx, shuffle_mem, Pi, *enc, *eval, *runtime);
    std::vector<boolIndex> perm((size_t)n);
    for (int i = 0; i < n; ++i) perm[(size_t)i] = boolIndex(Pi[(size_t)i].mData[0], Pi[(size_t)i].mData[1]);
    posMap = std::make_unique<ABY3PosMap>((u64)n, (u64)pack, (u64)S, perm, pIdx, *enc, *eval, *runtime);
}

sbMatrix ABY3SqrtOram::access(const boolIndex& index) {
    // (:412-438) The reference consults its stash while t > 0, but never
    // advances t (the accessed elements go to the derived class's own stash
    // vector while t is the base class's), so every access reads through the
    // position map with found = false, as here.
    const boolShare found(false, pIdx);
    const i64 phy = posMap->access(index, found);
    if (phy < 0 || phy >= n) throw std::runtime_error("sqrt-ORAM: physical index out of range");
    sbMatrix res;
    res.copyFrom(shuffle_mem[(size_t)phy]);
    StashElement se;
    se.data.copyFrom(res);
    se.logicalIndex = index;
    stash.push_back(std::move(se));
    return res;
}

}  // namespace aby3
