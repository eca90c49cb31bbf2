#include "Shuffle.h"
#include "aby3ML.h"
#include <numeric>

namespace aby3 {

// BoolBasic.cpp:925-934: std::random_shuffle(0..len-1, PRNG(seed)) -- libstdc++
// swaps element i with element rng(i + 1) for i = 1 .. len-1, and cryptoTools'
// PRNG functor returns get<u64>() % n (the same restatement as getSubset's,
// aby3ML.cpp BatchSampler).
void get_permutation(size_t len, std::vector<size_t>& permutation, block seed) {
    permutation.resize(len);
    std::iota(permutation.begin(), permutation.end(), size_t(0));
    HostPrng prng(seed);
    for (size_t i = 1; i < len; ++i) {
        const size_t j = (size_t)(prng.get<u64>() % (i + 1));
        if (i != j) std::swap(permutation[i], permutation[j]);
    }
}

// BoolBasic.cpp:936-944
void get_inverse_permutation(const std::vector<size_t>& permutation, std::vector<size_t>& inverse_permutation) {
    inverse_permutation.resize(permutation.size());
    for (size_t i = 0; i < permutation.size(); ++i) inverse_permutation[permutation[i]] = i;
}

// BoolBasic.cpp:946-961: the scattering plain_permutate of every permutation's
// inverse, last first, applied to the identity
void combine_permutation(const std::vector<std::vector<size_t>>& permutation_list,
                         std::vector<size_t>& final_permutation) {
    const size_t len = permutation_list[0].size();
    final_permutation.resize(len);
    std::iota(final_permutation.begin(), final_permutation.end(), size_t(0));
    for (size_t k = permutation_list.size(); k-- > 0;) {
        std::vector<size_t> inv;
        get_inverse_permutation(permutation_list[k], inv);
        std::vector<size_t> tmp(len);
        for (size_t i = 0; i < len; ++i) tmp[inv[i]] = final_permutation[i];
        final_permutation.swap(tmp);
    }
}

namespace {

// A party's permutation of (seed, len) on its GPU: forward and inverse index
// arrays (u32), built on the host once and cached with the Gpu (they depend
// on the seed and the length only).
struct DevPerm {
    DeviceBuffer fwd, inv;
    const u32* f() const { return fwd.as<u32>(); }
    const u32* i() const { return inv.as<u32>(); }
};
std::shared_ptr<DevPerm> devPerm(Gpu& g, block seed, u64 len) {
    if (len > 0xffffffffull) throw std::runtime_error("shuffle: at most 2^32 - 1 units");
    u64 h = seed.lo * 0x9E3779B97F4A7C15ull ^ (seed.hi + 0x632BE59BD9B4E019ull) * 0xC2B2AE3D27D4EB4Full;
    h ^= len * 0x165667B19E3779F9ull;
    const u64 key = (h << 8) | 0x05;
    return std::static_pointer_cast<DevPerm>(g.attachment(key, [&]() -> std::shared_ptr<void> {
        std::vector<size_t> p, q;
        get_permutation(len, p, seed);
        get_inverse_permutation(p, q);
        std::vector<u32> a(p.begin(), p.end()), b(q.begin(), q.end());
        auto d = std::make_shared<DevPerm>();
        d->fwd.reset(g, std::max<u64>(4 * len, 4));
        d->inv.reset(g, std::max<u64>(4 * len, 4));
        if (len) {
            toDevice(d->fwd.data(), a.data(), 4 * len, g);
            toDevice(d->inv.data(), b.data(), 4 * len, g);
        }
        return d;
    }));
}

// get_random_mask (BoolBasic.cpp:963-968): words [0, n) of a fresh PRNG(seed)
DeviceBuffer randomMask(Gpu& g, block seed, u64 n) {
    DeviceBuffer m(g, std::max<u64>(8 * n, 8));
    if (n) GPU_CALL(aby3g_prng_fill(seed.data(), 0, 8 * n, m.data(), g.stream()));
    return m;
}

// out[i] = a[g] ^ b[g] ^ c[g] ^ mask, g = idx[i] (idx null: i)
void xg(Gpu& g, u64 units, u64 unit, const u32* idx, const u64* a, const u64* b, const u64* c, const u64* mask,
        u64* out) {
    GPU_CALL(aby3g_u64_xor_gather_units(units, unit, idx, a, b, c, mask, out, g.stream()));
}

void sendWords(Sh3Runtime& rt, int p, bool toNext, const u64* d, u64 n) {
    large_data_sending(p, reinterpret_cast<const i64*>(d), n, rt, toNext);
}
void recvWords(Sh3Runtime& rt, int p, bool fromPrev, u64* d, u64 n) {
    large_data_receiving(p, reinterpret_cast<i64*>(d), n, rt, fromPrev);
}

struct Seeds {
    block prev, next;
};
Seeds seedsOf(Sh3Encryptor& enc) { return {enc.mShareGen.mPrevSeed, enc.mShareGen.mNextSeed}; }

}  // namespace

// Shuffle.cpp:14-226 on packed units. Every scattering plain_permutate(p, x)
// is the gather of x by p^-1; masks are the same for every unit.
int efficient_shuffle_units(const u64* T, u64 len, u64 unit, int pIdx, u64* Tres, Sh3Encryptor& enc,
                            Sh3Runtime& runtime) {
    if (T == Tres) throw std::invalid_argument("efficient_shuffle: Tres may not alias T");
    Gpu& g = runtime.gpu();
    const u64 L = len * unit;
    if (!L) return 0;
    const Seeds s = seedsOf(enc);
    auto pp = devPerm(g, s.prev, len), pn = devPerm(g, s.next, len);
    DeviceBuffer zp = randomMask(g, s.prev, unit), zn = randomMask(g, s.next, unit), zx(g, 8 * unit);
    xg(g, 1, unit, nullptr, zp.as<u64>(), zn.as<u64>(), nullptr, nullptr, zx.as<u64>());  // zp ^ zn
    const u64 *T0 = T, *T1 = T + L;
    u64 *R0 = Tres, *R1 = Tres + L;
    DeviceBuffer a(g, 8 * L), b(g, 8 * L);
    if (pIdx == 0) {
        // X1 = P(pn, T0 ^ T1 ^ Zn), X2 = P(pp, X1 ^ Zp) -> P1 (:52-81)
        xg(g, len, unit, pn->i(), T0, T1, nullptr, zn.as<u64>(), a.as<u64>());
        xg(g, len, unit, pp->i(), a.as<u64>(), nullptr, nullptr, zp.as<u64>(), b.as<u64>());
        sendWords(runtime, pIdx, true, b.as<u64>(), L);
        // (maskB, maskA) = (Zn, Zp) (:84-90)
        xg(g, len, unit, nullptr, nullptr, nullptr, nullptr, zn.as<u64>(), R0);
        xg(g, len, unit, nullptr, nullptr, nullptr, nullptr, zp.as<u64>(), R1);
    } else if (pIdx == 1) {
        // Y1 = P(pp, T0 ^ Zp) -> P2 (:100-117)
        xg(g, len, unit, pp->i(), T0, nullptr, nullptr, zp.as<u64>(), a.as<u64>());
        sendWords(runtime, pIdx, true, a.as<u64>(), L);
        // X2 <- P0; C1 = P(pn, X2 ^ Zn) ^ maskB (= Zp) -> P2 (:119-144)
        DeviceBuffer x2(g, 8 * L);
        recvWords(runtime, pIdx, true, x2.as<u64>(), L);
        xg(g, len, unit, pn->i(), x2.as<u64>(), nullptr, nullptr, zx.as<u64>(), b.as<u64>());
        sendWords(runtime, pIdx, true, b.as<u64>(), L);
        // C2 <- P2; shares (C1 ^ C2, Zp) (:146-158)
        recvWords(runtime, pIdx, false, a.as<u64>(), L);
        xg(g, len, unit, nullptr, a.as<u64>(), b.as<u64>(), nullptr, nullptr, R0);
        xg(g, len, unit, nullptr, nullptr, nullptr, nullptr, zp.as<u64>(), R1);
    } else {
        // Y1 <- P1; C2 = P(pp, P(pn, Y1 ^ Zn) ^ Zp) ^ maskA (= Zn) -> P1 (:168-202)
        recvWords(runtime, pIdx, true, a.as<u64>(), L);
        xg(g, len, unit, pn->i(), a.as<u64>(), nullptr, nullptr, zn.as<u64>(), b.as<u64>());
        xg(g, len, unit, pp->i(), b.as<u64>(), nullptr, nullptr, zx.as<u64>(), a.as<u64>());
        sendWords(runtime, pIdx, false, a.as<u64>(), L);
        // C1 <- P1; shares (Zn, C1 ^ C2) (:203-223)
        recvWords(runtime, pIdx, true, b.as<u64>(), L);
        xg(g, len, unit, nullptr, nullptr, nullptr, nullptr, zn.as<u64>(), R0);
        xg(g, len, unit, nullptr, a.as<u64>(), b.as<u64>(), nullptr, nullptr, R1);
    }
    return 0;
}

// Shuffle.cpp:229-385 on the first word of each row: gathering permutations
// (res(i) = x(p(i))) and one mask word per row (words [0, len) of the seed's
// stream).
int efficient_shuffle_rows(const u64* T, u64 len, int pIdx, u64* Tres, Sh3Encryptor& enc, Sh3Runtime& runtime) {
    if (T == Tres) throw std::invalid_argument("efficient_shuffle: Tres may not alias T");
    Gpu& g = runtime.gpu();
    if (!len) return 0;
    const Seeds s = seedsOf(enc);
    auto pp = devPerm(g, s.prev, len), pn = devPerm(g, s.next, len);
    DeviceBuffer Zp = randomMask(g, s.prev, len), Zn = randomMask(g, s.next, len);
    const u64 *T0 = T, *T1 = T + len;
    u64 *R0 = Tres, *R1 = Tres + len;
    DeviceBuffer a(g, 8 * len), b(g, 8 * len);
    if (pIdx == 0) {
        // X1 = gather(T0 ^ T1 ^ Zn, pn), X2 = gather(X1 ^ Zp, pp) -> P1 (:258-274)
        xg(g, len, 1, pn->f(), T0, T1, Zn.as<u64>(), nullptr, a.as<u64>());
        xg(g, len, 1, pp->f(), a.as<u64>(), Zp.as<u64>(), nullptr, nullptr, b.as<u64>());
        sendWords(runtime, pIdx, true, b.as<u64>(), len);
        xg(g, len, 1, nullptr, Zp.as<u64>(), nullptr, nullptr, nullptr, R1);  // maskA
        xg(g, len, 1, nullptr, Zn.as<u64>(), nullptr, nullptr, nullptr, R0);  // maskB
    } else if (pIdx == 1) {
        // Y1 = gather(T0 ^ Zp, pp) -> P2 (:288-296)
        xg(g, len, 1, pp->f(), T0, Zp.as<u64>(), nullptr, nullptr, a.as<u64>());
        sendWords(runtime, pIdx, true, a.as<u64>(), len);
        // X2 <- P0, X3 = gather(X2 ^ Zn, pn); C2 <- P2; C1 = X3 ^ maskB (= Zp) -> P2 (:298-327)
        DeviceBuffer x2(g, 8 * len), c2(g, 8 * len);
        recvWords(runtime, pIdx, true, x2.as<u64>(), len);
        xg(g, len, 1, pn->f(), x2.as<u64>(), Zn.as<u64>(), nullptr, nullptr, b.as<u64>());
        recvWords(runtime, pIdx, false, c2.as<u64>(), len);
        xg(g, len, 1, nullptr, b.as<u64>(), Zp.as<u64>(), nullptr, nullptr, a.as<u64>());
        sendWords(runtime, pIdx, true, a.as<u64>(), len);
        // shares (C1 ^ C2, Zp) (:330-334)
        xg(g, len, 1, nullptr, a.as<u64>(), c2.as<u64>(), nullptr, nullptr, R0);
        xg(g, len, 1, nullptr, Zp.as<u64>(), nullptr, nullptr, nullptr, R1);
    } else {
        // Y1 <- P1; Y3 = gather(gather(Y1 ^ Zn, pn) ^ Zp, pp); C2 = Y3 ^ maskA (= Zn) -> P1 (:341-365)
        recvWords(runtime, pIdx, true, a.as<u64>(), len);
        xg(g, len, 1, pn->f(), a.as<u64>(), Zn.as<u64>(), nullptr, nullptr, b.as<u64>());
        xg(g, len, 1, pp->f(), b.as<u64>(), Zp.as<u64>(), nullptr, nullptr, a.as<u64>());
        xg(g, len, 1, nullptr, a.as<u64>(), Zn.as<u64>(), nullptr, nullptr, b.as<u64>());
        sendWords(runtime, pIdx, false, b.as<u64>(), len);
        // C1 <- P1; shares (Zn, C1 ^ C2) (:367-381)
        recvWords(runtime, pIdx, true, a.as<u64>(), len);
        xg(g, len, 1, nullptr, Zn.as<u64>(), nullptr, nullptr, nullptr, R0);
        xg(g, len, 1, nullptr, a.as<u64>(), b.as<u64>(), nullptr, nullptr, R1);
    }
    return 0;
}

// Shuffle.cpp:388-903 on packed units: the shuffle as efficient_shuffle, then
// the binary shares of the applied permutation: party 2's plain index tags
// (i, ~0) travel back through the inverse permutations (RX), party 1's
// (~0, ~0) likewise (RY), and the parties reshare the result (maskRB).
// Masks R* are words [0, len) of the seed streams (every get_random_mask call
// restarts the stream, so maskRA / maskRC equal the RZ masks of their seed).
int efficient_shuffle_with_random_permutation_units(const u64* T, u64 len, u64 unit, int pIdx, u64* Tres, u64* Pi,
                                                    Sh3Encryptor& enc, Sh3Runtime& runtime) {
    if (T == Tres) throw std::invalid_argument("efficient_shuffle: Tres may not alias T");
    Gpu& g = runtime.gpu();
    const u64 L = len * unit;
    if (!L) return 0;
    const Seeds s = seedsOf(enc);
    auto pp = devPerm(g, s.prev, len), pn = devPerm(g, s.next, len);
    DeviceBuffer zp = randomMask(g, s.prev, unit), zn = randomMask(g, s.next, unit);
    DeviceBuffer Rp = randomMask(g, s.prev, len), Rn = randomMask(g, s.next, len);
    const u64 *T0 = T, *T1 = T + L;
    u64 *R0 = Tres, *R1 = Tres + L, *Pi0 = Pi, *Pi1 = Pi + len;
    DeviceBuffer a(g, 8 * L), b(g, 8 * L), r(g, 8 * len), q(g, 8 * len);
    if (pIdx == 0) {
        // X2 = P(pp, P(pn, T0 ^ T1 ^ Zn) ^ Zp) -> P1 (:435-477)
        xg(g, len, unit, pn->i(), T0, T1, nullptr, zn.as<u64>(), a.as<u64>());
        xg(g, len, unit, pp->i(), a.as<u64>(), nullptr, nullptr, zp.as<u64>(), b.as<u64>());
        sendWords(runtime, pIdx, true, b.as<u64>(), L);
        // RY1 <- P1; RY3 = P(pn^-1, P(pp^-1, RY1 ^ RZp) ^ RZn) (:492-531)
        recvWords(runtime, pIdx, false, r.as<u64>(), len);
        xg(g, len, 1, pp->f(), r.as<u64>(), Rp.as<u64>(), nullptr, nullptr, q.as<u64>());
        xg(g, len, 1, pn->f(), q.as<u64>(), Rn.as<u64>(), nullptr, nullptr, r.as<u64>());
        // maskRB2 = RY3 ^ maskRA (= RZp) <-> P1; Pi = (maskRB1 ^ maskRB2, maskRA) (:541-570)
        xg(g, len, 1, nullptr, r.as<u64>(), Rp.as<u64>(), nullptr, nullptr, q.as<u64>());
        sendWords(runtime, pIdx, true, q.as<u64>(), len);
        recvWords(runtime, pIdx, false, r.as<u64>(), len);
        xg(g, len, 1, nullptr, r.as<u64>(), q.as<u64>(), nullptr, nullptr, Pi0);
        xg(g, len, 1, nullptr, Rp.as<u64>(), nullptr, nullptr, nullptr, Pi1);
        // Tres = (maskB, maskA) = (Zn, Zp) (:577-588)
        xg(g, len, unit, nullptr, nullptr, nullptr, nullptr, zn.as<u64>(), R0);
        xg(g, len, unit, nullptr, nullptr, nullptr, nullptr, zp.as<u64>(), R1);
    } else if (pIdx == 1) {
        // Y1 = P(pp, T0 ^ Zp) -> P2; X2 <- P0 (:597-640)
        xg(g, len, unit, pp->i(), T0, nullptr, nullptr, zp.as<u64>(), a.as<u64>());
        sendWords(runtime, pIdx, true, a.as<u64>(), L);
        recvWords(runtime, pIdx, true, b.as<u64>(), L);
        // C1 = P(pn, X2 ^ Zn) ^ maskB (= Zp) -> P2, C2 <- P2, Tres = (C1 ^ C2, Zp) (:650-683)
        xg(g, len, unit, pn->i(), b.as<u64>(), nullptr, nullptr, zn.as<u64>(), a.as<u64>());
        xg(g, len, unit, nullptr, a.as<u64>(), nullptr, nullptr, zp.as<u64>(), b.as<u64>());
        sendWords(runtime, pIdx, true, b.as<u64>(), L);
        recvWords(runtime, pIdx, false, a.as<u64>(), L);
        xg(g, len, unit, nullptr, a.as<u64>(), b.as<u64>(), nullptr, nullptr, R0);
        xg(g, len, unit, nullptr, nullptr, nullptr, nullptr, zp.as<u64>(), R1);
        // RY1 = P(pn^-1, ~0 ^ RZn) -> P0; RX2 <- P2 (:691-719)
        DeviceBuffer ones(g, 8);
        GPU_CALL(aby3g_memset(ones.data(), 0xff, 8, g.stream()));
        xg(g, len, 1, pn->f(), Rn.as<u64>(), nullptr, nullptr, ones.as<u64>(), r.as<u64>());
        sendWords(runtime, pIdx, false, r.as<u64>(), len);
        recvWords(runtime, pIdx, false, q.as<u64>(), len);
        // RX3 = P(pp^-1, RX2 ^ RZp); maskRB1 = RX3 ^ maskRC (= RZn) <-> P0 (:725-757)
        xg(g, len, 1, pp->f(), q.as<u64>(), Rp.as<u64>(), nullptr, nullptr, r.as<u64>());
        xg(g, len, 1, nullptr, r.as<u64>(), Rn.as<u64>(), nullptr, nullptr, q.as<u64>());
        sendWords(runtime, pIdx, false, q.as<u64>(), len);
        recvWords(runtime, pIdx, true, r.as<u64>(), len);
        // Pi = (maskRC, maskRB1 ^ maskRB2) (:762-765)
        xg(g, len, 1, nullptr, Rn.as<u64>(), nullptr, nullptr, nullptr, Pi0);
        xg(g, len, 1, nullptr, q.as<u64>(), r.as<u64>(), nullptr, nullptr, Pi1);
    } else {
        // Y1 <- P1; C2 = P(pp, P(pn, Y1 ^ Zn) ^ Zp) ^ maskA (= Zn) <-> P1 (:772-841)
        recvWords(runtime, pIdx, true, a.as<u64>(), L);
        xg(g, len, unit, pn->i(), a.as<u64>(), nullptr, nullptr, zn.as<u64>(), b.as<u64>());
        xg(g, len, unit, pp->i(), b.as<u64>(), nullptr, nullptr, zp.as<u64>(), a.as<u64>());
        xg(g, len, unit, nullptr, a.as<u64>(), nullptr, nullptr, zn.as<u64>(), b.as<u64>());
        sendWords(runtime, pIdx, false, b.as<u64>(), L);
        recvWords(runtime, pIdx, true, a.as<u64>(), L);
        xg(g, len, unit, nullptr, nullptr, nullptr, nullptr, zn.as<u64>(), R0);
        xg(g, len, unit, nullptr, a.as<u64>(), b.as<u64>(), nullptr, nullptr, R1);
        // RX1 = P(pp^-1, (i ^ ~0) ^ RZp); RX2 = P(pn^-1, RX1 ^ RZn) -> P1 (:852-878)
        std::vector<u64> tags(len);
        for (u64 i = 0; i < len; ++i) tags[i] = ~i;
        toDevice(q.data(), tags.data(), 8 * len, g);
        xg(g, len, 1, pp->f(), q.as<u64>(), Rp.as<u64>(), nullptr, nullptr, r.as<u64>());
        xg(g, len, 1, pn->f(), r.as<u64>(), Rn.as<u64>(), nullptr, nullptr, q.as<u64>());
        sendWords(runtime, pIdx, false, q.as<u64>(), len);
        // Pi = (maskRA, maskRC) = (RZn, RZp) (:885-894)
        xg(g, len, 1, nullptr, Rn.as<u64>(), nullptr, nullptr, nullptr, Pi0);
        xg(g, len, 1, nullptr, Rp.as<u64>(), nullptr, nullptr, nullptr, Pi1);
        g.sync();  // the host tag buffer is released on return
    }
    return 0;
}

namespace {
// the vector forms' units: T[i] one column of `unit` words each (the
// reference indexes T[i].mShares[s](j) for j < i64Size(), one column only)
u64 unitOf(const std::vector<sbMatrix>& T) {
    if (T.empty()) return 0;
    const u64 unit = T[0].rows();
    for (const auto& t : T)
        if (t.i64Cols() != 1 || t.rows() != unit)
            throw std::invalid_argument("efficient_shuffle: every unit must be one column of the same rows");
    return unit;
}
DeviceBuffer pack(const std::vector<sbMatrix>& T, u64 unit, Gpu& g) {
    const u64 len = T.size(), L = len * unit;
    DeviceBuffer d(g, std::max<u64>(16 * L, 16));
    for (u64 i = 0; i < len; ++i)
        for (int s = 0; s < 2; ++s) d2d(d.as<u64>() + s * L + i * unit, T[i].share(s), 8 * unit, g);
    return d;
}
void unpack(const DeviceBuffer& d, u64 unit, u64 bits, std::vector<sbMatrix>& Tres, Gpu& g) {
    const u64 L = Tres.size() * unit;
    for (u64 i = 0; i < Tres.size(); ++i) {
        Tres[i].resize(unit, bits);
        for (int s = 0; s < 2; ++s) d2d(Tres[i].share(s), d.as<u64>() + s * L + i * unit, 8 * unit, g);
    }
}
}  // namespace

int efficient_shuffle(std::vector<sbMatrix>& T, int pIdx, std::vector<sbMatrix>& Tres, Sh3Encryptor& enc,
                      Sh3Evaluator&, Sh3Runtime& runtime) {
    Gpu& g = runtime.gpu();
    const u64 unit = unitOf(T), len = T.size();
    if (!len) return 0;
    DeviceBuffer in = pack(T, unit, g), out(g, 16 * len * unit);
    efficient_shuffle_units(in.as<u64>(), len, unit, pIdx, out.as<u64>(), enc, runtime);
    Tres.resize(len);
    unpack(out, unit, T[0].bitCount(), Tres, g);
    return 0;
}

int efficient_shuffle(sbMatrix& T, int pIdx, sbMatrix& Tres, Sh3Encryptor& enc, Sh3Evaluator&, Sh3Runtime& runtime) {
    if (T.bitCount() > 64) throw std::invalid_argument("efficient_shuffle(sbMatrix): at most 64 bits per row");
    Gpu& g = runtime.gpu();
    const u64 len = T.rows();
    sbMatrix out(len, T.bitCount());
    efficient_shuffle_rows(reinterpret_cast<const u64*>(T.data()), len, pIdx, reinterpret_cast<u64*>(out.data()), enc,
                           runtime);
    Tres = std::move(out);
    (void)g;
    return 0;
}

int efficient_shuffle_with_random_permutation(std::vector<sbMatrix>& T, int pIdx, std::vector<sbMatrix>& Tres,
                                              std::vector<si64>& Pi, Sh3Encryptor& enc, Sh3Evaluator&,
                                              Sh3Runtime& runtime) {
    Gpu& g = runtime.gpu();
    const u64 unit = unitOf(T), len = T.size();
    Pi.resize(len);
    if (!len) return 0;
    DeviceBuffer in = pack(T, unit, g), out(g, 16 * len * unit), pi(g, 16 * len);
    efficient_shuffle_with_random_permutation_units(in.as<u64>(), len, unit, pIdx, out.as<u64>(), pi.as<u64>(), enc,
                                                    runtime);
    Tres.resize(len);
    unpack(out, unit, 64, Tres, g);  // BITSIZE (Shuffle.cpp:579)
    std::vector<i64> h(2 * len);
    toHost(h.data(), pi.data(), 16 * len, g);
    for (u64 i = 0; i < len; ++i) {
        Pi[i].mData[0] = h[i];
        Pi[i].mData[1] = h[len + i];
    }
    return 0;
}

}  // namespace aby3
