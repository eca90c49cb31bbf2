// TEST INFRASTRUCTURE ONLY -- CPU oracle. Only tests/, __graft_entry__.smoke()
// and bench.py's cpu_baseline leg may use anything under oracle/.
//
// Restatement of the 3-party shuffle of aby3-Basic/Shuffle.cpp with the
// helpers of BoolBasic.cpp:925-1042, written the reference's way: vectors of
// units, host permutations, one party after the other in message order.
// Units are rows of an SMat [len][unit].
#include "orc_core.h"
#include <numeric>

namespace orc {

namespace {
u64 word(const u8 seed[16], u64 i) {
    u64 v;
    prng_bytes(seed, 8 * i, 8, (u8*)&v);
    return v;
}
}  // namespace

// get_permutation (BoolBasic.cpp:925-934): std::random_shuffle(0..len-1, prng)
// with libstdc++'s loop (swap i with rng(i + 1), i = 1..len-1) and
// cryptoTools' functor rng(n) = get<u64>() % n.
std::vector<u64> shufflePermutation(u64 len, const u8 seed[16]) {
    std::vector<u64> p(len);
    std::iota(p.begin(), p.end(), 0ull);
    Stream s;
    s.init(seed);
    for (u64 i = 1; i < len; ++i) {
        u64 r;
        s.get(&r, 8);
        const u64 j = r % (i + 1);
        if (i != j) std::swap(p[i], p[j]);
    }
    return p;
}

namespace {
std::vector<u64> inverse(const std::vector<u64>& p) {
    std::vector<u64> q(p.size());
    for (u64 i = 0; i < p.size(); ++i) q[p[i]] = i;
    return q;
}
// get_random_mask (BoolBasic.cpp:963-968): words 0..n-1 of a fresh PRNG(seed)
std::vector<i64> randomMask(const u8 seed[16], u64 n) {
    std::vector<i64> m(n);
    for (u64 i = 0; i < n; ++i) m[i] = (i64)word(seed, i);
    return m;
}
using Units = std::vector<std::vector<i64>>;
// plain_permutate for std::vector<T> (Basics.h:324-332): tmp[p[i]] = data[i]
template <class T>
void scatter(const std::vector<u64>& p, std::vector<T>& data) {
    std::vector<T> tmp(data.size());
    for (u64 i = 0; i < data.size(); ++i) tmp[p[i]] = data[i];
    data.swap(tmp);
}
// plain_permutate for i64Matrix (BoolBasic.cpp:1033-1042): res(i) = data(p[i])
void gather(const std::vector<u64>& p, std::vector<i64>& data) {
    std::vector<i64> tmp(data.size());
    for (u64 i = 0; i < data.size(); ++i) tmp[i] = data[p[i]];
    data.swap(tmp);
}
Units unitsOf(const Mat& m) {
    Units u(m.rows, std::vector<i64>(m.cols));
    for (u64 i = 0; i < m.rows; ++i)
        for (u64 j = 0; j < m.cols; ++j) u[i][j] = m(i, j);
    return u;
}
void put(Mat& m, const Units& u) {
    for (u64 i = 0; i < m.rows; ++i)
        for (u64 j = 0; j < m.cols; ++j) m(i, j) = u[i][j];
}
Units xorMask(const Units& x, const std::vector<i64>& mask) {
    Units y = x;
    for (auto& r : y)
        for (u64 j = 0; j < r.size(); ++j) r[j] ^= mask[j];
    return y;
}
Units xorUnits(const Units& a, const Units& b) {
    Units y = a;
    for (u64 i = 0; i < y.size(); ++i)
        for (u64 j = 0; j < y[i].size(); ++j) y[i][j] ^= b[i][j];
    return y;
}
Units tile(u64 len, const std::vector<i64>& mask) { return Units(len, mask); }
struct PartyRand {
    std::vector<u64> pp, pn;  // prev / next permutations
    const u8* ps;
    const u8* ns;
};
PartyRand partyRand(Party& p, u64 len) {
    PartyRand r;
    r.ps = p.gen.prev.seed;
    r.ns = p.gen.next.seed;
    r.pp = shufflePermutation(len, r.ps);
    r.pn = shufflePermutation(len, r.ns);
    return r;
}
}  // namespace

// efficient_shuffle(std::vector<sbMatrix>) (Shuffle.cpp:14-226)
Shared shuffleUnits(std::array<Party, 3>& enc, const Shared& T) {
    const u64 len = T[0].rows(), unit = T[0].cols();
    std::array<PartyRand, 3> R = {partyRand(enc[0], len), partyRand(enc[1], len), partyRand(enc[2], len)};
    std::array<std::vector<i64>, 3> zp, zn;
    for (int i = 0; i < 3; ++i) {
        zp[i] = randomMask(R[i].ps, unit);
        zn[i] = randomMask(R[i].ns, unit);
    }
    Shared out;
    for (int i = 0; i < 3; ++i) out[i] = SMat(len, unit);
    // P0 (:41-91)
    Units x1 = xorMask(xorUnits(unitsOf(T[0].s[0]), unitsOf(T[0].s[1])), zn[0]);
    scatter(R[0].pn, x1);
    Units x2 = xorMask(x1, zp[0]);
    scatter(R[0].pp, x2);  // -> P1
    put(out[0].s[1], tile(len, zp[0]));  // maskA
    put(out[0].s[0], tile(len, zn[0]));  // maskB
    // P1 (:92-117): Y1 -> P2
    Units y1 = xorMask(unitsOf(T[1].s[0]), zp[1]);
    scatter(R[1].pp, y1);
    // P1 (:119-144): C1 -> P2
    Units x3 = xorMask(x2, zn[1]);
    scatter(R[1].pn, x3);
    Units c1 = xorMask(x3, zp[1]);  // maskB = Zp
    // P2 (:160-202): C2 -> P1
    Units y2 = xorMask(y1, zn[2]);
    scatter(R[2].pn, y2);
    Units y3 = xorMask(y2, zp[2]);
    scatter(R[2].pp, y3);
    Units c2 = xorMask(y3, zn[2]);  // maskA = Zn
    put(out[2].s[1], xorUnits(c1, c2));
    put(out[2].s[0], tile(len, zn[2]));
    // P1 (:146-158)
    put(out[1].s[1], tile(len, zp[1]));
    put(out[1].s[0], xorUnits(c1, c2));
    return out;
}

// efficient_shuffle(sbMatrix) (Shuffle.cpp:229-385): the first word of each row
Shared shuffleRows(std::array<Party, 3>& enc, const Shared& T) {
    const u64 len = T[0].rows();
    std::array<PartyRand, 3> R = {partyRand(enc[0], len), partyRand(enc[1], len), partyRand(enc[2], len)};
    std::array<std::vector<i64>, 3> Zp, Zn;
    for (int i = 0; i < 3; ++i) {
        Zp[i] = randomMask(R[i].ps, len);
        Zn[i] = randomMask(R[i].ns, len);
    }
    auto col = [&](const Mat& m) {
        std::vector<i64> v(len);
        for (u64 i = 0; i < len; ++i) v[i] = m(i, 0);
        return v;
    };
    auto x = [](std::vector<i64> a, const std::vector<i64>& b) {
        for (u64 i = 0; i < a.size(); ++i) a[i] ^= b[i];
        return a;
    };
    Shared out;
    for (int i = 0; i < 3; ++i) out[i] = SMat(len, 1);
    // P0 (:251-282)
    std::vector<i64> x1 = x(x(col(T[0].s[0]), col(T[0].s[1])), Zn[0]);
    gather(R[0].pn, x1);
    std::vector<i64> x2 = x(x1, Zp[0]);
    gather(R[0].pp, x2);
    out[0].s[1].v = Zp[0];
    out[0].s[0].v = Zn[0];
    // P1 (:283-296): Y1 -> P2
    std::vector<i64> y1 = x(col(T[1].s[0]), Zp[1]);
    gather(R[1].pp, y1);
    // P1 (:298-307)
    std::vector<i64> x3 = x(x2, Zn[1]);
    gather(R[1].pn, x3);
    // P2 (:336-365): C2 -> P1
    std::vector<i64> y2 = x(y1, Zn[2]);
    gather(R[2].pn, y2);
    std::vector<i64> y3 = x(y2, Zp[2]);
    gather(R[2].pp, y3);
    std::vector<i64> c2 = x(y3, Zn[2]);
    // P1 (:317-334): C1 = X3 ^ maskB (Zp) -> P2
    std::vector<i64> c1 = x(x3, Zp[1]);
    out[1].s[1].v = Zp[1];
    out[1].s[0].v = x(c1, c2);
    // P2 (:367-381)
    out[2].s[1].v = x(c1, c2);
    out[2].s[0].v = Zn[2];
    return out;
}

// efficient_shuffle_with_random_permutation (Shuffle.cpp:388-903); Pi [3] x (len x 1)
Shared shuffleWithPermutation(std::array<Party, 3>& enc, const Shared& T, Shared& Pi) {
    const u64 len = T[0].rows(), unit = T[0].cols();
    std::array<PartyRand, 3> R = {partyRand(enc[0], len), partyRand(enc[1], len), partyRand(enc[2], len)};
    std::array<std::vector<i64>, 3> zp, zn, Rp, Rn;
    for (int i = 0; i < 3; ++i) {
        zp[i] = randomMask(R[i].ps, unit);
        zn[i] = randomMask(R[i].ns, unit);
        Rp[i] = randomMask(R[i].ps, len);
        Rn[i] = randomMask(R[i].ns, len);
    }
    auto x = [](std::vector<i64> a, const std::vector<i64>& b) {
        for (u64 i = 0; i < a.size(); ++i) a[i] ^= b[i];
        return a;
    };
    Shared out;
    for (int i = 0; i < 3; ++i) {
        out[i] = SMat(len, unit);
        Pi[i] = SMat(len, 1);
    }
    // Pi initial values (:411-425): P1 (~0, ~0), P2 (i, ~0)
    const std::vector<i64> ones(len, ~0ll);
    std::vector<i64> idx(len);
    for (u64 i = 0; i < len; ++i) idx[i] = (i64)i;
    // P0 (:435-477): X2 -> P1
    Units x1 = xorMask(xorUnits(unitsOf(T[0].s[0]), unitsOf(T[0].s[1])), zn[0]);
    scatter(R[0].pn, x1);
    Units x2 = xorMask(x1, zp[0]);
    scatter(R[0].pp, x2);
    // P1 (:597-640): Y1 -> P2; X3 from X2
    Units y1 = xorMask(unitsOf(T[1].s[0]), zp[1]);
    scatter(R[1].pp, y1);
    Units x3 = xorMask(x2, zn[1]);
    scatter(R[1].pn, x3);
    // P1 (:652-661): X3 ^= maskB (Zp) -> P2
    Units c1 = xorMask(x3, zp[1]);
    // P2 (:772-827): C2 -> P1
    Units y2 = xorMask(y1, zn[2]);
    scatter(R[2].pn, y2);
    Units y3 = xorMask(y2, zp[2]);
    scatter(R[2].pp, y3);
    Units c2 = xorMask(y3, zn[2]);
    put(out[2].s[0], tile(len, zn[2]));
    put(out[2].s[1], xorUnits(c1, c2));  // (:830-841)
    put(out[1].s[1], tile(len, zp[1]));
    put(out[1].s[0], xorUnits(c1, c2));  // (:666-683)
    put(out[0].s[1], tile(len, zp[0]));
    put(out[0].s[0], tile(len, zn[0]));  // (:577-588)
    // P1 (:689-700): RY1 = P(pn^-1, Pi1 ^ RZn) -> P0
    std::vector<i64> ry1 = x(ones, Rn[1]);
    scatter(inverse(R[1].pn), ry1);
    // P2 (:851-878): RX2 -> P1
    std::vector<i64> rx1 = x(x(idx, ones), Rp[2]);
    scatter(inverse(R[2].pp), rx1);
    std::vector<i64> rx2 = x(rx1, Rn[2]);
    scatter(inverse(R[2].pn), rx2);
    // P0 (:492-547): RY2 = P(pp^-1, RY1 ^ RZp), RY3 = P(pn^-1, RY2 ^ RZn), maskRB2 = RY3 ^ maskRA (RZp)
    std::vector<i64> ry2 = x(ry1, Rp[0]);
    scatter(inverse(R[0].pp), ry2);
    std::vector<i64> ry3 = x(ry2, Rn[0]);
    scatter(inverse(R[0].pn), ry3);
    std::vector<i64> rb2 = x(ry3, Rp[0]);
    // P1 (:725-741): RX3 = P(pp^-1, RX2 ^ RZp), maskRB1 = RX3 ^ maskRC (RZn)
    std::vector<i64> rx3 = x(rx2, Rp[1]);
    scatter(inverse(R[1].pp), rx3);
    std::vector<i64> rb1 = x(rx3, Rn[1]);
    // Pi (:546, 568, 762-765, 891-894)
    Pi[0].s[1].v = Rp[0];
    Pi[0].s[0].v = x(rb1, rb2);
    Pi[1].s[0].v = Rn[1];
    Pi[1].s[1].v = x(rb1, rb2);
    Pi[2].s[0].v = Rn[2];
    Pi[2].s[1].v = Rp[2];
    return out;
}

}  // namespace orc
