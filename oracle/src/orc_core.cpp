// TEST INFRASTRUCTURE ONLY -- CPU oracle. See orc_core.h for the contract.
#include "orc_core.h"
#include <cstring>
#include <algorithm>

namespace orc {

// ---------------------------------------------------------------- ShareGen --
void ShareGen::init(const Block& prevSeed, const Block& nextSeed) {
    // Sh3ShareGen.h:9-23: mNextCommon/mPrevCommon seeded, then each stream's
    // first block becomes the AES key of one zero-share buffer.
    prev.init((const u8*)&prevSeed);
    next.init((const u8*)&nextSeed);
    Block kp = prev.getBlock();
    Block kn = next.getBlock();
    memcpy(keyBytes[0], &kp, 16);
    memcpy(keyBytes[1], &kn, 16);
    key[0].setKey(keyBytes[0]);
    key[1].setKey(keyBytes[1]);
    drawIdx = 0;
}

void ShareGen::halves(u64 j, u64& v0, u64& v1) const {
    // Sh3ShareGen.h:50-56 refills 256 blocks of AES(k, ctr) per buffer with a
    // running counter; draw j reads bytes 8j.. of the concatenated stream,
    // i.e. half (j & 1) of block j >> 1.
    Block b0 = key[0].encrypt(toBlock(j >> 1));
    Block b1 = key[1].encrypt(toBlock(j >> 1));
    v0 = (j & 1) ? b0.hi : b0.lo;
    v1 = (j & 1) ? b1.hi : b1.lo;
}

i64 ShareGen::getShare() {
    u64 v0, v1;
    halves(drawIdx++, v0, v1);
    return (i64)(v0 - v1);  // Sh3ShareGen.h:67-69
}
i64 ShareGen::getBinaryShare() {
    u64 v0, v1;
    halves(drawIdx++, v0, v1);
    return (i64)(v0 ^ v1);  // Sh3ShareGen.h:84-86
}
std::array<i64, 2> ShareGen::getRandIntShare() {
    u64 v0, v1;
    halves(drawIdx++, v0, v1);
    return {(i64)v1, (i64)v0};  // Sh3ShareGen.h:102-103
}

// ---------------------------------------------------------------- SharedOT --
std::vector<std::array<i64, 2>> SharedOT::send(const std::vector<std::array<i64, 2>>& m) {
    if (idx == ~0ull) throw std::runtime_error("SharedOT: no seed");
    std::vector<std::array<i64, 2>> msgs(m.size());
    std::vector<Block> pads(m.size());
    aes.ctr(idx, m.size(), pads.data());
    idx += m.size();
    for (size_t i = 0; i < m.size(); ++i) {
        msgs[i][0] = (i64)pads[i].lo ^ m[i][0];
        msgs[i][1] = (i64)pads[i].hi ^ m[i][1];
    }
    return msgs;
}

std::vector<i64> SharedOT::help(const std::vector<u8>& choices) {
    if (idx == ~0ull) throw std::runtime_error("SharedOT: no seed");
    // SharedOT.cpp:46-76 processes 128 counters at a time and then single
    // counters; either way pad i uses counter idx + i.
    std::vector<Block> pads(choices.size());
    aes.ctr(idx, choices.size(), pads.data());
    idx += choices.size();
    std::vector<i64> mc(choices.size());
    for (size_t i = 0; i < choices.size(); ++i) mc[i] = (i64)(choices[i] ? pads[i].hi : pads[i].lo);
    return mc;
}

std::vector<i64> ot_recv(const std::vector<std::array<i64, 2>>& msgs, const std::vector<i64>& mc,
                         const std::vector<u8>& choices) {
    std::vector<i64> out(choices.size());
    for (size_t i = 0; i < choices.size(); ++i) out[i] = msgs[i][choices[i]] ^ mc[i];
    return out;
}

void Party::initEvaluator(int pIdx, const Block& prevSeed, const Block& nextSeed) {
    idx = pIdx;
    gen.init(prevSeed, nextSeed);
    otPrev.setSeed(gen.next.getBlock());  // Sh3Evaluator.cpp:13
    otNext.setSeed(gen.prev.getBlock());  // Sh3Evaluator.cpp:14
}
void Party::initEncryptor(int pIdx, const Block& prevSeed, const Block& nextSeed) {
    idx = pIdx;
    gen.init(prevSeed, nextSeed);
}

std::array<Party, 3> makeEvaluators(u64 c) {
    std::array<Party, 3> p;
    for (int i = 0; i < 3; ++i) p[i].initEvaluator(i, toBlock(c, (u64)i), toBlock(c, (u64)((i + 1) % 3)));
    return p;
}
std::array<Party, 3> makeEncryptors(u64 c) {
    std::array<Party, 3> p;
    for (int i = 0; i < 3; ++i) p[i].initEncryptor(i, toBlock(c, (u64)i), toBlock(c, (u64)((i + 1) % 3)));
    return p;
}

// --------------------------------------------------------------- Encryptor --
static void reshareRing(Shared& x) {
    // P_i sends share 0 to next; share 1 <- prev (e.g. Sh3Encryptor.cpp:242-243)
    for (int i = 0; i < 3; ++i) x[i].s[1] = x[(i + 2) % 3].s[0];
}

Shared shareInt(std::array<Party, 3>& enc, int owner, const Mat& m) {
    Shared x;
    for (int i = 0; i < 3; ++i) {
        x[i] = SMat(m.rows, m.cols);
        for (u64 k = 0; k < m.size(); ++k)
            x[i].s[0].v[k] = (i64)((u64)enc[i].gen.getShare() + (i == owner ? (u64)m.v[k] : 0));
    }
    reshareRing(x);
    return x;
}

Shared shareBin(std::array<Party, 3>& enc, int owner, const Mat& m) {
    Shared x;
    for (int i = 0; i < 3; ++i) {
        x[i] = SMat(m.rows, m.cols);
        for (u64 k = 0; k < m.size(); ++k)
            x[i].s[0].v[k] = enc[i].gen.getBinaryShare() ^ (i == owner ? m.v[k] : 0);
    }
    reshareRing(x);
    return x;
}

Mat revealInt(const Shared& x) {
    Mat r(x[0].rows(), x[0].cols());
    for (u64 k = 0; k < r.size(); ++k)
        r.v[k] = (i64)((u64)x[0].s[0].v[k] + (u64)x[1].s[0].v[k] + (u64)x[2].s[0].v[k]);
    return r;
}
Mat revealBin(const Shared& x) {
    Mat r(x[0].rows(), x[0].cols());
    for (u64 k = 0; k < r.size(); ++k) r.v[k] = x[0].s[0].v[k] ^ x[1].s[0].v[k] ^ x[2].s[0].v[k];
    return r;
}
bool consistent(const Shared& x) {
    for (int i = 0; i < 3; ++i)
        if (x[i].s[1].v != x[(i + 2) % 3].s[0].v) return false;
    return true;
}

// -------------------------------------------------------------- Arithmetic --
// Eigen 3.3.4 has no 64-bit integer packet ops under -mavx2, so its i64 GEBP
// is scalar; keep this kernel scalar too so the CPU baseline is faithful.
__attribute__((optimize("no-tree-vectorize"))) static void gemmAcc(const i64* A, const i64* B, u64* C, u64 M,
                                                                     u64 K, u64 N) {
    const u64 KB = 256, NB = 512;
    for (u64 k0 = 0; k0 < K; k0 += KB)
        for (u64 j0 = 0; j0 < N; j0 += NB) {
            u64 k1 = std::min(K, k0 + KB), j1 = std::min(N, j0 + NB);
            for (u64 i = 0; i < M; ++i) {
                u64* c = C + i * N;
                for (u64 k = k0; k < k1; ++k) {
                    u64 a = (u64)A[i * K + k];
                    const i64* b = B + k * N;
                    for (u64 j = j0; j < j1; ++j) c[j] += a * (u64)b[j];
                }
            }
        }
}

void localProduct(MulMode mode, const SMat& A, const SMat& B, Mat& C0) {
    if (mode == MUL_HADAMARD) {
        if (A.rows() != B.rows() || A.cols() != B.cols()) throw std::runtime_error("hadamard shape");
        C0 = Mat(A.rows(), A.cols());
        for (u64 i = 0; i < C0.size(); ++i) {
            u64 a0 = A.s[0].v[i], a1 = A.s[1].v[i], b0 = B.s[0].v[i], b1 = B.s[1].v[i];
            C0.v[i] = (i64)(a0 * b0 + a0 * b1 + a1 * b0);
        }
    } else {
        if (A.cols() != B.rows()) throw std::runtime_error("gemm shape");
        u64 M = A.rows(), K = A.cols(), N = B.cols();
        C0 = Mat(M, N);
        u64* c = (u64*)C0.v.data();
        gemmAcc(A.s[0].v.data(), B.s[0].v.data(), c, M, K, N);
        gemmAcc(A.s[0].v.data(), B.s[1].v.data(), c, M, K, N);
        gemmAcc(A.s[1].v.data(), B.s[0].v.data(), c, M, K, N);
    }
}

Shared mul(std::array<Party, 3>& ev, MulMode mode, const Shared& A, const Shared& B) {
    Shared C;
    for (int i = 0; i < 3; ++i) {
        Mat c0;
        localProduct(mode, A[i], B[i], c0);
        for (u64 k = 0; k < c0.size(); ++k) c0.v[k] = (i64)((u64)c0.v[k] + (u64)ev[i].gen.getShare());
        C[i].s[0] = c0;
    }
    reshareRing(C);
    return C;
}

TruncPair truncationTuple(Party& p, u64 rows, u64 cols, u64 d) {
    // Sh3Evaluator.cpp:520-538: t0 <- next stream, t1 <- prev stream,
    // r = t0 >> 2, t0 >>= d+2, t1 >>= d+2 (arithmetic shifts on i64).
    TruncPair t;
    t.R = Mat(rows, cols);
    t.RT = SMat(rows, cols);
    p.gen.next.get(t.RT.s[0].v.data(), 8 * rows * cols);
    p.gen.prev.get(t.RT.s[1].v.data(), 8 * rows * cols);
    for (u64 i = 0; i < rows * cols; ++i) {
        i64& t0 = t.RT.s[0].v[i];
        i64& t1 = t.RT.s[1].v[i];
        t.R.v[i] = t0 >> 2;
        t0 >>= (d + 2);
        t1 >>= (d + 2);
    }
    return t;
}

void mulTruncLocal(Party& p, MulMode mode, const SMat& A, const SMat& B, u64 d, Mat& z, SMat& C) {
    localProduct(mode, A, B, z);                       // :662-668
    TruncPair t = truncationTuple(p, z.rows, z.cols, d);  // :670
    for (u64 k = 0; k < z.size(); ++k) z.v[k] = (i64)((u64)z.v[k] - (u64)t.R.v[k]);  // :672
    C = t.RT;                                          // :673
}

void truncFinalize(int pIdx, const Mat& zSum3, u64 d, SMat& C) {
    // Sh3Evaluator.cpp:712-718: C[pIdx] += (z0+z1+z2) >> d, parties 0 and 1 only
    if (pIdx >= 2) return;
    for (u64 k = 0; k < zSum3.size(); ++k)
        C.s[pIdx].v[k] = (i64)((u64)C.s[pIdx].v[k] + (u64)(zSum3.v[k] >> d));
}

Shared mulTrunc(std::array<Party, 3>& ev, MulMode mode, const Shared& A, const Shared& B, u64 d) {
    Shared C;
    std::array<Mat, 3> z;
    for (int i = 0; i < 3; ++i) mulTruncLocal(ev[i], mode, A[i], B[i], d, z[i], C[i]);
    // P0 and P1 receive the other two z's (:681-699)
    Mat s = z[0];
    for (u64 k = 0; k < s.size(); ++k) s.v[k] = (i64)((u64)z[0].v[k] + (u64)z[1].v[k] + (u64)z[2].v[k]);
    for (int i = 0; i < 2; ++i) truncFinalize(i, s, d, C[i]);
    return C;
}

Shared mulBit(std::array<Party, 3>& ev, const Shared& A, const Shared& B) {
    const u64 n = A[0].size();
    if (A[0].cols() != 1 || B[0].rows() != A[0].rows()) throw std::runtime_error("mulBit shape");
    Shared C;
    for (int i = 0; i < 3; ++i) C[i] = SMat(A[i].rows(), 1);

    // P0 (Sh3Evaluator.cpp:132-163), reading A before writing C (the
    // reference aliases A and C in Sh3Piecewise::eval -- SURVEY.md §0.3).
    std::vector<std::array<i64, 2>> s0(n);
    std::vector<u8> p0help(n);
    for (u64 i = 0; i < n; ++i) {
        u8 bb0 = (u8)((B[0].s[0].v[i] ^ B[0].s[1].v[i]) & 1);
        u8 bb1 = (u8)(B[0].s[0].v[i] & 1);
        u64 a = (u64)A[0].s[0].v[i] + (u64)A[0].s[1].v[i];
        i64 z = ev[0].gen.prev.getI64();
        i64 c0 = ev[0].gen.next.getI64();
        i64 c1 = ev[0].gen.prev.getI64();
        C[0].s[0].v[i] = c0;
        C[0].s[1].v[i] = c1;
        p0help[i] = bb1;
        u64 zz = (u64)0 - ((u64)c0 + (u64)c1) - (u64)z;
        s0[i][bb0] = (i64)zz;
        s0[i][bb0 ^ 1] = (i64)(a + zz);
    }
    auto p0send = ev[0].otNext.send(s0);
    auto p0helpMsg = ev[0].otNext.help(p0help);

    // P1 (:165-200)
    std::vector<u8> b0(n), b1(n);
    for (u64 i = 0; i < n; ++i) {
        b0[i] = (u8)(B[1].s[0].v[i] & 1);
        b1[i] = (u8)(B[1].s[1].v[i] & 1);
        C[1].s[1].v[i] = ev[1].gen.prev.getI64();
    }

    // P2 (:202-240)
    std::vector<std::array<i64, 2>> s1(n);
    std::vector<u8> p2help(n);
    for (u64 i = 0; i < n; ++i) {
        u8 bb0 = (u8)(B[2].s[1].v[i] & 1);
        u8 bb1 = (u8)((B[2].s[0].v[i] ^ B[2].s[1].v[i]) & 1);
        i64 a1 = A[2].s[1].v[i];
        i64 z = ev[2].gen.next.getI64();
        C[2].s[0].v[i] = ev[2].gen.next.getI64();
        p2help[i] = bb0;
        s1[i][bb1] = z;
        s1[i][bb1 ^ 1] = (i64)((u64)a1 + (u64)z);
    }
    auto p2helpMsg = ev[2].otPrev.help(p2help);
    auto p2send = ev[2].otPrev.send(s1);

    // P1 combines: recv0 from (sender P0, helper P2), recv1 from (sender P2, helper P0)
    auto recv0 = ot_recv(p0send, p2helpMsg, b0);
    auto recv1 = ot_recv(p2send, p0helpMsg, b1);
    for (u64 i = 0; i < n; ++i) C[1].s[0].v[i] = (i64)((u64)recv1[i] + (u64)recv0[i]);
    // P1 -> P2
    C[2].s[1] = C[1].s[0];
    return C;
}

Shared mulPubBit(std::array<Party, 3>& ev, i64 a, const Shared& B) {
    const u64 n = B[0].rows();
    Shared C;
    for (int i = 0; i < 3; ++i) C[i] = SMat(n, 1);
    // P0 (Sh3Evaluator.cpp:430-447)
    std::vector<std::array<i64, 2>> s0(n);
    for (u64 i = 0; i < n; ++i) {
        u8 bb = (u8)((B[0].s[0].v[i] ^ B[0].s[1].v[i]) & 1);
        i64 zs = ev[0].gen.getShare();
        s0[i][bb] = zs;
        s0[i][bb ^ 1] = (i64)((u64)a + (u64)zs);
    }
    auto toP1 = ev[0].otNext.send(s0);
    auto toP2 = ev[0].otPrev.send(s0);
    // P1 (:452-467)
    std::vector<u8> c1(n);
    for (u64 i = 0; i < n; ++i) {
        C[1].s[1].v[i] = ev[1].gen.getShare();
        c1[i] = (u8)(B[1].s[0].v[i] & 1);
    }
    auto p1help = ev[1].otNext.help(c1);  // to P2
    // P2 (:470-487)
    std::vector<u8> c2(n);
    for (u64 i = 0; i < n; ++i) {
        C[2].s[0].v[i] = ev[2].gen.getShare();
        c2[i] = (u8)(B[2].s[1].v[i] & 1);
    }
    auto p2help = ev[2].otPrev.help(c2);  // to P1
    auto r1 = ot_recv(toP1, p2help, c1);
    auto r2 = ot_recv(toP2, p1help, c2);
    for (u64 i = 0; i < n; ++i) {
        C[1].s[0].v[i] = r1[i];
        C[2].s[1].v[i] = r2[i];
    }
    C[0].s[0] = C[1].s[1];  // P1 -> P0
    C[0].s[1] = C[2].s[0];  // P2 -> P0
    return C;
}

// ------------------------------------------------------------------ Binary --
static inline u64 gateLocal(u32 t, u64 a, u64 b) {
    switch (t) {
        case G_XOR: return a ^ b;
        case G_NXOR: return ~(a ^ b);
        case G_COPY: return a;
        case G_INV: return ~a;
        default: throw std::runtime_error("not a local gate");
    }
}

// a[r] bit j <-> a[j] bit r (recursive block swaps, 6 x 32 steps)
static void transpose64(u64* a) {
    u64 m = 0x00000000FFFFFFFFull;
    for (int j = 32; j; j >>= 1, m ^= m << j)
        for (int k = 0; k < 64; k = ((k | j) + 1) & ~j) {
            const u64 t = ((a[k] >> j) ^ a[k | j]) & m;
            a[k] ^= t << j;
            a[k | j] ^= t;
        }
}

void evalLevel(const Circuit& cir, u64 gateBegin, u64 gateCount, u64 andBegin, std::vector<u64>& mem, u64 words,
               const std::vector<u64>& zFlat, std::vector<u64>& sendBuf) {
    // Gate formulas: Sh3BinaryEvaluator.cpp:700-1065. Gates of one level are
    // evaluated in list order; AND-type outputs only get their share 1 at
    // the start of the next level.
    const u64 W = cir.wireCount;
    u64* s0 = mem.data();
    u64* s1 = mem.data() + W * words;
    u64 andIdx = andBegin;
    sendBuf.clear();
    for (u64 g = gateBegin; g < gateBegin + gateCount; ++g) {
        const Gate& gt = cir.gates[g];
        u64* o0 = s0 + gt.out * words;
        u64* o1 = s1 + gt.out * words;
        const u64* x0 = s0 + gt.in0 * words;
        const u64* x1 = s1 + gt.in0 * words;
        const u64* y0 = s0 + gt.in1 * words;
        const u64* y1 = s1 + gt.in1 * words;
        if (!isAndType(gt.type)) {
            for (u64 w = 0; w < words; ++w) {
                o0[w] = gateLocal(gt.type, x0[w], y0[w]);
                o1[w] = gateLocal(gt.type, x1[w], y1[w]);
            }
            continue;
        }
        const u64* z = zFlat.data() + andIdx * words;
        ++andIdx;
        for (u64 w = 0; w < words; ++w) {
            u64 a0 = x0[w], a1 = x1[w], b0 = y0[w], b1 = y1[w], r;
            switch (gt.type) {
                case G_AND: r = (a0 & b0) ^ (a0 & b1) ^ (a1 & b0); break;
                case G_OR: r = (a0 & b0) ^ (a0 & b1) ^ (a1 & b0) ^ a0 ^ b0; break;
                case G_NOR: r = (~a0 & ~b0) ^ (~a0 & ~b1) ^ (~a1 & ~b0); break;
                default /*NA_AND*/: r = (~a0 & b0) ^ (~a0 & b1) ^ (~a1 & b0); break;
            }
            o0[w] = r ^ z[w];
        }
        sendBuf.insert(sendBuf.end(), o0, o0 + words);
    }
}

std::vector<Shared> evalCircuit(std::array<Party, 3>& ev, const Circuit& cir,
                                const std::vector<const Shared*>& inputs) {
    if (inputs.size() != cir.inputs.size()) throw std::runtime_error("input bundle count");
    const u64 rows = (*inputs[0])[0].rows();
    const u64 words = paddedWords(rows);
    const u64 W = cir.wireCount;

    u64 nAnd = 0;
    for (auto& g : cir.gates) nAnd += isAndType(g.type);

    std::array<std::vector<u64>, 3> mem, z;
    for (int p = 0; p < 3; ++p) {
        // setCir (Sh3BinaryEvaluator.h:96-102, .cpp:87-88)
        Block kp = ev[p].gen.prev.getBlock();
        Block kn = ev[p].gen.next.getBlock();
        AesNI ap, an;
        ap.setKey((const u8*)&kp);
        an.setKey((const u8*)&kn);
        // getShares (:1406-1440): gate k uses counters [k*words/2, (k+1)*words/2)
        z[p].resize(nAnd * words);
        std::vector<Block> bp(nAnd * words / 2), bn(nAnd * words / 2);
        ap.ctr(0, bp.size(), bp.data());
        an.ctr(0, bn.size(), bn.data());
        for (u64 i = 0; i < bp.size(); ++i) {
            z[p][2 * i] = bp[i].lo ^ bn[i].lo;
            z[p][2 * i + 1] = bp[i].hi ^ bn[i].hi;
        }
        // setInput (:200-276): transpose rows x bits -> wire-major, zero pad;
        // 64 x 64 bit blocks (as cryptoTools' transpose does it)
        mem[p].assign(2 * W * words, 0);
        for (size_t b = 0; b < cir.inputs.size(); ++b) {
            const SMat& in = (*inputs[b])[p];
            const auto& wires = cir.inputs[b];
            if (in.rows() != rows) throw std::runtime_error("input rows");
            if (in.cols() * 64 < wires.size()) throw std::runtime_error("input bits");
            for (int s = 0; s < 2; ++s)
                for (u64 rb = 0; rb * 64 < rows; ++rb)
                    for (size_t c = 0; c * 64 < wires.size(); ++c) {
                        u64 blk[64];
                        for (u64 r = 0; r < 64; ++r)
                            blk[r] = rb * 64 + r < rows ? (u64)in.s[s].v[(rb * 64 + r) * in.cols() + c] : 0;
                        transpose64(blk);
                        for (size_t j = 0; j < 64 && c * 64 + j < wires.size(); ++j)
                            mem[p][(s * W + wires[c * 64 + j]) * words + rb] = blk[j];
                    }
        }
    }

    u64 gateBegin = 0, andBegin = 0;
    for (u32 cnt : cir.levelCounts) {
        std::array<std::vector<u64>, 3> sends;
        u64 levelAnds = 0;
        for (u64 g = gateBegin; g < gateBegin + cnt; ++g) levelAnds += isAndType(cir.gates[g].type);
        for (int p = 0; p < 3; ++p) evalLevel(cir, gateBegin, cnt, andBegin, mem[p], words, z[p], sends[p]);
        // message to next: share 1 of each AND-type output <- prev's share 0 (:555-573)
        for (int p = 0; p < 3; ++p) {
            const auto& recv = sends[(p + 2) % 3];
            u64 j = 0;
            for (u64 g = gateBegin; g < gateBegin + cnt; ++g) {
                if (!isAndType(cir.gates[g].type)) continue;
                std::copy(recv.begin() + j * words, recv.begin() + (j + 1) * words,
                          mem[p].begin() + (W + cir.gates[g].out) * words);
                ++j;
            }
        }
        gateBegin += cnt;
        andBegin += levelAnds;
    }
    if (gateBegin != cir.gates.size()) throw std::runtime_error("levelCounts do not cover gates");

    // getOutput (:1285-1404): transpose back
    std::vector<Shared> outs(cir.outputs.size());
    for (size_t o = 0; o < cir.outputs.size(); ++o) {
        const auto& wires = cir.outputs[o];
        u64 cols = (wires.size() + 63) / 64;
        for (int p = 0; p < 3; ++p) {
            outs[o][p] = SMat(rows, cols);
            for (int s = 0; s < 2; ++s)
                for (u64 rb = 0; rb * 64 < rows; ++rb)
                    for (u64 c = 0; c < cols; ++c) {
                        u64 blk[64];
                        for (u64 j = 0; j < 64; ++j)
                            blk[j] = c * 64 + j < wires.size() ? mem[p][(s * W + wires[c * 64 + j]) * words + rb] : 0;
                        transpose64(blk);
                        for (u64 r = 0; r < 64 && rb * 64 + r < rows; ++r)
                            outs[o][p].s[s].v[(rb * 64 + r) * cols + c] = (i64)blk[r];
                    }
        }
    }
    return outs;
}

// --------------------------------------------------------------- Piecewise --
i64 Coef::fixed(u64 D) const {
    // Sh3Piecewise.h:55-61
    if (isInt) return (i64)((u64)i * (1ull << D));
    return (i64)(d * (double)(1ull << D));
}

// P0 reshares x0+x2 as a binary sharing (x0+x2, 0, 0) and P1/P2 expose x1 as
// (0, x1, 0) (Sh3Piecewise.cpp:392-458, BuildingBlocks.cpp:475-502).
static void twoInputSharing(const Shared& x, Shared& c0, Shared& c1) {
    const u64 rows = x[0].rows(), cols = x[0].cols();
    for (int p = 0; p < 3; ++p) {
        c0[p] = SMat(rows, cols);
        c1[p] = SMat(rows, cols);
    }
    for (u64 k = 0; k < x[0].size(); ++k) c0[0].s[0].v[k] = (i64)((u64)x[0].s[0].v[k] + (u64)x[0].s[1].v[k]);
    c1[1].s[0] = x[1].s[0];
    c1[2].s[1] = x[2].s[1];
    reshareRing(c0);
}

Shared fetchMsb(std::array<Party, 3>& ev, const Circuit& msbCir, const Shared& diff) {
    Shared c0, c1;
    twoInputSharing(diff, c0, c1);
    auto out = evalCircuit(ev, msbCir, {&c0, &c1});
    return out[0];
}

Shared boolNot(const Shared& x) {
    Shared r = x;
    for (auto& v : r[1].s[0].v) v = ~v;
    for (auto& v : r[2].s[1].v) v = ~v;
    return r;
}

Shared piecewiseEval(std::array<Party, 3>& ev, const Piecewise& pw, const Circuit& helper, const Shared& x, u64 D) {
    const u64 T = pw.thresholds.size();
    const u64 n = x[0].size();
    if (pw.coefs.size() != T + 1) throw std::runtime_error("piecewise coefs");
    // getInputRegions (Sh3Piecewise.cpp:381-516)
    Shared c0, c1;
    twoInputSharing(x, c0, c1);
    std::vector<Shared> a(T, c0);
    for (u64 t = 0; t < T; ++t) {
        i64 thr = pw.thresholds[t].fixed(D);
        for (int p = 0; p < 2; ++p)
            for (auto& v : a[t][p].s[p].v) v = (i64)((u64)v - (u64)thr);
    }
    std::vector<const Shared*> ins;
    for (u64 t = 0; t < T; ++t) ins.push_back(&a[t]);
    ins.push_back(&c1);
    auto regions = evalCircuit(ev, helper, ins);

    // getFunctionValues (:518-567) and the region products (:284-330)
    Shared out;
    for (int p = 0; p < 3; ++p) out[p] = SMat(x[0].rows(), x[0].cols());
    for (u64 c = 0; c < pw.coefs.size(); ++c) {
        const auto& co = pw.coefs[c];
        if (co.empty()) continue;
        Shared f;
        if (co.size() > 1) {
            if (!co[1].isInt) throw std::runtime_error("piecewise: non-integer slope not implemented");
            i64 cst = co[0].fixed(D);
            for (int p = 0; p < 3; ++p) {
                f[p] = SMat(x[0].rows(), x[0].cols());
                for (int s = 0; s < 2; ++s)
                    for (u64 k = 0; k < n; ++k) f[p].s[s].v[k] = (i64)((u64)co[1].i * (u64)x[p].s[s].v[k]);
                if (cst && p < 2)
                    for (auto& v : f[p].s[p].v) v = (i64)((u64)v + (u64)cst);
            }
            f = mulBit(ev, f, regions[c]);
        } else {
            f = mulPubBit(ev, co[0].fixed(D), regions[c]);
        }
        for (int p = 0; p < 3; ++p)
            for (int s = 0; s < 2; ++s)
                for (u64 k = 0; k < n; ++k) out[p].s[s].v[k] = (i64)((u64)out[p].s[s].v[k] + (u64)f[p].s[s].v[k]);
    }
    return out;
}

i64 fixedMulPlain(i64 a, i64 b, u64 D) {
    __int128 v = (__int128)a * (__int128)b;
    v = v / (__int128)(1ull << D);  // truncates toward zero like boost int128 division
    return (i64)v;
}

}  // namespace orc

// ---------------------------------------------------------------------------
// Sh3Converter (aby3/sh3/Sh3Converter.cpp)
// ---------------------------------------------------------------------------
namespace orc {

std::array<ConvParty, 3> converterInit(std::array<Party, 3>& ev) {
    std::array<ConvParty, 3> cv;
    cv[0].ot02.setSeed(ev[0].gen.prev.getBlock());  // Sh3Converter.h:31-32
    cv[1].ot12.setSeed(ev[1].gen.next.getBlock());  // :33-34
    cv[2].ot12.setSeed(ev[2].gen.prev.getBlock());  // :35-39
    cv[2].ot02.setSeed(ev[2].gen.next.getBlock());
    return cv;
}

static inline u8 bitAt(const Mat& m, u64 row, u64 bit) {
    return (u8)(((u64)m(row, bit / 64) >> (bit % 64)) & 1);
}

SMat toPackedBin(const SMat& in, u64 bitCount) {
    const u64 rows = in.rows(), simd = (rows + 63) / 64;
    SMat out(bitCount, simd);
    for (int s = 0; s < 2; ++s)
        for (u64 i = 0; i < rows; ++i)
            for (u64 j = 0; j < bitCount; ++j)
                if (bitAt(in.s[s], i, j)) out.s[s](j, i / 64) |= (i64)(1ull << (i % 64));
    return out;
}

SMat fromPackedBin(const SMat& packed, u64 shareCount, u64 bitCount) {
    SMat out(shareCount, (bitCount + 63) / 64);
    for (int s = 0; s < 2; ++s)
        for (u64 j = 0; j < bitCount; ++j)
            for (u64 i = 0; i < shareCount; ++i)
                if (bitAt(packed.s[s], j, i)) out.s[s](i, j / 64) |= (i64)(1ull << (j % 64));
    return out;
}

Shared toBinaryMatrix(std::array<Party, 3>& ev, const Circuit& addCir, const Shared& x, u64 bitCount) {
    const u64 rows = x[0].rows(), cols64 = (bitCount + 63) / 64;
    if (cols64 != x[0].cols()) throw std::runtime_error("toBinaryMatrix: ceil(bitCount/64) != in.cols()");
    const u64 n = rows * cols64;
    const u64 mask = bitCount % 64 ? (1ull << (bitCount % 64)) - 1 : ~0ull;
    auto m = [&](u64 e) { return e % cols64 == cols64 - 1 ? mask : ~0ull; };
    Shared c0, c1;
    for (int p = 0; p < 3; ++p) {
        c0[p] = SMat(rows, cols64);
        c1[p] = SMat(rows, cols64);
    }
    // P0 (:90-93) and P2 (:179-182) draw one stream word per element; the
    // PRNG buffers whole blocks, so draw them in one call
    std::vector<i64> r0(n), r2(n);
    ev[0].gen.prev.get(r0.data(), 8 * n);
    ev[2].gen.next.get(r2.data(), 8 * n);
    for (u64 e = 0; e < n; ++e) {
        // P0 (:90-106): r = prev stream word, x0 = ((in0 + in1) ^ r, r)
        const u64 r = (u64)r0[e];
        c0[0].s[1].v[e] = (i64)(r & m(e));
        c0[0].s[0].v[e] = (i64)((((u64)x[0].s[0].v[e] + (u64)x[0].s[1].v[e]) ^ r) & m(e));
    }
    for (u64 e = 0; e < n; ++e) {
        // P2 (:179-194): x0 = (r, 0) with the same words, x1 = (0, in1)
        c0[2].s[0].v[e] = (i64)((u64)r2[e] & m(e));
        c1[2].s[1].v[e] = (i64)((u64)x[2].s[1].v[e] & m(e));
        // P1 (:132-147): x0 = (0, P0's message), x1 = (in0, 0)
        c1[1].s[0].v[e] = (i64)((u64)x[1].s[0].v[e] & m(e));
    }
    c0[1].s[1] = c0[0].s[0];  // P0 -> P1 (:108, :149)
    auto out = evalCircuit(ev, addCir, {&c0, &c1});
    return out[0];
}

Shared bitInjection(std::array<Party, 3>& ev, std::array<ConvParty, 3>& cv, const Shared& b, u64 bitCount,
                    bool twoRounds) {
    const u64 rows = b[0].rows(), n = rows * bitCount;
    auto choices = [&](const Mat& m) {  // BitVector::append per row (:241-247)
        std::vector<u8> c(n);
        for (u64 i = 0, k = 0; i < rows; ++i)
            for (u64 j = 0; j < bitCount; ++j, ++k) c[k] = bitAt(m, i, j);
        return c;
    };
    Shared d;
    for (int p = 0; p < 3; ++p) d[p] = SMat(rows, bitCount);
    // P2, sender (:319-363)
    std::vector<std::array<i64, 2>> m(n);
    {
        ev[2].gen.next.get(d[2].s[0].v.data(), 8 * n);  // mNextCommon.get(dest0) (:325)
        ev[2].gen.prev.get(d[2].s[1].v.data(), 8 * n);  // mPrevCommon.get(dest1) (:326)
        auto c0 = choices(b[2].s[0]), c1 = choices(b[2].s[1]);
        for (u64 k = 0; k < n; ++k) {
            const u8 bb = c0[k] ^ c1[k];
            m[k][0] = m[k][1] = (i64)(0 - (u64)d[2].s[0].v[k] - (u64)d[2].s[1].v[k]);
            m[k][bb ^ 1] = (i64)((u64)m[k][bb ^ 1] + 1);
        }
    }
    auto msgsTo0 = cv[2].ot12.send(m);                         // P2 -> P0
    std::vector<std::array<i64, 2>> msgsTo1;
    if (!twoRounds) msgsTo1 = cv[2].ot02.send(m);               // P2 -> P1
    const auto ch0 = choices(b[0].s[0]), ch1 = choices(b[1].s[1]);  // P0's and P1's copy of share 0
    auto help1 = cv[1].ot12.help(ch1);                          // P1 -> P0 (:290)
    ev[1].gen.next.get(d[1].s[0].v.data(), 8 * n);  // :291
    std::vector<i64> help0;
    if (!twoRounds) help0 = cv[0].ot02.help(ch0);                // P0 -> P1 (:269)
    ev[0].gen.prev.get(d[0].s[1].v.data(), 8 * n);  // :274
    d[0].s[0].v = ot_recv(msgsTo0, help1, ch0);                 // :255-258
    if (twoRounds)
        d[1].s[1] = d[0].s[0];                                  // :262, :312
    else
        d[1].s[1].v = ot_recv(msgsTo1, help0, ch1);             // :303-306
    return d;
}

}  // namespace orc
