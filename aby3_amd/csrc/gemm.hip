// Share product of Sh3Evaluator::asyncMul on gfx950.
//
// GEMM mode (upstream semantics, Sh3Evaluator.cpp:96-99 / 662-665):
//   C0 = A0 B0 + A0 B1 + A1 B0 = [A0 | A1] . [[B0 + B1]; [B0]]   (mod 2^64)
// CDNA4 has no 64-bit integer MFMA, so every 64-bit operand is split into 8
// balanced base-256 digits d_p in [-128, 127] (x = sum_p d_p 2^(8p) mod 2^64)
// and the product mod 2^64 is
//   sum_{s=0..7} 2^(8s) * sum_{p+q=s} A_p . B_q
// i.e. 36 int8 digit-pair GEMMs accumulated into 8 exact i32 planes
// (|plane| <= 8 * K' * 2^14 < 2^31 for K' <= 8192 per split) and recombined
// in i64 in the epilogue. MFMA: v_mfma_i32_16x16x64_i8 (k_share_gemm16s), a
// 128 x 64 output tile per 512-thread workgroup, each wave a 32 x 32 tile of
// 2 x 2 16x16 blocks with 8 planes (128 accumulator VGPRs).
//
// Digit layout in HBM (built once per call by k_digits_*): for every row of
// A (resp. column of B) and every 32-wide slice of K', the 8 planes x 32
// digits are one contiguous 256-byte record, so a K-stage of a 64-row tile is
// 64 contiguous-per-row 256 B records. In LDS a record's 16-byte chunk g of
// row r is stored at slot g ^ (r & 15): the 16 lanes of each ds_read_b128
// lane group read 16 different rows at the same chunk and land on 16
// different bank slots.
#include <atomic>
#include <map>
#include <mutex>
#include "epilogue.h"

#ifndef ABY3G_TILE_GROUP
#define ABY3G_TILE_GROUP 4  // row panels per tile group (tile_of)
#endif
namespace aby3g {

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr u32 BN = 64, BK = 32;  // output tile width, K' per stage
constexpr u32 kRec = 256;        // bytes per (row, stage) record

constexpr u32 TBM = 128;  // output tile height (8 waves of 32 x 32)
// Share GEMMs of this many parties run side by side on the calling thread's
// device (aby3g_set_gemm_sharing): split-K fills 1/k of the CUs per GEMM.
thread_local u32 t_gemm_sharing = 1;
inline u32 gemm_target_wgs() { return 256u / t_gemm_sharing; }

inline u64 roundup(u64 x, u64 m) { return (x + m - 1) / m * m; }

// GEMMs up to this many product terms run on the VALU (k_small_gemm), with
// no digit split and no MFMA; the epilogue then works in place on the product.
constexpr u64 kSmallGemmTerms = 1ull << 23;
inline bool small_gemm(u64 M, u64 K, u64 N) { return M * N * K <= kSmallGemmTerms; }

// C0-part of the share product, out = [A0 | A1] . [[B0 + B1]; [B0]] mod 2^64,
// one wave per output element: the lanes split the K terms and a butterfly
// sums them, so an element costs K / 64 dependent load rounds, not K (the
// small GEMMs of an LR iteration have 128-256 outputs of 128-256 terms).
__global__ void __launch_bounds__(256) k_small_gemm(const i64* __restrict__ A0, const i64* __restrict__ A1,
                                                    const i64* __restrict__ B0, const i64* __restrict__ B1, u64 M,
                                                    u64 K, u64 N, i64* __restrict__ out) {
    const u32 lane = threadIdx.x & 63;
    const u64 n = M * N, waves = (u64)gridDim.x * (blockDim.x >> 6);
    for (u64 i = (u64)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < n; i += waves) {
        const u64 m = i / N, c = i % N;
        const i64* a0 = A0 + m * K;
        const i64* a1 = A1 + m * K;
        u64 acc = 0;
        for (u64 k = lane; k < K; k += 64) {
            const u64 b0 = (u64)B0[k * N + c], b1 = (u64)B1[k * N + c];
            acc += (u64)a0[k] * (b0 + b1) + (u64)a1[k] * b0;
        }
#pragma unroll
        for (int o = 32; o; o >>= 1) acc += __shfl_xor(acc, o, 64);
        if (lane == 0) out[i] = (i64)acc;
    }
}

void run_small_gemm(const i64* A, const i64* B, u64 M, u64 K, u64 N, i64* out, hipStream_t s) {
    const u64 n = M * N;
    const u32 grid = (u32)std::min<u64>((n + 3) / 4, 2048);
    launch(PROBE_EPILOGUE, k_small_gemm, dim3(grid), dim3(256), 0, s, A, A + M * K, B, B + K * N, M, K, N, out);
}

struct GemmPlan {
    u64 M, K, N;
    u32 tbm;             // tile height (64 or 128)
    u64 Mp, Np, Kp, Kc;  // padded sizes; Kc = K' = 2*Kp
    u32 splits;          // split-K factor
    u64 kPerSplit;       // K' per split (multiple of BK)
    size_t aBytes, bBytes, pBytes, total;
};

GemmPlan plan_gemm(u64 M, u64 K, u64 N) {
    GemmPlan p;
    p.M = M;
    p.K = K;
    p.N = N;
    p.tbm = TBM;
    p.Mp = roundup(M ? M : 1, p.tbm);
    p.Np = roundup(N ? N : 1, BN);
    p.Kp = roundup(K ? K : 1, 32);  // each half of K' a whole number of stages
    p.Kc = 2 * p.Kp;
    const u64 stages = p.Kc / BK;
    const u64 tiles = (p.Mp / p.tbm) * (p.Np / BN);
    // Enough workgroups for one per CU, at least 8 stages per split, and
    // K' per split <= 8192 so every i32 plane stays exact.
    u32 s = 1;
    while (tiles * s < gemm_target_wgs() && stages / (2 * s) >= 8) s *= 2;
    while ((stages + s - 1) / s * BK > 8192) s *= 2;
    p.splits = s;
    p.kPerSplit = (stages + s - 1) / s * BK;
    p.aBytes = p.Mp * p.Kc * 8;
    p.bBytes = p.Np * p.Kc * 8;
    p.pBytes = (u64)s * M * N * 8;
    p.total = roundup(p.aBytes, 256) + roundup(p.bBytes, 256) + roundup(p.pBytes, 256);
    return p;
}

// Balanced base-256 digits. With y = x + 0x8080...80 (mod 2^64), byte p of
// y is b_p + 128 + carry_p (mod 256) and the carry out of byte p is exactly
// the balanced-digit borrow, so digit p = byte p of y minus 128, i.e. the
// int8 whose bits are (byte p of y) ^ 0x80:  x = sum_p d_p 2^(8p) mod 2^64.
constexpr u64 kDigitBias = 0x8080808080808080ull;

// One launch builds both digit operands. K' = [first half | second half]
// with Kp (a multiple of 32) per half, so a 32-wide slice st of the original K
// yields record stage st of the first half and st + Kp/32 of the second:
//   A-workgroup: 32 rows x 32 k of A0 and A1 -> 64 records
//   B-workgroup: 32 k x 64 columns of B0, B1 -> 128 records (B0 + B1, B0)
// so every input element is read once. A thread holds 4 consecutive k of one
// row / column, forms the 8 digit-plane words of those 4 values with 16
// v_perm_b32 (a 4 x 8 byte transpose), and writes them into the record image
// in LDS (272-byte pitch: a ds_write_b32 pass of 32 lanes hits 32 banks on
// the A side, 2-way on the B side); the images then leave as 16-byte chunks,
// 16 lanes per 256-byte record.
constexpr u32 kDigitPitch = 272;  // LDS bytes per record image (256 + 16)
constexpr u32 kDigitRows = 32;    // A rows per A-workgroup
constexpr u32 kDigitCols = 64;    // B columns per B-workgroup (the widest form)
static_assert(BN % kDigitCols == 0, "padded columns are whole B-workgroups");

// digit-plane words of 4 values: word p = digit p of v0..v3, one byte each
__device__ __forceinline__ void digit_words(const u64 (&v)[4], u32 (&w)[8]) {
    u32 lo[4], hi[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const u64 y = v[i] + kDigitBias;
        lo[i] = (u32)y;
        hi[i] = (u32)(y >> 32);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const u32* q = h ? hi : lo;
        const u32 t0 = __builtin_amdgcn_perm(q[1], q[0], 0x05010400u), t1 = __builtin_amdgcn_perm(q[1], q[0], 0x07030602u);
        const u32 u0 = __builtin_amdgcn_perm(q[3], q[2], 0x05010400u), u1 = __builtin_amdgcn_perm(q[3], q[2], 0x07030602u);
        w[4 * h + 0] = __builtin_amdgcn_perm(u0, t0, 0x05040100u) ^ 0x80808080u;
        w[4 * h + 1] = __builtin_amdgcn_perm(u0, t0, 0x07060302u) ^ 0x80808080u;
        w[4 * h + 2] = __builtin_amdgcn_perm(u1, t1, 0x05040100u) ^ 0x80808080u;
        w[4 * h + 3] = __builtin_amdgcn_perm(u1, t1, 0x07060302u) ^ 0x80808080u;
    }
}

// One digit group: an A-group (32 rows x 32 k of A0, A1) or a B-group (32 k x
// 64 columns of B0, B1) -> its records. t in [0, 256); img: 2 * 64 record
// images. Every thread of the workgroup reaches the one barrier inside, also
// when `valid` is false.
template <u32 COLS>
__device__ __forceinline__ void digit_group(bool valid, u64 gid, u32 t, u8* img, const i64* __restrict__ A0,
                                            const i64* __restrict__ A1, const i64* __restrict__ B0,
                                            const i64* __restrict__ B1, u64 M, u64 K, u64 N, u64 S2, u64 aGroups,
                                            u64 stages, u8* __restrict__ Ad, u8* __restrict__ Bd) {
    const bool isA = gid < aGroups;
    const u64 g = isA ? gid : gid - aGroups;
    const u64 st = g % S2, k0 = st * 32;
    u32 nrec;
    u8* out;
    u64 r0;
    if (isA) {
        // record (row, half) at image index 2 * row + half
        r0 = (g / S2) * kDigitRows;
        const u32 row = t >> 3, kq = t & 7;
        const u64 m = r0 + row;
        u64 v0[4], v1[4];
        const u64 kk = k0 + 4 * kq;
        if (valid && m < M && kk + 4 <= K && K % 2 == 0 && (((u64)A0 | (u64)A1) & 15) == 0) {
            // the row's 4 values as two 16-byte loads per share
            typedef u64 u64v2 __attribute__((ext_vector_type(2)));
            const u64v2* p0 = reinterpret_cast<const u64v2*>(A0 + m * K + kk);
            const u64v2* p1 = reinterpret_cast<const u64v2*>(A1 + m * K + kk);
            const u64v2 a0 = p0[0], a1 = p0[1], b0 = p1[0], b1 = p1[1];
            v0[0] = a0.x, v0[1] = a0.y, v0[2] = a1.x, v0[3] = a1.y;
            v1[0] = b0.x, v1[1] = b0.y, v1[2] = b1.x, v1[3] = b1.y;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const u64 k = kk + j;
                const bool in = valid && m < M && k < K;
                v0[j] = in ? (u64)A0[m * K + k] : 0;
                v1[j] = in ? (u64)A1[m * K + k] : 0;
            }
        }
        u32 w0[8], w1[8];
        digit_words(v0, w0);
        digit_words(v1, w1);
        u32* i0 = reinterpret_cast<u32*>(img + (2 * row) * kDigitPitch) + kq;
        u32* i1 = reinterpret_cast<u32*>(img + (2 * row + 1) * kDigitPitch) + kq;
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            i0[8 * p] = w0[p];
            i1[8 * p] = w1[p];
        }
        nrec = 2 * kDigitRows;
        out = Ad;
    } else {
        // record (column, half) at image index half * COLS + column
        r0 = (g / S2) * COLS;
        const u32 col = t & (COLS - 1);
        const u64 n = r0 + col;
#pragma unroll
        for (u32 e = 0; e < 8 * COLS / 256; ++e) {
            const u32 kq = t / COLS + (256 / COLS) * e;
            u64 vs[4], vb[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const u64 k = k0 + 4 * kq + j;
                const bool in = valid && n < N && k < K;
                const u64 b0 = in ? (u64)B0[k * N + n] : 0, b1 = in ? (u64)B1[k * N + n] : 0;
                vs[j] = b0 + b1;
                vb[j] = b0;
            }
            u32 ws[8], wb[8];
            digit_words(vs, ws);
            digit_words(vb, wb);
            u32* i0 = reinterpret_cast<u32*>(img + col * kDigitPitch) + kq;
            u32* i1 = reinterpret_cast<u32*>(img + (COLS + col) * kDigitPitch) + kq;
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                i0[8 * p] = ws[p];
                i1[8 * p] = wb[p];
            }
        }
        nrec = 2 * COLS;
        out = Bd;
    }
    __syncthreads();
    if (!valid) return;
    // 16 chunks of 16 B per record; record (r, half) -> stage st + half * S2 of row / column r0 + r
    for (u32 c = t; c < nrec * 16; c += 256) {
        const u32 rec = c >> 4, ch = c & 15;
        const u32 rr = isA ? rec >> 1 : rec & (COLS - 1), half = isA ? rec & 1 : rec / COLS;
        const u64 r = r0 + rr, stg = st + half * S2;
        const v4i x = *reinterpret_cast<const v4i*>(img + rec * kDigitPitch + ch * 16);
        *reinterpret_cast<v4i*>(out + (r * stages + stg) * kRec + ch * 16) = x;
    }
}

// COLS = 32: 64 records per group on both sides (17 KiB of LDS, twice the
// workgroups resident per CU of the 64-column form)
template <u32 COLS>
__global__ void __launch_bounds__(256) k_digits(const i64* __restrict__ A0, const i64* __restrict__ A1,
                                                const i64* __restrict__ B0, const i64* __restrict__ B1, u64 M,
                                                u64 K, u64 N, u64 S2, u64 aGroups, u64 stages, u8* __restrict__ Ad,
                                                u8* __restrict__ Bd) {
    constexpr u32 kRecs = 2 * (COLS > kDigitRows ? COLS : kDigitRows);
    __shared__ __attribute__((aligned(16))) u8 img[kRecs * kDigitPitch];  // record images
    digit_group<COLS>(true, blockIdx.x, threadIdx.x, img, A0, A1, B0, B1, M, K, N, S2, aGroups, stages, Ad, Bd);
}

// B-workgroups of 32 columns: 64 records per group on both sides (17 KiB of
// LDS; measured ahead of 64-column groups at half the occupancy, round 4)
constexpr u32 kBGroupCols = 32;

// XCD-aware tile order. Workgroup ids are dealt round-robin to the 8 XCDs
// (id % 8), each with its own 4 MiB L2. Remap so every XCD gets one
// contiguous range of the tile order, and order tiles split-major, then in
// groups of 4 row-panels, column-major within a group: an XCD's 32 tiles at
// 1024^3 (split-K 2) are then 4 row x 8 column panels, 8 MB of digit panels
// instead of 10 MB for 8 x 4 (equal time measured; less fabric traffic).
struct TileCoord {
    u32 tm, tn, split;
};
__device__ __forceinline__ u32 tile_group() { return ABY3G_TILE_GROUP; }
__device__ __forceinline__ TileCoord tile_of(u32 pid, u32 TM, u32 TN, u32 splits) {
    const u32 T = TM * TN * splits;
    const u32 per = (T + 7) / 8;
    const u32 xcd = pid % 8, idx = pid / 8;
    // a bijection when T is a multiple of 8; otherwise keep the launch order
    const u32 np = (per * 8 == T) ? xcd * per + idx : pid;
    const u32 tilesPerSplit = TM * TN;
    TileCoord c;
    c.split = np / tilesPerSplit;
    const u32 rem = np % tilesPerSplit;
    const u32 G = tile_group();
    const u32 group = rem / (G * TN), first = group * G;
    const u32 gm = min(G, TM - first);
    const u32 inGroup = rem % (G * TN);
    c.tm = first + inGroup % gm;
    c.tn = inGroup / gm;
    return c;
}

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

// k_share_gemm16s: one 128 x 64 output tile over the K' stages of its split,
// v_mfma_i32_16x16x64_i8, which sustains ~1.5x the int8 rate of the 32x32x32
// form on gfx950 with random operands (scripts/mfma_peak.hip: 87 % vs 56 % of
// the spec peak). Each wave's 32 x 32 tile is 2 x 2 16x16 blocks. One MFMA
// sums TWO digit pairs of the same plane s over a 32-wide K' slice: its
// 64-deep K is [plane P1 | plane P2] of the stage (lanes 0-31 read plane P1,
// lanes 32-63 plane P2, each lane its 16-byte chunk of the record), so
// A-pair e = planes (2e, 2e+1) times B-pair f = planes (f, f-1) adds
// A_2e B_f + A_2e+1 B_f-1 into plane 2e + f. B-pair "0Z" is plane 0 with a
// zero upper half, for the odd pair (A_s, B_0) of an even plane s. 20 MFMAs
// per block and stage cover the 36 digit pairs (4 of them half-used).
//
// The two waves of each SIMD run half a stage apart. Waves 0-3 ("X") and 4-7
// ("Y") alternate between a read phase (this stage's 24 fragments from LDS,
// and 6 DMA pieces of the stage two ahead) and an MFMA phase (80 MFMAs),
// separated by raw barriers; Y starts one phase late, so in every phase one
// wave of each SIMD feeds the MFMA pipe while the other reads: the LDS reads
// and DMA issue hide behind the other wave's MFMAs instead of stalling both.
// 3-deep ring (144 KiB):
//   X: phase 2s = read s + DMA s+2, phase 2s+1 = MFMA s
//   Y: phase 2s+1 = read s + DMA s+2, phase 2s+2 = MFMA s
// Stage s+2's buffer (that of s-1) was last read in phase 2s-1 (Y), retired
// by Y's lgkmcnt(0) before barrier 2s. Stage s+1 is needed from phase 2s+2:
// both groups retire their pieces of it (vmcnt(6): stage s+2's stay in
// flight) before barrier 2s+2. Measured at 4096^3: MFMA pipe busy 85 % of
// the shader clock, which under this load settles near 1.65 GHz (power).
__global__ void __launch_bounds__(512, 1)
    k_share_gemm16s(const u8* __restrict__ Ad, const u8* __restrict__ Bd, u64 M, u64 N, u64 stagesTotal,
                    u64 stagesPerSplit, u32 TM, u32 TN, u32 splits, i64* __restrict__ P, const i64* __restrict__ sub) {
    constexpr u32 NBUF = 3, kT = 512;
    constexpr u32 kStageA = TBM * kRec, kStageB = BN * kRec, kStage = kStageA + kStageB;
    constexpr u32 kPiecesA = TBM / 4, kPieces = kPiecesA + BN / 4, kPerWave = kPieces / 8;
    __shared__ __attribute__((aligned(16))) u8 lds[NBUF * kStage];
    const u32 tid = threadIdx.x, lane = tid & 63;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool Y = wave >= 4;
    const TileCoord tc = tile_of(blockIdx.x, TM, TN, splits);
    const u64 m0 = (u64)tc.tm * TBM, n0 = (u64)tc.tn * BN;
    const u64 s0 = (u64)tc.split * stagesPerSplit;
    const u64 s1 = min(stagesTotal, s0 + stagesPerSplit);
    i64* dst = P + (splits > 1 ? (u64)tc.split * M * N : 0);
    if (s0 >= s1) {
        for (u32 i = tid; i < TBM * BN; i += kT) {
            u64 m = m0 + i / BN, n = n0 + i % BN;
            if (m < M && n < N) dst[m * N + n] = 0;
        }
        return;
    }
    const u32 nst = (u32)(s1 - s0);

    const u32 lrow = lane >> 4, lslot = lane & 15;
    const u8* src[kPerWave];
    u32 ldsOff[kPerWave];
#pragma unroll
    for (u32 j = 0; j < kPerWave; ++j) {
        const u32 q = wave * kPerWave + j;
        const bool isA = q < kPiecesA;
        const u32 r = 4 * (isA ? q : q - kPiecesA) + lrow;
        const u32 g = lslot ^ (r & 15);
        src[j] = (isA ? Ad + (m0 + r) * stagesTotal * kRec : Bd + (n0 + r) * stagesTotal * kRec) + g * 16;
        ldsOff[j] = (isA ? 0 : kStageA) + 4 * (isA ? q : q - kPiecesA) * kRec;
    }
    auto issue = [&](u64 st, u32 b) {
#pragma unroll
        for (u32 j = 0; j < kPerWave; ++j)
            __builtin_amdgcn_global_load_lds((glb_void*)(src[j] + st * kRec), (lds_void*)(lds + b * kStage + ldsOff[j]),
                                             16, 0, 0);
    };

    v4i acc[8][2][2];
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[s][i][j] = v4i{0};

    const u32 wr = (wave >> 1 & 1) * 32 + (wave >> 2) * 64, wc = (wave & 1) * 32;
    const u32 r16 = lane & 15, g4 = lane >> 4, hi = g4 >> 1, hf = g4 & 1;
    u32 offA[4][2], offB[8][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const u32 row = wr + 16 * i + r16;
#pragma unroll
        for (int e = 0; e < 4; ++e) offA[e][i] = row * kRec + (((2 * (2 * e + hi) + hf) ^ r16) * 16);
        const u32 col = wc + 16 * i + r16;
#pragma unroll
        for (int f = 0; f < 8; ++f) {
            const u32 g = 2 * (f == 0 ? 0 : (hi ? f - 1 : f)) + hf;
            offB[f][i] = kStageA + col * kRec + ((g ^ r16) * 16);
        }
    }
    const bool zhalf = hi != 0;

    {
        issue(s0, 0);
        issue(min(s0 + 1, s1 - 1), 1);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kPerWave) : "memory");
    }
    __builtin_amdgcn_s_barrier();      // barrier 0: stage 0 visible
    if (Y) __builtin_amdgcn_s_barrier();  // Y starts one phase late

    u32 buf = 0;
    for (u32 it = 0; it < nst; ++it) {
        // ---- read phase: DMA of stage it + 2 into the free buffer, this stage's fragments
        issue(min(s0 + it + 2, s1 - 1), buf == 0 ? 2 : buf - 1);
        const u8* ls = lds + buf * kStage;
        v4i a[4][2], b[8][2];
#pragma unroll
        for (int f = 0; f < 8; ++f)
#pragma unroll
            for (int j = 0; j < 2; ++j) b[f][j] = *reinterpret_cast<const v4i*>(ls + offB[f][j]);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int i = 0; i < 2; ++i) a[e][i] = *reinterpret_cast<const v4i*>(ls + offA[e][i]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (Y) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kPerWave) : "memory");
        __builtin_amdgcn_s_barrier();
        // ---- MFMA phase
#pragma unroll
        for (int j = 0; j < 2; ++j)
            if (zhalf) b[0][j] = v4i{0};
        // (no s_setprio around the MFMAs: raising the MFMA wave's priority
        // over its SIMD partner's reads measured 2 % slower on C2, 0.2591-0.2611
        // vs 0.2546-0.2557 ms)
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int f = 0; f + 2 * e < 8; ++f)
                        acc[2 * e + f][i][j] =
                            __builtin_amdgcn_mfma_i32_16x16x64_i8(a[e][i], b[f][j], acc[2 * e + f][i][j], 0, 0, 0);
        if (!Y) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kPerWave) : "memory");
        __builtin_amdgcn_s_barrier();
        buf = buf == 2 ? 0 : buf + 1;
    }
    if (!Y) __builtin_amdgcn_s_barrier();  // equal barrier counts
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                u64 v = 0;
#pragma unroll
                for (int s = 0; s < 8; ++s) v += (u64)(i64)acc[s][i][j][r] << (8 * s);
                const u64 m = m0 + wr + 16 * i + 4 * g4 + r;
                const u64 n = n0 + wc + 16 * j + r16;
                if (m < M && n < N) {
                    const u64 x = m * N + n;
                    if (sub) v -= (u64)sub[x];
                    dst[x] = (i64)v;
                }
            }
}

// Optional turn-taking of share-GEMM launches on one device (in issue order,
// whichever stream issues them) through a device-wide event chain (stream
// waits on the previous GEMM's completion event; no host sync): bench.py's
// roofline pass uses it (aby3g_mfma_turn) so that a launch's event span is
// its own. Off otherwise: letting co-located parties' GEMMs overlap measured
// +6 % on C2 -- the next GEMM's workgroups fill the CUs the previous one's
// tail frees.
class MfmaTurn {
public:
    explicit MfmaTurn(hipStream_t s) : s_(s) {
        if (!enabled()) return;
        dev_ = current_device();
        mu().lock();
        hipEvent_t& last = events()[dev_];
        if (last) {
            hipError_t e = hipStreamWaitEvent(s_, last, 0);
            if (e != hipSuccess) {
                mu().unlock();
                ABY3G_CHECK_HIP(e);
            }
        }
    }
    ~MfmaTurn() {
        if (!enabled()) return;
        hipEvent_t& last = events()[dev_];
        if (!last) (void)hipEventCreateWithFlags(&last, hipEventDisableTiming);
        if (last) (void)hipEventRecord(last, s_);
        mu().unlock();
    }

    static std::atomic<int>& mode() {
        static std::atomic<int> on{0};
        return on;
    }

private:
    static bool enabled() { return mode().load(std::memory_order_relaxed) != 0; }
    static std::mutex& mu() {
        static std::mutex m;
        return m;
    }
    static std::map<int, hipEvent_t>& events() {
        static std::map<int, hipEvent_t> e;
        return e;
    }
    hipStream_t s_;
    int dev_ = 0;
};

struct Workspace {
    u8* Ad;
    u8* Bd;
    i64* P;
};

Workspace carve(const GemmPlan& p, void* ws) {
    u8* base = (u8*)ws;
    Workspace w;
    w.Ad = base;
    w.Bd = base + roundup(p.aBytes, 256);
    w.P = (i64*)(base + roundup(p.aBytes, 256) + roundup(p.bBytes, 256));
    return w;
}

struct DigitArgs {
    const i64 *A0, *A1, *B0, *B1;
    u64 M, K, N, S2, aGroups, groups, stages;
    u8 *Ad, *Bd;
};
DigitArgs digit_args(const GemmPlan& p, const i64* A, const i64* B, const Workspace& w) {
    DigitArgs da;
    da.A0 = A;
    da.A1 = A + p.M * p.K;
    da.B0 = B;
    da.B1 = B + p.K * p.N;
    da.M = p.M;
    da.K = p.K;
    da.N = p.N;
    da.stages = p.Kc / BK;
    da.S2 = p.Kp / 32;
    da.aGroups = (p.Mp / kDigitRows) * da.S2;
    da.groups = da.aGroups + (p.Np / kBGroupCols) * da.S2;
    da.Ad = w.Ad;
    da.Bd = w.Bd;
    return da;
}

// The MFMA GEMM over digit records already in the workspace. One split: the
// GEMM writes the product (minus `sub`, when given) straight to `out`;
// several: `splits` partial slabs in w.P (the caller reduces them).
void run_share_gemm(const GemmPlan& p, const Workspace& w, hipStream_t s, i64* out = nullptr,
                    const i64* sub = nullptr, hipEvent_t subReady = nullptr) {
    const u64 stages = p.Kc / BK;
    const u32 TM = (u32)(p.Mp / p.tbm), TN = (u32)(p.Np / BN);
    const bool direct = p.splits == 1 && out != nullptr;
    if (direct && sub && subReady) ABY3G_CHECK_HIP(hipStreamWaitEvent(s, subReady, 0));
    MfmaTurn turn(s);
    i64* dst = direct ? out : w.P;
    const i64* sb = direct ? sub : nullptr;
    const dim3 grid(TM * TN * p.splits);
    const u64 sps = p.kPerSplit / BK;
    launch(PROBE_GEMM, k_share_gemm16s, grid, dim3(512), 0, s, (const u8*)w.Ad, (const u8*)w.Bd, p.M, p.N, stages, sps,
           TM, TN, p.splits, dst, sb);
}

// Runs the digit split and the MFMA GEMM.
void run_gemm(const GemmPlan& p, const i64* A, const i64* B, const Workspace& w, hipStream_t s, i64* out = nullptr,
              const i64* sub = nullptr, hipEvent_t subReady = nullptr) {
    const DigitArgs da = digit_args(p, A, B, w);
    launch(PROBE_DIGITS, k_digits<kBGroupCols>, dim3((u32)da.groups), dim3(256), 0, s, da.A0, da.A1, da.B0, da.B1, p.M,
           p.K, p.N, da.S2, da.aGroups, da.stages, w.Ad, w.Bd);
    run_share_gemm(p, w, s, out, sub, subReady);
}

void check_ws(const GemmPlan& p, void* ws, size_t bytes) {
    ABY3G_REQUIRE(ws != nullptr && bytes >= p.total, "workspace too small (see aby3g_mul_workspace_bytes)");
}

}  // namespace

}  // namespace aby3g

using namespace aby3g;

extern "C" {

int aby3g_set_gemm_sharing(int parties) {
    return guarded([&] {
        ABY3G_REQUIRE(parties >= 1 && parties <= 256, "parties out of range");
        t_gemm_sharing = (u32)parties;
    });
}

int aby3g_mfma_turn(int on) {
    return guarded([&] { MfmaTurn::mode().store(on ? 1 : 0); });
}

int aby3g_mul_prefers_fused(int mode, uint64_t M, uint64_t K, uint64_t N) {
    return mode != ABY3G_MUL_GEMM || small_gemm(M, K, N);
}

size_t aby3g_mul_workspace_bytes(int mode, uint64_t M, uint64_t K, uint64_t N) {
    if (mode != ABY3G_MUL_GEMM || small_gemm(M, K, N)) return 0;
    return plan_gemm(M, K, N).total;
}

int aby3g_mul_local(int mode, const int64_t* A, const int64_t* B, int64_t* C0, uint64_t M, uint64_t K, uint64_t N,
                    const aby3g_zero_share* zs, void* workspace, size_t workspace_bytes, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(mode == ABY3G_MUL_HADAMARD || mode == ABY3G_MUL_GEMM, "bad mode");
        const u64 n = M * N;
        if (!n) return;
        if (mode == ABY3G_MUL_HADAMARD) {
            SrcHadamard src{A, A + n, B, B + n};
            if (zs)
                launch_finish_zero_share(src, n, *zs, C0, S(stream));
            else
                launch_finish_plain(src, n, C0, S(stream));
            return;
        }
        if (small_gemm(M, K, N)) {
            run_small_gemm(A, B, M, K, N, C0, S(stream));
            if (zs) launch_finish_zero_share(SrcSlabs{C0, 1, n}, n, *zs, C0, S(stream));
            return;
        }
        GemmPlan p = plan_gemm(M, K, N);
        check_ws(p, workspace, workspace_bytes);
        Workspace w = carve(p, workspace);
        if (p.splits == 1) {
            // the GEMM writes the product into C0; the zero-share is added in place
            run_gemm(p, A, B, w, S(stream), C0);
            if (zs) launch_finish_zero_share(SrcSlabs{C0, 1, n}, n, *zs, C0, S(stream));
            return;
        }
        run_gemm(p, A, B, w, S(stream));
        SrcSlabs src{w.P, p.splits, n};
        if (zs)
            launch_finish_zero_share(src, n, *zs, C0, S(stream));
        else
            launch_finish_plain(src, n, C0, S(stream));
    });
}

int aby3g_mul_trunc_local(int mode, const int64_t* A, const int64_t* B, uint64_t M, uint64_t K, uint64_t N,
                          unsigned d, const aby3g_trunc_streams* ts, int64_t* z, int64_t* C, void* workspace,
                          size_t workspace_bytes, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(mode == ABY3G_MUL_HADAMARD || mode == ABY3G_MUL_GEMM, "bad mode");
        ABY3G_REQUIRE(ts != nullptr, "null trunc streams");
        const u64 n = M * N;
        if (!n) return;
        if (mode == ABY3G_MUL_HADAMARD) {
            SrcHadamard src{A, A + n, B, B + n};
            launch_finish_trunc(src, *ts, n, d, nullptr, C, C + n, z, S(stream));
            return;
        }
        if (small_gemm(M, K, N)) {
            run_small_gemm(A, B, M, K, N, z, S(stream));  // product into z, then z -= r in place
            launch_finish_trunc(SrcSlabs{z, 1, n}, *ts, n, d, nullptr, C, C + n, z, S(stream));
            return;
        }
        GemmPlan p = plan_gemm(M, K, N);
        check_ws(p, workspace, workspace_bytes);
        Workspace w = carve(p, workspace);
        if (p.splits == 1) {
            run_gemm(p, A, B, w, S(stream), z);  // product into z, then z -= r in place
            launch_finish_trunc(SrcSlabs{z, 1, n}, *ts, n, d, nullptr, C, C + n, z, S(stream));
            return;
        }
        run_gemm(p, A, B, w, S(stream));
        SrcSlabs src{w.P, p.splits, n};
        launch_finish_trunc(src, *ts, n, d, nullptr, C, C + n, z, S(stream));
    });
}

int aby3g_mul_sub_local(int mode, const int64_t* A, const int64_t* B, const int64_t* sub, aby3g_event sub_ready,
                        int64_t* out, uint64_t M, uint64_t K, uint64_t N, void* workspace, size_t workspace_bytes,
                        aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(mode == ABY3G_MUL_HADAMARD || mode == ABY3G_MUL_GEMM, "bad mode");
        ABY3G_REQUIRE(sub != nullptr && out != nullptr, "null operand");
        const u64 n = M * N;
        if (!n) return;
        if (mode == ABY3G_MUL_HADAMARD) {
            if (sub_ready) ABY3G_CHECK_HIP(hipStreamWaitEvent(S(stream), (hipEvent_t)sub_ready, 0));
            launch_finish_plain(SrcHadamardMinus{A, A + n, B, B + n, sub}, n, out, S(stream));
            return;
        }
        if (small_gemm(M, K, N)) {
            run_small_gemm(A, B, M, K, N, out, S(stream));
            if (sub_ready) ABY3G_CHECK_HIP(hipStreamWaitEvent(S(stream), (hipEvent_t)sub_ready, 0));
            launch_finish_plain(SrcSlabsMinus{out, 1, n, sub}, n, out, S(stream));
            return;
        }
        GemmPlan p = plan_gemm(M, K, N);
        check_ws(p, workspace, workspace_bytes);
        Workspace w = carve(p, workspace);
        if (p.splits == 1) {
            // out = product - sub in the GEMM's epilogue (waits for sub_ready before the GEMM)
            run_gemm(p, A, B, w, S(stream), out, sub, (hipEvent_t)sub_ready);
            return;
        }
        run_gemm(p, A, B, w, S(stream));
        if (sub_ready) ABY3G_CHECK_HIP(hipStreamWaitEvent(S(stream), (hipEvent_t)sub_ready, 0));
        launch_finish_plain(SrcSlabsMinus{w.P, p.splits, n, sub}, n, out, S(stream));
    });
}

}  // extern "C"
