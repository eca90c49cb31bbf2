// Bit-sliced binary engine (Sh3BinaryEvaluator) on gfx950.
//
// Memory is wire-major: mem[share][wire][word], one u64 word = 64 rows, the
// row count padded to a multiple of 2048 (Sh3BinaryEvaluator.cpp:84). A gate
// batch is a set of mutually independent gates of one communication level;
// each workgroup handles one gate (wave-uniform type and wire ids, read
// through the scalar cache) over 512 consecutive words, 2 words (16 B) per
// lane, so every load and store is a fully coalesced 1 KiB wave access.
// The AND-gate masks z are produced up front by aby3g_share_draws
// (ABY3G_DRAW_BIN: z[k][w] = getShares() of Sh3BinaryEvaluator.cpp:1406-1434
// for the k-th AND-type gate), so the gate kernel is pure streaming.
#include "common.h"

namespace aby3g {

namespace {

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

constexpr u32 kGateBlock = 256;

__global__ void __launch_bounds__(kGateBlock) k_bin_gates(const aby3g_gate* __restrict__ gates, u64* __restrict__ mem,
                                                          u64 wires, u64 words, const u64* __restrict__ z,
                                                          u64* __restrict__ sendbuf) {
    const aby3g_gate g = gates[blockIdx.y];
    const u64 w = ((u64)blockIdx.x * kGateBlock + threadIdx.x) * 2;
    if (w >= words) return;
    u64* s0 = mem;
    u64* s1 = mem + wires * words;
    const u64x2 x0 = *reinterpret_cast<const u64x2*>(s0 + g.in0 * words + w);
    const u64x2 x1 = *reinterpret_cast<const u64x2*>(s1 + g.in0 * words + w);
    u64x2 o0, o1;
    switch (g.type) {
        case ABY3G_GATE_COPY:
            o0 = x0;
            o1 = x1;
            break;
        case ABY3G_GATE_INV:
            o0 = ~x0;
            o1 = ~x1;
            break;
        default: {
            const u64x2 y0 = *reinterpret_cast<const u64x2*>(s0 + g.in1 * words + w);
            const u64x2 y1 = *reinterpret_cast<const u64x2*>(s1 + g.in1 * words + w);
            if (g.type == ABY3G_GATE_XOR) {
                o0 = x0 ^ y0;
                o1 = x1 ^ y1;
                break;
            }
            if (g.type == ABY3G_GATE_NXOR) {
                o0 = ~(x0 ^ y0);
                o1 = ~(x1 ^ y1);
                break;
            }
            // AND-type (Sh3BinaryEvaluator.cpp:700-1065): share 0 only.
            u64x2 r;
            if (g.type == ABY3G_GATE_AND)
                r = (x0 & y0) ^ (x0 & y1) ^ (x1 & y0);
            else if (g.type == ABY3G_GATE_OR)
                r = (x0 & y0) ^ (x0 & y1) ^ (x1 & y0) ^ x0 ^ y0;
            else if (g.type == ABY3G_GATE_NOR)
                r = (~x0 & ~y0) ^ (~x0 & ~y1) ^ (~x1 & ~y0);
            else /* NA_AND */
                r = (~x0 & y0) ^ (~x0 & y1) ^ (~x1 & y0);
            r ^= *reinterpret_cast<const u64x2*>(z + (u64)g.z_row * words + w);
            *reinterpret_cast<u64x2*>(s0 + g.out * words + w) = r;
            *reinterpret_cast<u64x2*>(sendbuf + (u64)g.send_row * words + w) = r;
            return;
        }
    }
    *reinterpret_cast<u64x2*>(s0 + g.out * words + w) = o0;
    *reinterpret_cast<u64x2*>(s1 + g.out * words + w) = o1;
}

// One whole communication level per launch. A workgroup owns 32 consecutive
// words (2048 rows) of every wire; its 256 threads are 16 gate slots x 16
// lanes of two words (or, for launches of few workgroups, 1024 threads: 32
// slots x 32 lanes of one word). It first unpacks the
// previous level's received AND shares into share 1, then runs the level's
// gate batches in order, the slots striding over a batch's (independent)
// gates, with a workgroup barrier
// between batches: a gate only ever reads words of its own rows, so the
// per-workgroup barrier orders every dependency of the level.
constexpr u32 kLevelWords = 32;
// launches of fewer workgroups than this take the 1024-thread form (more
// gate parallelism per workgroup), larger ones the 256-thread form
constexpr u32 kLevelSmallMaxWgs = 128;

// Words per lane: a lane of the level kernels' gate slots handles W
// consecutive words of a gate's rows. The 256-thread forms take W = 2
// (16-byte accesses, 16 lanes a slot, twice the slots of a workgroup): a
// level alone 18.3 against 21.1 us (`scripts/bench_level.py`), C5 59.7-59.8
// against 66.9-67.3 ms and C3 0.302-0.305 against 0.331 ms in a same-box
// A/B. The 1024-thread forms of small launches keep W = 1 (C3's circuit over
// 2^17 rows: 0.106-0.112 against 0.138-0.141 ms with W = 2).
template <u32 W>
struct Words;
template <>
struct Words<1> {
    typedef u64 T;
};
template <>
struct Words<2> {
    typedef u64x2 T;
};
template <u32 W>
using WordsT = typename Words<W>::T;

template <u32 W>
__device__ __forceinline__ WordsT<W> wzero() {
    if constexpr (W == 1)
        return 0;
    else
        return u64x2{0, 0};
}
template <u32 W>
__device__ __forceinline__ WordsT<W> wld(const u64* p) {
    return *reinterpret_cast<const WordsT<W>*>(p);
}
template <u32 W>
__device__ __forceinline__ void wst(u64* p, WordsT<W> v) {
    *reinterpret_cast<WordsT<W>*>(p) = v;
}
// received shares handed over in-kernel: read past this CU's L1 (sc1); sent
// ones stored write-through
template <u32 W>
__device__ __forceinline__ WordsT<W> wld_hs(const u64* p) {
    if constexpr (W == 1)
        return hs_load(p);
    else
        return u64x2{hs_load(p), hs_load(p + 1)};
}
template <u32 W>
__device__ __forceinline__ void wst_hs(u64* p, WordsT<W> v) {
    if constexpr (W == 1) {
        hs_store(p, v);
    } else {
        hs_store(p, v.x);
        hs_store(p + 1, v.y);
    }
}

// Operands of one gate on a lane's words, loaded ahead of its evaluation so
// that a slot can have several independent gates' loads in flight.
template <u32 W>
struct GateOps {
    WordsT<W> x0, x1, y0, y1, z;
};

// rr: the recv rows of the inputs' share 1 when they are the previous
// level's AND outputs (~0u: read the engine memory), so that the gates need
// not wait for the unpack of this launch
template <u32 W>
__device__ __forceinline__ void gate_load(const aby3g_gate& g, uint2 rr, const u64* s0, const u64* s1,
                                          const u64* __restrict__ recv, u64 words, u64 w, const u64* __restrict__ z,
                                          GateOps<W>& o, bool sc1) {  // sc1: compile-time constant at every call
    // unary gates read in0 twice (in1 of an external gate list may be anything)
    const bool unary = g.type == ABY3G_GATE_COPY || g.type == ABY3G_GATE_INV;
    const u64 in1 = unary ? g.in0 : g.in1;
    const u32 r1 = unary ? rr.x : rr.y;
    o.x0 = wld<W>(s0 + g.in0 * words + w);
    o.x1 = rr.x != ~0u ? (sc1 ? wld_hs<W>(recv + (u64)rr.x * words + w) : wld<W>(recv + (u64)rr.x * words + w))
                       : wld<W>(s1 + g.in0 * words + w);
    o.y0 = wld<W>(s0 + in1 * words + w);
    o.y1 = r1 != ~0u ? (sc1 ? wld_hs<W>(recv + (u64)r1 * words + w) : wld<W>(recv + (u64)r1 * words + w))
                     : wld<W>(s1 + in1 * words + w);
    o.z = gate_is_and(g.type) ? wld<W>(z + (u64)g.z_row * words + w) : wzero<W>();
}

template <u32 W>
__device__ __forceinline__ void gate_eval(const aby3g_gate& g, const GateOps<W>& o, u64* s0, u64* s1, u64 words,
                                          u64 w, u64* __restrict__ sendbuf, bool wt) {
    if (gate_is_and(g.type)) {
        const WordsT<W> r = gate_and_share(g.type, o.x0, o.x1, o.y0, o.y1) ^ o.z;
        wst<W>(s0 + g.out * words + w, r);
        if (wt)  // a message handed over in-kernel: write-through
            wst_hs<W>(sendbuf + (u64)g.send_row * words + w, r);
        else
            wst<W>(sendbuf + (u64)g.send_row * words + w, r);
        return;
    }
    WordsT<W> o0, o1;
    gate_local(g.type, o.x0, o.x1, o.y0, o.y1, o0, o1);
    wst<W>(s0 + g.out * words + w, o0);
    wst<W>(s1 + g.out * words + w, o1);
}

// SLOTS * W gate slots x 32 / W lanes. Each slot takes kLevelUnroll gates of
// a batch per iteration, all their loads issued before any evaluation (the
// gates of a batch are independent), so a batch of G gates costs about
// G / (SLOTS * W * kLevelUnroll) dependent memory round trips -- the bound for
// the few-workgroup launches of small row counts (LR: 256 rows, one workgroup).
constexpr u32 kLevelUnroll = 4;
// With rrows (per gate, see gate_load) no gate reads the wires this launch
// unpacks, so the first batch starts without a barrier after the unpack.
// In-kernel hand-off (co-located parties): a workgroup owns exactly one
// ABY3G_HANDOFF_ROWS chunk (its 32 words), so it waits only for the previous
// party's workgroup of the same rows (hw: the received AND shares) and
// publishes its own send rows for the next party's same workgroup (hp) --
// the levels of the three parties pipeline chunk by chunk.
static_assert(kLevelWords * 64 == ABY3G_HANDOFF_ROWS, "a level workgroup is one hand-off chunk");
template <u32 SLOTS, bool HS, u32 W, u32 U = kLevelUnroll>
__global__ void __launch_bounds__(SLOTS * 32) k_bin_level(const aby3g_gate* __restrict__ gates,
                                                         const uint2* __restrict__ rrows,
                                                         const u32* __restrict__ batch_ends, u32 nbatches,
                                                         const u64* __restrict__ recv,
                                                         const u32* __restrict__ unpack_wires, u32 nunpack,
                                                         u64* __restrict__ mem, u64 wires, u64 words,
                                                         const u64* __restrict__ z, u64* __restrict__ sendbuf,
                                                         HsWait hw, HsPost hp) {
    // HS: the in-kernel hand-off instantiation (sc1 payload accesses, waits
    // and posts); the other is the plain streaming kernel
    if (HS && !hs_wait(hw, blockIdx.x, blockIdx.x + 1)) return;
    constexpr u32 kLanes = 32 / W, NS = SLOTS * W;
    const u32 lane = threadIdx.x % kLanes, slot = threadIdx.x / kLanes;
    const u64 w = (u64)blockIdx.x * kLevelWords + W * lane;
    u64* s0 = mem;
    u64* s1 = mem + wires * words;
#pragma unroll 4
    for (u32 j = slot; j < nunpack; j += NS)
        wst<W>(s1 + (u64)unpack_wires[j] * words + w,
               (HS && hw.flags) ? wld_hs<W>(recv + (u64)j * words + w) : wld<W>(recv + (u64)j * words + w));
    u32 begin = 0;
    for (u32 b = 0; b < nbatches; ++b) {
        if (b || !rrows) __syncthreads();
        const u32 end = batch_ends[b];
        for (u32 g0 = begin + slot; g0 < end; g0 += U * NS) {
            aby3g_gate g[U];
            uint2 rr[U];
            GateOps<W> o[U];
#pragma unroll
            for (u32 k = 0; k < U; ++k)
                if (g0 + k * NS < end) {
                    g[k] = gates[g0 + k * NS];
                    rr[k] = rrows ? rrows[g0 + k * NS] : make_uint2(~0u, ~0u);
                }
#pragma unroll
            for (u32 k = 0; k < U; ++k)
                if (g0 + k * NS < end) gate_load<W>(g[k], rr[k], s0, s1, recv, words, w, z, o[k], HS);
#pragma unroll
            for (u32 k = 0; k < U; ++k)
                if (g0 + k * NS < end) gate_eval<W>(g[k], o[k], s0, s1, words, w, sendbuf, HS);
        }
        begin = end;
    }
    if (HS) hs_post(hp, blockIdx.x, blockIdx.x + 1);
}

__global__ void __launch_bounds__(kGateBlock) k_bin_unpack(const u64* __restrict__ recv, const u32* __restrict__ outw,
                                                           u64* __restrict__ mem, u64 wires, u64 words) {
    const u32 j = blockIdx.y;
    const u64 w = ((u64)blockIdx.x * kGateBlock + threadIdx.x) * 2;
    if (w >= words) return;
    const u32 wire = outw[j];
    *reinterpret_cast<u64x2*>(mem + (wires + wire) * words + w) =
        *reinterpret_cast<const u64x2*>(recv + (u64)j * words + w);
}

// One wave per (64-row word w, 64-bit column c): lane r holds row 64w + r;
// after the wave transpose lane b holds word w of wire b (LSB = row 64w).
// blockIdx.y = share: input share s at in + s * rows * cols64, its wire rows
// at wrows + s * shareStride
__global__ void __launch_bounds__(256) k_bits_to_wires(const i64* __restrict__ in, u64 rows, u64 cols64, u32 nbits,
                                                       u64* __restrict__ wrows, u64 shareStride, u64 words) {
    in += (u64)blockIdx.y * rows * cols64;
    wrows += (u64)blockIdx.y * shareStride;
    const u32 lane = threadIdx.x & 63;
    const u64 waveId = ((u64)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const u64 nw = words * cols64;
    if (waveId >= nw) return;
    const u64 w = waveId % words, c = waveId / words;
    const u64 r = w * 64 + lane;
    const u64 v = r < rows ? (u64)in[r * cols64 + c] : 0;
    const u64 mine = transpose64(v, lane);
    const u64 bit = c * 64 + lane;
    if (bit < nbits) wrows[bit * words + w] = mine;
}

// blockIdx.y = share: wire rows of share s at mem + s * shareStride, output
// share s at out + s * rows * ceil(nbits / 64)
__global__ void __launch_bounds__(256) k_wires_to_bits(const u64* __restrict__ mem, u64 shareStride,
                                                       const u32* __restrict__ wires, u32 nbits, u64 words,
                                                       i64* __restrict__ out, u64 rows) {
    const u32 lane = threadIdx.x & 63;
    const u64 waveId = ((u64)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const u64 cols = (nbits + 63) / 64;
    mem += (u64)blockIdx.y * shareStride;
    out += (u64)blockIdx.y * rows * cols;
    const u64 nw = ((rows + 63) / 64) * cols;
    if (waveId >= nw) return;
    const u64 rw = (rows + 63) / 64;
    const u64 w = waveId % rw, c = waveId / rw;
    const u64 bit = c * 64 + lane;
    const u64 v = bit < nbits ? mem[(u64)wires[bit] * words + w] : 0;
    const u64 mine = transpose64(v, lane);
    const u64 row = w * 64 + lane;
    if (row < rows) out[row * cols + c] = (i64)mine;
}

// LDS-tiled transposes (the mapped forms below): a workgroup owns 64
// consecutive words (4096 rows) of one 64-bit column. bits -> wires: each
// wave bit-transposes 16 words (transpose64) into an LDS tile [bit][word], then
// the tile leaves as 64 contiguous 512-byte wire segments. wires -> bits:
// the reverse, reading 512-byte wire segments into the tile.
constexpr u32 kTileWords = 32;                   // words of a 256-thread tile workgroup
constexpr u32 kWaveWords = kTileWords / 4;       // words a wave transposes (64 x 64 bits each)
constexpr u32 kTilePitch = kTileWords + 1;  // u64 per tile row (+1: bank spread)

// ---- register transposes: one thread per 64-row word ----------------------
// A thread holds the 64 rows of one word (R[r] = row r) and transposes them
// in registers (T[b] bit r = bit b of row r): six delta-swap stages over
// row pairs (r, r + j), 32-bit halves independent for j < 32 (the stage mask
// never takes a bit across the half boundary). About 25 VALU ops per row and
// no LDS or cross-lane traffic, so the bit-slicing passes run at the rate of
// their HBM streams: row loads / stores are 512 contiguous bytes per thread
// (16 B per lane-instruction), wire-word stores / loads 512 B per wave
// instruction (64 consecutive words of one wire).
__device__ __forceinline__ void transpose64_regs(u64 (&R)[64]) {
#pragma unroll
    for (int r = 0; r < 32; ++r) {  // j = 32: swap hi(R[r]) with lo(R[r + 32])
        const u32 a_hi = (u32)(R[r] >> 32), b_lo = (u32)R[r + 32];
        R[r] = (R[r] & 0xffffffffull) | ((u64)b_lo << 32);
        R[r + 32] = (R[r + 32] & 0xffffffff00000000ull) | a_hi;
    }
    constexpr u32 kM[5] = {0x0000ffffu, 0x00ff00ffu, 0x0f0f0f0fu, 0x33333333u, 0x55555555u};
#pragma unroll
    for (int st = 0; st < 5; ++st) {
        const int j = 16 >> st;
        const u32 m = kM[st];
#pragma unroll
        for (int r = 0; r < 64; ++r) {
            if (r & j) continue;
            u32 al = (u32)R[r], ah = (u32)(R[r] >> 32);
            u32 bl = (u32)R[r + j], bh = (u32)(R[r + j] >> 32);
            const u32 tl = ((al >> j) ^ bl) & m, th = ((ah >> j) ^ bh) & m;
            bl ^= tl;
            bh ^= th;
            al ^= tl << j;
            ah ^= th << j;
            R[r] = ((u64)ah << 32) | al;
            R[r + j] = ((u64)bh << 32) | bl;
        }
    }
}

// 64 rows of one 64-bit column -> R (rows past `rows` read as zero); a
// contiguous column (cols64 == 1) loads 16 B per lane-instruction
template <class F>
__device__ __forceinline__ void load_rows(u64 (&R)[64], u64 r0, u64 rows, u64 cols64, u64 c, F&& at) {
    if (cols64 == 1 && r0 + 64 <= rows) {
#pragma unroll
        for (int k = 0; k < 64; k += 2) {
            const u64x2 v = at.pair(r0 + k);
            R[k] = v.x;
            R[k + 1] = v.y;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 64; ++k) R[k] = (r0 + k < rows) ? at.one((r0 + k) * cols64 + c) : 0;
    }
}

struct RowsOf {
    const u64* p;
    __device__ __forceinline__ u64x2 pair(u64 r) const { return *reinterpret_cast<const u64x2*>(p + r); }
    __device__ __forceinline__ u64 one(u64 i) const { return p[i]; }
};

// bits -> wires, both shares (blockIdx.y = share), a thread per (word, column)
__global__ void __launch_bounds__(64) k_b2w_regs(const i64* __restrict__ in, u64 rows, u64 cols64, u32 nbits,
                                                 u64* __restrict__ wrows, u64 shareStride, u64 words) {
    in += (u64)blockIdx.y * rows * cols64;
    wrows += (u64)blockIdx.y * shareStride;
    const u64 wpc = (words + 63) / 64;  // workgroups per column
    const u64 c = blockIdx.x / wpc, w = (blockIdx.x % wpc) * 64 + threadIdx.x;
    if (w >= words) return;
    u64 R[64];
    load_rows(R, w * 64, rows, cols64, c, RowsOf{(const u64*)in});
    transpose64_regs(R);
#pragma unroll
    for (int b = 0; b < 64; ++b)
        if (c * 64 + b < nbits) wrows[(c * 64 + b) * words + w] = R[b];
}

// wires -> bits, both shares (blockIdx.y = share), a thread per (word, column)
__global__ void __launch_bounds__(64) k_w2b_regs(const u64* __restrict__ mem, u64 shareStride,
                                                 const u32* __restrict__ wires, u32 nbits, u64 words,
                                                 i64* __restrict__ out, u64 rows) {
    const u64 cols = (nbits + 63) / 64;
    mem += (u64)blockIdx.y * shareStride;
    out += (u64)blockIdx.y * rows * cols;
    const u64 rw = (rows + 63) / 64;
    const u64 wpc = (rw + 63) / 64;
    const u64 c = blockIdx.x / wpc, w = (blockIdx.x % wpc) * 64 + threadIdx.x;
    if (w >= rw) return;
    u64 R[64];
#pragma unroll
    for (int b = 0; b < 64; ++b) R[b] = (c * 64 + b < nbits) ? mem[(u64)wires[c * 64 + b] * words + w] : 0;
    transpose64_regs(R);
    const u64 r0 = w * 64;
    if (cols == 1 && r0 + 64 <= rows) {
#pragma unroll
        for (int k = 0; k < 64; k += 2) *reinterpret_cast<u64x2*>(out + r0 + k) = u64x2{R[k], R[k + 1]};
    } else {
#pragma unroll
        for (int k = 0; k < 64; ++k)
            if (r0 + k < rows) out[(r0 + k) * cols + c] = (i64)R[k];
    }
}

// wires -> bits for a few wires (nbits <= 8, one output column): a thread per
// output row and share gathers bit (row & 63) of each wire's word (the words
// are shared by 64 neighbouring threads and come from the cache); the row
// stores are fully coalesced and no 64 x 64 transpose is done for the one or
// few bits that exist (a comparison's output bit, the piecewise regions).
__global__ void __launch_bounds__(256) k_w2b_few(const u64* __restrict__ mem, u64 shareStride,
                                                 const u32* __restrict__ wires, u32 nbits, u64 words,
                                                 i64* __restrict__ out, u64 rows) {
    // two rows a thread: one 16-byte store when both exist and are 16-byte
    // aligned (r is even: an even row count and an aligned output)
    const u64 r = 2 * ((u64)blockIdx.x * 256 + threadIdx.x);
    if (r >= rows) return;
    mem += (u64)blockIdx.y * shareStride;
    out += (u64)blockIdx.y * rows;
    const u64 w = r >> 6;
    const u32 sh = (u32)(r & 63);  // even: rows r, r + 1 share the word
    u64 v0 = 0, v1 = 0;
    for (u32 b = 0; b < nbits; ++b) {
        const u64 x = mem[(u64)wires[b] * words + w] >> sh;
        v0 |= (x & 1ull) << b;
        v1 |= ((x >> 1) & 1ull) << b;
    }
    if (r + 1 < rows && ((uintptr_t)(out + r) & 15) == 0) {
        *reinterpret_cast<u64x2*>(out + r) = u64x2{v0, v1};
    } else {
        out[r] = (i64)v0;
        if (r + 1 < rows) out[r + 1] = (i64)v1;
    }
}

// The mapped (gather / scatter) transposes keep the LDS-tiled kernels below:
// their rows are scattered, and both register forms measured slower on C5 --
// 64 separate 8-byte row accesses per thread (118-121 vs 103 ms), and rows
// gathered wave-wide into an LDS stage then transposed per thread (101 vs
// 88-90 ms: 194 VGPRs leave too few waves to hide the gathers).

struct WireSrcs {
    aby3g_wire_src s[ABY3G_WIRE_SRC_MAX];
};
// setInput of linear combinations (aby3g_bits_to_wires_lin), one thread per
// (word, column) with register transposes. The source descriptor is
// copied out of the kernarg array first and the copy-out is stored only after
// every term load: a store through copy_out between loads would force the
// compiler (which cannot rule out aliasing) to serialise the row loads.
__global__ void __launch_bounds__(64) k_b2w_lin_regs(WireSrcs ws, u64 rows, u64 words) {
    const aby3g_wire_src src = ws.s[blockIdx.y];
    const u64 wpc = (words + 63) / 64;
    const u64 c = blockIdx.x / wpc, w = (blockIdx.x % wpc) * 64 + threadIdx.x;
    if (c * 64 >= src.nbits || w >= words) return;
    const u64 r0 = w * 64;
    const bool contig = src.cols64 == 1 && r0 + 64 <= rows;
    u64 R[64];
#pragma unroll
    for (int k = 0; k < 64; ++k) R[k] = 0;
    bool any = false;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const u64* __restrict__ p = (const u64*)src.term[t];
        if (!p) continue;
        any = true;
        const u64 cf = (u64)src.coef[t];
        if (contig) {
#pragma unroll
            for (int k = 0; k < 64; k += 2) {
                const u64x2 x = *reinterpret_cast<const u64x2*>(p + r0 + k);
                R[k] += cf * x.x;
                R[k + 1] += cf * x.y;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 64; ++k)
                if (r0 + k < rows) R[k] += cf * p[(r0 + k) * src.cols64 + c];
        }
    }
    if (any) {
        if (src.copy_out) {
            i64* __restrict__ o = src.copy_out;
            if (contig) {
#pragma unroll
                for (int k = 0; k < 64; k += 2) *reinterpret_cast<u64x2*>(o + r0 + k) = u64x2{R[k], R[k + 1]};
            } else {
#pragma unroll
                for (int k = 0; k < 64; ++k)
                    if (r0 + k < rows) o[(r0 + k) * src.cols64 + c] = (i64)R[k];
            }
        }
#pragma unroll
        for (int k = 0; k < 64; ++k)
            if (r0 + k < rows) R[k] += (u64)src.constant;  // padded rows stay zero
        transpose64_regs(R);  // (a source without terms writes zero wires as they are)
    }
    u64* __restrict__ out = src.wire_rows;
#pragma unroll
    for (int b = 0; b < 64; ++b)
        if (c * 64 + b < src.nbits) out[(c * 64 + b) * words + w] = R[b];
}

// copy_out of every source only (aby3g_lin_copy_out), a thread per two
// elements: 16-byte loads and stores (1 KiB per wave instruction; the copy-out
// is the reshare message the next party's first level waits for)
__global__ void __launch_bounds__(256) k_lin_copy(WireSrcs ws, u32 nsrc, u64 rows) {
    const u64 i = ((u64)blockIdx.x * 256 + threadIdx.x) * 2;
#pragma unroll
    for (u32 k = 0; k < ABY3G_WIRE_SRC_MAX; ++k) {
        if (k >= nsrc) break;
        const aby3g_wire_src& src = ws.s[k];
        const u64 n = rows * src.cols64;
        if (!src.copy_out || i >= n) continue;
        // 16-byte accesses when every pointer allows them (pool blocks do)
        bool vec = i + 1 < n && ((uintptr_t)src.copy_out & 15) == 0;
#pragma unroll
        for (int t = 0; t < 4; ++t) vec = vec && ((uintptr_t)src.term[t] & 15) == 0;
        if (vec) {
            u64x2 v = u64x2{0, 0};
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (src.term[t]) v += (u64)src.coef[t] * *reinterpret_cast<const u64x2*>(src.term[t] + i);
            *reinterpret_cast<u64x2*>(src.copy_out + i) = v;
        } else {
            for (u64 j = i; j < i + 2 && j < n; ++j) {
                u64 v = 0;
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    if (src.term[t]) v += (u64)src.coef[t] * (u64)src.term[t][j];
                src.copy_out[j] = (i64)v;
            }
        }
    }
}

// The first level with its inputs (aby3g_bin_level_in). A source: one 64-bit
// input (at most 64 wires from `wire` on) of one share, the sum of its terms
// plus the constant on rows < rows.
struct LevelInSrc {
    const u64* term[4];
    u64 coef[4];
    u64 constant;
    u32 wire, share, nbits, pad;
};
struct LevelInSrcs {
    LevelInSrc s[ABY3G_WIRE_SRC_MAX];
};
constexpr u32 kInMax = ABY3G_LEVEL_IN_MAX_WIRES;

// operands of one gate: input wires through tab (the LDS row of (wire - inLo,
// share) in win, kInZero: an all-zero source), other wires from mem
constexpr u32 kInZero = 0xffff;
template <u32 W = 1>
__device__ __forceinline__ WordsT<W> in_word(const u64* win, unsigned short row, u32 wl) {
    return row == kInZero ? wzero<W>() : wld<W>(win + (u32)row * kLevelWords + wl);
}
template <u32 W>
__device__ __forceinline__ void gate_load_in(const aby3g_gate& g, const u64* win, const unsigned short* tab, u32 inLo,
                                             u32 nin, const u64* s0, const u64* s1, u64 words, u64 w, u32 wl,
                                             const u64* __restrict__ z, GateOps<W>& o) {
    const bool unary = g.type == ABY3G_GATE_COPY || g.type == ABY3G_GATE_INV;
    const u32 in1 = unary ? g.in0 : g.in1;
    const u32 a = g.in0 - inLo, b = in1 - inLo;
    if (a < nin) {
        o.x0 = in_word<W>(win, tab[2 * a], wl);
        o.x1 = in_word<W>(win, tab[2 * a + 1], wl);
    } else {
        o.x0 = wld<W>(s0 + (u64)g.in0 * words + w);
        o.x1 = wld<W>(s1 + (u64)g.in0 * words + w);
    }
    if (b < nin) {
        o.y0 = in_word<W>(win, tab[2 * b], wl);
        o.y1 = in_word<W>(win, tab[2 * b + 1], wl);
    } else {
        o.y0 = wld<W>(s0 + (u64)in1 * words + w);
        o.y1 = wld<W>(s1 + (u64)in1 * words + w);
    }
    o.z = gate_is_and(g.type) ? wld<W>(z + (u64)g.z_row * words + w) : wzero<W>();
}

// One workgroup per ABY3G_HANDOFF_ROWS chunk, as k_bin_level. Its waves first
// build the chunk's input words of every source WITH terms in LDS (16 KiB a
// source, dynamic: a source without terms is all zero and takes no LDS, so a
// party's comparison input -- one or two non-zero sources of the four --
// keeps the level kernel's occupancy): a wave per (source, word), lane = row,
// the sum of the terms transposed with transpose64 (lane b gets bit b of the
// 64 rows). The inputs are read once, as the rows of the shares, and the
// level's gates then read the input wires from LDS instead of HBM (the first
// level of a 64-bit comparison reads each input wire 2-3 times).
template <u32 SLOTS, bool HS, u32 W>
__global__ void __launch_bounds__(SLOTS * 32) k_bin_level_in(LevelInSrcs srcs, u32 nsrc, u64 rows, u32 inLo, u32 nin,
                                                            int writeInputs, const aby3g_gate* __restrict__ gates,
                                                            const u32* __restrict__ batch_ends, u32 nbatches,
                                                            u64* __restrict__ mem, u64 wires, u64 words,
                                                            const u64* __restrict__ z, u64* __restrict__ sendbuf,
                                                            HsPost hp) {
    extern __shared__ __attribute__((aligned(16))) u64 win[];  // [source][64 wires][32 words]
    __shared__ unsigned short tab[2 * kInMax];                           // (wire - inLo, share) -> win row
    constexpr u32 kT = SLOTS * 32, kWaves = kT / 64;
    const u32 tid = threadIdx.x, lane64 = tid & 63, wave = tid >> 6;
    for (u32 i = tid; i < 2 * nin; i += kT) tab[i] = kInZero;  // uncovered wires read zero
    __syncthreads();
    // sources are in LDS-slot order (the launcher passes only sources with terms)
    for (u32 i = tid; i < nsrc * 64; i += kT) {
        const u32 k = i >> 6, b = i & 63;
        u32 wire = 0, share = 0, nbits = 0;
#pragma unroll
        for (u32 j = 0; j < ABY3G_WIRE_SRC_MAX; ++j)
            if (j == k) wire = srcs.s[j].wire, share = srcs.s[j].share, nbits = srcs.s[j].nbits;
        if (b < nbits) tab[2 * (wire - inLo + b) + share] = (unsigned short)(k * 64 + b);
    }
    const u64 w0 = (u64)blockIdx.x * kLevelWords;
    // a wave's words of a source: every load issued before the first
    // transpose (one memory latency per source, not one per word)
    constexpr u32 kPer = kLevelWords / kWaves;
#pragma unroll
    for (u32 k = 0; k < ABY3G_WIRE_SRC_MAX; ++k) {
        if (k >= nsrc) break;
        const LevelInSrc& src = srcs.s[k];
        u64 v[kPer];
#pragma unroll
        for (u32 i = 0; i < kPer; ++i) v[i] = 0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const u64* __restrict__ p = src.term[t];
            if (!p) continue;
            const u64 cf = src.coef[t];
#pragma unroll
            for (u32 i = 0; i < kPer; ++i) {
                const u64 r = (w0 + wave + i * kWaves) * 64 + lane64;
                if (r < rows) v[i] += cf * p[r];
            }
        }
#pragma unroll
        for (u32 i = 0; i < kPer; ++i) {
            const u64 r = (w0 + wave + i * kWaves) * 64 + lane64;
            const u64 tw = transpose64(r < rows ? v[i] + src.constant : 0, lane64);
            win[(k * 64 + lane64) * kLevelWords + wave + i * kWaves] = tw;  // rows >= nbits: never looked up
        }
    }
    __syncthreads();
    u64* s0 = mem;
    u64* s1 = mem + wires * words;
    if (writeInputs)
        for (u32 i = tid; i < nin * 2 * kLevelWords; i += kT) {
            const u32 wl = i % kLevelWords, sh = (i / kLevelWords) & 1, wi = i / (2 * kLevelWords);
            (sh ? s1 : s0)[(u64)(inLo + wi) * words + w0 + wl] = in_word(win, tab[2 * wi + sh], wl);
        }
    constexpr u32 kLanes = 32 / W, NS = SLOTS * W;
    const u32 wl = W * (tid % kLanes), slot = tid / kLanes;
    const u64 w = w0 + wl;
    u32 begin = 0;
    for (u32 b = 0; b < nbatches; ++b) {
        if (b) __syncthreads();
        const u32 end = batch_ends[b];
        for (u32 g0 = begin + slot; g0 < end; g0 += kLevelUnroll * NS) {
            aby3g_gate g[kLevelUnroll];
            GateOps<W> o[kLevelUnroll];
#pragma unroll
            for (u32 k = 0; k < kLevelUnroll; ++k)
                if (g0 + k * NS < end) g[k] = gates[g0 + k * NS];
#pragma unroll
            for (u32 k = 0; k < kLevelUnroll; ++k)
                if (g0 + k * NS < end) gate_load_in<W>(g[k], win, tab, inLo, nin, s0, s1, words, w, wl, z, o[k]);
#pragma unroll
            for (u32 k = 0; k < kLevelUnroll; ++k)
                if (g0 + k * NS < end) gate_eval<W>(g[k], o[k], s0, s1, words, w, sendbuf, HS);
        }
        begin = end;
    }
    if (HS) hs_post(hp, blockIdx.x, blockIdx.x + 1);
}


// Rows p, p + 64, p + 128, ... of a merge round's compare-exchange list ->
// rows of the merge array (aby3g_rowmap), without a division per row (a 32-
// or 64-bit division is ~20-40 VALU ops, 16 of them per thread made the
// mapped transposes VALU-bound): one division at the start, then each step
// adds 64 / per_rep reps and 64 % per_rep positions with one carry.
struct MapWalk {
    u64 q, rep, k, qd, qm;
};
__device__ __forceinline__ MapWalk map_walk(const aby3g_rowmap& m, u64 p) {
    MapWalk w;
    w.q = m.first + p;
    if (m.idx) return w;
    if (((w.q | m.per_rep) >> 32) == 0) {
        const u32 qq = (u32)w.q, pr = (u32)m.per_rep, r32 = qq / pr;
        w.rep = r32;
        w.k = qq - r32 * pr;
        w.qd = 64u / pr;
        w.qm = 64u - (u32)w.qd * pr;
    } else {
        w.rep = w.q / m.per_rep;
        w.k = w.q - w.rep * m.per_rep;
        w.qd = 64 / m.per_rep;
        w.qm = 64 - w.qd * m.per_rep;
    }
    return w;
}
__device__ __forceinline__ u64 map_walk_row(const aby3g_rowmap& m, const MapWalk& w) {
    return m.idx ? m.idx[w.q] : m.start + w.rep * m.rep_stride + w.k * m.step;
}
__device__ __forceinline__ void map_walk_next(const aby3g_rowmap& m, MapWalk& w) {
    w.q += 64;
    if (m.idx) return;
    w.k += w.qm;
    w.rep += w.qd;
    if (w.k >= m.per_rep) {
        w.k -= m.per_rep;
        ++w.rep;
    }
}

// LDS-tiled bits -> wires over mapped source rows (the round's gather fused
// into setInput). Rows mapped outside the source read as zero.
// Up to two (map, destination) pairs per launch, blockIdx.z selecting one:
// the two inputs of a compare-exchange round (its two gathers) or its two
// outputs (its two scatters) in one grid.
struct MapPair {
    aby3g_rowmap map[2];
    u64* wrows[2];            // k_bits_to_wires_map
    const u32* wires[2];      // k_wires_to_bits_map
};

__global__ void __launch_bounds__(256) k_bits_to_wires_map(const i64* __restrict__ in, u64 inRows, u64 cols64,
                                                           u32 nbits, MapPair jobs, u64 rows, u64 shareStride,
                                                           u64 words) {
    __shared__ u64 tile[64 * kTilePitch];
    const aby3g_rowmap& map = jobs.map[blockIdx.z];
    u64* wrows = jobs.wrows[blockIdx.z];
    in += (u64)blockIdx.y * inRows * cols64;
    wrows += (u64)blockIdx.y * shareStride;
    const u64 tilesPerCol = (words + kTileWords - 1) / kTileWords;
    const u64 c = blockIdx.x / tilesPerCol, w0 = (blockIdx.x % tilesPerCol) * kTileWords;
    const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    u64 vv[kWaveWords];
    MapWalk mw = map_walk(map, (w0 + wave * kWaveWords) * 64 + lane);  // the thread's rows step by 64
#pragma unroll
    for (u32 k = 0; k < kWaveWords; ++k) {
        const u32 wl = wave * kWaveWords + k;
        const u64 r = (w0 + wl) * 64 + lane;
        u64 v = 0;
        if (w0 + wl < words && r < rows) {
            const u64 src = map_walk_row(map, mw);
            if (src < inRows) v = (u64)in[src * cols64 + c];
        }
        vv[k] = v;
        map_walk_next(map, mw);
    }
    // unrolled: the transposes are independent, so their exchange stages
    // interleave instead of waiting out each one's latency in turn
#pragma unroll
    for (u32 k = 0; k < kWaveWords; ++k) vv[k] = transpose64(vv[k], lane);
#pragma unroll
    for (u32 k = 0; k < kWaveWords; ++k) tile[lane * kTilePitch + wave * kWaveWords + k] = vv[k];
    __syncthreads();
    // two words a thread: one 16-byte store when both are in the row and aligned
    for (u32 idx = threadIdx.x; idx < 32 * kTileWords; idx += 256) {
        const u32 b = idx / (kTileWords / 2), wl = 2 * (idx % (kTileWords / 2));
        const u64 bit = c * 64 + b;
        if (bit < nbits && w0 + wl < words) {
            u64* dst = wrows + bit * words + w0 + wl;
            const u64 v0 = tile[b * kTilePitch + wl], v1 = tile[b * kTilePitch + wl + 1];
            const bool both = w0 + wl + 1 < words;
            if (both && ((uintptr_t)dst & 15) == 0) {
                *reinterpret_cast<u64x2*>(dst) = u64x2{v0, v1};
            } else {
                dst[0] = v0;
                if (both) dst[1] = v1;
            }
        }
    }
}

// LDS-tiled wires -> bits scattering circuit row p to row map(p) of `out`
// (the round's scatter fused into getOutput).
__global__ void __launch_bounds__(256) k_wires_to_bits_map(const u64* __restrict__ mem, u64 shareStride, u32 nbits,
                                                           u64 words, i64* __restrict__ out, u64 outRows, MapPair jobs,
                                                           u64 rows) {
    __shared__ u64 tile[64 * kTilePitch];
    const aby3g_rowmap& map = jobs.map[blockIdx.z];
    const u32* __restrict__ wires = jobs.wires[blockIdx.z];
    const u64 cols = (nbits + 63) / 64;
    mem += (u64)blockIdx.y * shareStride;
    out += (u64)blockIdx.y * outRows * cols;
    const u64 rw = (rows + 63) / 64;
    const u64 tilesPerCol = (rw + kTileWords - 1) / kTileWords;
    const u64 c = blockIdx.x / tilesPerCol, w0 = (blockIdx.x % tilesPerCol) * kTileWords;
    u64 vv[kWaveWords];  // 64 x kTileWords words over 256 threads, two words a thread per load (16 bytes)
#pragma unroll
    for (u32 j = 0; j < kWaveWords / 2; ++j) {
        const u32 idx = threadIdx.x + 256 * j, b = idx / (kTileWords / 2), wl = 2 * (idx % (kTileWords / 2));
        const u64 bit = c * 64 + b;
        u64x2 v = u64x2{0, 0};
        if (bit < nbits && w0 + wl < rw) {
            const u64* src = mem + (u64)wires[bit] * words + w0 + wl;
            const bool both = w0 + wl + 1 < rw;
            if (both && ((uintptr_t)src & 15) == 0)
                v = *reinterpret_cast<const u64x2*>(src);
            else
                v = u64x2{src[0], both ? src[1] : 0};
        }
        vv[2 * j] = v.x;
        vv[2 * j + 1] = v.y;
    }
#pragma unroll
    for (u32 j = 0; j < kWaveWords / 2; ++j) {
        const u32 idx = threadIdx.x + 256 * j, b = idx / (kTileWords / 2), wl = 2 * (idx % (kTileWords / 2));
        tile[b * kTilePitch + wl] = vv[2 * j];
        tile[b * kTilePitch + wl + 1] = vv[2 * j + 1];
    }
    __syncthreads();
    const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // unrolled, as in k_bits_to_wires_map: independent transposes in flight
#pragma unroll
    for (u32 k = 0; k < kWaveWords; ++k) vv[k] = transpose64(tile[lane * kTilePitch + wave * kWaveWords + k], lane);
    MapWalk mw = map_walk(map, (w0 + wave * kWaveWords) * 64 + lane);
#pragma unroll
    for (u32 k = 0; k < kWaveWords; ++k) {
        const u32 wl = wave * kWaveWords + k;
        const u64 row = (w0 + wl) * 64 + lane;
        if (w0 + wl < rw && row < rows) {
            const u64 dst = map_walk_row(map, mw);
            if (dst < outRows) out[dst * cols + c] = (i64)vv[k];
        }
        map_walk_next(map, mw);
    }
}

// Largest row an affine map reaches over p < rows (strides are unsigned, so
// the maximum is at the last element of the last or the next-to-last rep).
static u64 affine_max_row(const aby3g_rowmap& m, u64 rows) {
    const u64 q0 = m.first, q1 = m.first + rows - 1;
    const u64 r0 = q0 / m.per_rep, r1 = q1 / m.per_rep;
    u64 mx = m.start + r1 * m.rep_stride + (q1 % m.per_rep) * m.step;
    if (r1 > r0) mx = std::max(mx, m.start + (r1 - 1) * m.rep_stride + (m.per_rep - 1) * m.step);
    return mx;
}

static void check_map(const aby3g_rowmap* map, u64 rows, u64 limit) {
    ABY3G_REQUIRE(map != nullptr, "null row map");
    if (map->idx || !rows) return;  // explicit maps: out-of-range rows are skipped by the kernels
    ABY3G_REQUIRE(map->per_rep > 0, "row map: per_rep must be positive");
    ABY3G_REQUIRE(affine_max_row(*map, rows) < limit, "row map reaches past the matrix");
}

}  // namespace

}  // namespace aby3g

using namespace aby3g;

extern "C" {

int aby3g_bin_gates(const aby3g_gate* gates, uint32_t ngates, uint64_t* mem, uint64_t wires, uint64_t words,
                    const uint64_t* z, uint64_t* sendbuf, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(words % 32 == 0, "words must be padded to a multiple of 32 (2048 rows)");
        if (!ngates || !words) return;
        dim3 grid((u32)((words / 2 + kGateBlock - 1) / kGateBlock), ngates);
        launch(PROBE_BINARY, k_bin_gates, grid, dim3(kGateBlock), 0, S(stream), gates, mem, wires, words, z, sendbuf);
    });
}

int aby3g_bin_level(const aby3g_gate* gates, const uint32_t* batch_ends, uint32_t nbatches, const uint64_t* recvbuf,
                    const uint32_t* unpack_wires, uint32_t nunpack, uint64_t* mem, uint64_t wires, uint64_t words,
                    const uint64_t* z, uint64_t* sendbuf, aby3g_stream stream) {
    return aby3g_bin_level_rr(gates, nullptr, batch_ends, nbatches, recvbuf, unpack_wires, nunpack, mem, wires, words, z,
                              sendbuf, stream);
}

int aby3g_bin_level_rr(const aby3g_gate* gates, const uint32_t* recv_rows, const uint32_t* batch_ends,
                       uint32_t nbatches, const uint64_t* recvbuf, const uint32_t* unpack_wires, uint32_t nunpack,
                       uint64_t* mem, uint64_t wires, uint64_t words, const uint64_t* z, uint64_t* sendbuf,
                       aby3g_stream stream) {
    return aby3g_bin_level_hs(gates, recv_rows, batch_ends, nbatches, recvbuf, unpack_wires, nunpack, mem, wires, words,
                              z, sendbuf, nullptr, nullptr, stream);
}

static int bin_level(const aby3g_gate* gates, const uint32_t* recv_rows, const uint32_t* batch_ends,
                     uint32_t nbatches, const uint64_t* recvbuf, const uint32_t* unpack_wires, uint32_t nunpack,
                     uint64_t* mem, uint64_t wires, uint64_t words, const uint64_t* z, uint64_t* sendbuf,
                     const aby3g_handoff* wait, const aby3g_handoff* post, aby3g_stream stream) {
    const uint2* rrows = reinterpret_cast<const uint2*>(recv_rows);
    return guarded([&] {
        ABY3G_REQUIRE(!rrows || recvbuf, "recv_rows without a recv buffer");
        ABY3G_REQUIRE(words % kLevelWords == 0, "words must be padded to a multiple of 32 (2048 rows)");
        ABY3G_REQUIRE(!(wait && wait->flags) || nunpack, "a hand-off wait without received shares");
        ABY3G_REQUIRE(!(post && post->flags) || sendbuf, "a hand-off post without a send buffer");
        if ((!nbatches && !nunpack) || !words) return;
        // one workgroup per chunk; in-kernel hand-offs are used only for
        // launches of at most 64 chunks, or 512 from a light producer
        // (Channel::handoffPost), so the spinning workgroups of two parties'
        // launches never fill the device (4 of the 5 wave slots per SIMD)
        const u32 wgs = (u32)(words / kLevelWords);
        const HsWait hw = hs_wait_arg(wait);
        const HsPost hp = hs_post_arg(post);
        // few workgroups (small row counts): 32 slots per workgroup for gate parallelism
        const bool hs = hw.flags || hp.flags;
        // with hand-offs the send rows are stored write-through and the
        // received ones read past L1 (both ways, so one instantiation covers
        // a launch that only waits or only posts)
        if (wgs < kLevelSmallMaxWgs) {
            if (hs)
                launch(PROBE_BINARY, k_bin_level<32, true, 1>, dim3(wgs), dim3(32 * 32), 0, S(stream), gates, rrows,
                       batch_ends, nbatches, recvbuf, unpack_wires, nunpack, mem, wires, words, z, sendbuf, hw, hp);
            else
                launch(PROBE_BINARY, k_bin_level<32, false, 1>, dim3(wgs), dim3(32 * 32), 0, S(stream), gates, rrows,
                       batch_ends, nbatches, recvbuf, unpack_wires, nunpack, mem, wires, words, z, sendbuf, hw, hp);
        } else {
            // the hand-off form unrolls two gates a slot, not four: 74 VGPRs
            // against 130, six workgroups a CU against three, so that C3's
            // 512-chunk messages still pass the residency rule (C3 0.302-0.305
            // against 0.337-0.338 ms with the four-gate form and stream
            // hand-offs, and 0.308-0.311 with one word per lane)
            if (hs)
                launch(PROBE_BINARY, k_bin_level<8, true, 2, 2>, dim3(wgs), dim3(8 * 32), 0, S(stream), gates, rrows,
                       batch_ends, nbatches, recvbuf, unpack_wires, nunpack, mem, wires, words, z, sendbuf, hw, hp);
            else
                launch(PROBE_BINARY, k_bin_level<8, false, 2>, dim3(wgs), dim3(8 * 32), 0, S(stream), gates, rrows,
                       batch_ends, nbatches, recvbuf, unpack_wires, nunpack, mem, wires, words, z, sendbuf, hw, hp);
        }
    });
}

int aby3g_bin_level_hs(const aby3g_gate* gates, const uint32_t* recv_rows, const uint32_t* batch_ends,
                       uint32_t nbatches, const uint64_t* recvbuf, const uint32_t* unpack_wires, uint32_t nunpack,
                       uint64_t* mem, uint64_t wires, uint64_t words, const uint64_t* z, uint64_t* sendbuf,
                       const aby3g_handoff* wait, const aby3g_handoff* post, aby3g_stream stream) {
    return bin_level(gates, recv_rows, batch_ends, nbatches, recvbuf, unpack_wires, nunpack, mem, wires, words, z,
                     sendbuf, wait, post, stream);
}

int aby3g_bin_level_residency(int* cus, int* per_cu_small, int* per_cu_large, int* small_max_wgs) {
    return guarded([&] {
        ABY3G_REQUIRE(cus && per_cu_small && per_cu_large && small_max_wgs, "null argument");
        const int dev = current_device();
        ABY3G_CHECK_HIP(hipDeviceGetAttribute(cus, hipDeviceAttributeMultiprocessorCount, dev));
        // the consumers that spin: the hand-off instantiations of the level
        // kernel, one chunk per workgroup (the only in-kernel waiters of the
        // binary engine)
        int a = 0;
        ABY3G_CHECK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &a, reinterpret_cast<const void*>(k_bin_level<32, true, 1>), 32 * 32, 0));
        *per_cu_small = a;
        ABY3G_CHECK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &a, reinterpret_cast<const void*>(k_bin_level<8, true, 2, 2>), 8 * 32, 0));
        *per_cu_large = a;
        *small_max_wgs = (int)kLevelSmallMaxWgs;
    });
}

int aby3g_bin_unpack(const uint64_t* recvbuf, const uint32_t* out_wires, uint32_t n, uint64_t* mem, uint64_t wires,
                     uint64_t words, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(words % 32 == 0, "words must be padded to a multiple of 32 (2048 rows)");
        if (!n || !words) return;
        dim3 grid((u32)((words / 2 + kGateBlock - 1) / kGateBlock), n);
        launch(PROBE_BINARY, k_bin_unpack, grid, dim3(kGateBlock), 0, S(stream), recvbuf, out_wires, mem, wires,
               words);
    });
}

static void bits_to_wires(const int64_t* in, u64 rows, u64 cols64, u32 nbits, u64* wire_rows, u64 shareStride,
                          u32 shares, u64 words, hipStream_t s) {
    ABY3G_REQUIRE(nbits <= cols64 * 64, "nbits exceeds input columns");
    ABY3G_REQUIRE(words * 64 >= rows, "words too small for rows");
    if (!nbits || !words) return;
    u64 waves = words * cols64;
    launch(PROBE_OTHER, k_bits_to_wires, dim3((u32)((waves * 64 + 255) / 256), shares), dim3(256), 0, s, in, rows,
           cols64, nbits, wire_rows, shareStride, words);
}

static void wires_to_bits(const u64* mem, u64 shareStride, u32 shares, const u32* wires, u32 nbits, u64 words,
                          int64_t* out, u64 rows, hipStream_t s) {
    ABY3G_REQUIRE(words * 64 >= rows, "words too small for rows");
    if (!nbits || !rows) return;
    u64 waves = ((rows + 63) / 64) * ((nbits + 63) / 64);
    launch(PROBE_OTHER, k_wires_to_bits, dim3((u32)((waves * 64 + 255) / 256), shares), dim3(256), 0, s, mem,
           shareStride, wires, nbits, words, out, rows);
}

int aby3g_bits_to_wires(const int64_t* in, uint64_t rows, uint64_t cols64, uint32_t nbits, uint64_t* wire_rows,
                        uint64_t words, aby3g_stream stream) {
    return guarded([&] { bits_to_wires(in, rows, cols64, nbits, wire_rows, 0, 1, words, S(stream)); });
}

int aby3g_bits_to_wires2(const int64_t* in, uint64_t rows, uint64_t cols64, uint32_t nbits, uint64_t* wire_rows,
                         uint64_t share_stride, uint64_t words, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(nbits <= cols64 * 64, "nbits exceeds input columns");
        ABY3G_REQUIRE(words * 64 >= rows, "words too small for rows");
        if (!nbits || !words) return;
        const u64 wgs = ((words + 63) / 64) * ((nbits + 63) / 64);
        launch(PROBE_OTHER, k_b2w_regs, dim3((u32)wgs, 2), dim3(64), 0, S(stream), in, rows, cols64, nbits, wire_rows,
               share_stride, words);
    });
}

int aby3g_bits_to_wires_lin(const aby3g_wire_src* srcs, uint32_t nsrc, uint64_t rows, uint64_t words,
                            aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(nsrc <= ABY3G_WIRE_SRC_MAX, "too many sources");
        ABY3G_REQUIRE(words * 64 >= rows, "words too small for rows");
        if (!nsrc || !words) return;
        WireSrcs ws{};
        u64 cols = 0;
        for (u32 k = 0; k < nsrc; ++k) {
            ABY3G_REQUIRE(srcs[k].wire_rows != nullptr, "null wire rows");
            ABY3G_REQUIRE(srcs[k].nbits <= srcs[k].cols64 * 64, "nbits exceeds input columns");
            ws.s[k] = srcs[k];
            cols = std::max<u64>(cols, (srcs[k].nbits + 63) / 64);
        }
        if (!cols) return;
        const u64 wgs = ((words + 63) / 64) * cols;
        launch(PROBE_OTHER, k_b2w_lin_regs, dim3((u32)wgs, nsrc), dim3(64), 0, S(stream), ws, (u64)rows, (u64)words);
    });
}

int aby3g_lin_copy_out(const aby3g_wire_src* srcs, uint32_t nsrc, uint64_t rows, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(nsrc <= ABY3G_WIRE_SRC_MAX, "too many sources");
        WireSrcs ws{};
        u64 n = 0;
        for (u32 k = 0; k < nsrc; ++k) {
            ws.s[k] = srcs[k];
            if (srcs[k].copy_out) n = std::max<u64>(n, rows * srcs[k].cols64);
        }
        if (!n) return;
        launch(PROBE_OTHER, k_lin_copy, dim3((u32)((n + 511) / 512)), dim3(256), 0, S(stream), ws, nsrc, (u64)rows);
    });
}

int aby3g_bin_level_in(const aby3g_wire_src* srcs, uint32_t nsrc, uint64_t rows, uint32_t in_lo, uint32_t in_hi,
                       int write_inputs, const aby3g_gate* gates, const uint32_t* batch_ends, uint32_t nbatches,
                       uint64_t* mem, uint64_t wires, uint64_t words, const uint64_t* z, uint64_t* sendbuf,
                       const aby3g_handoff* post, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(nsrc <= ABY3G_WIRE_SRC_MAX, "too many sources");
        ABY3G_REQUIRE(words % kLevelWords == 0, "words must be padded to a multiple of 32 (2048 rows)");
        ABY3G_REQUIRE(words * 64 >= rows, "words too small for rows");
        ABY3G_REQUIRE(in_lo <= in_hi && in_hi - in_lo <= kInMax && in_hi <= wires, "input wires out of range");
        ABY3G_REQUIRE(!(post && post->flags) || sendbuf, "a hand-off post without a send buffer");
        if (!words) return;
        const u64 shareStride = wires * words;
        LevelInSrcs ls{};
        u32 nl = 0;  // sources with terms, in LDS-slot order
        for (u32 k = 0; k < nsrc; ++k) {
            const aby3g_wire_src& s = srcs[k];
            ABY3G_REQUIRE(s.wire_rows != nullptr, "null wire rows");
            ABY3G_REQUIRE(s.cols64 == 1 && s.nbits <= 64, "fused inputs take one 64-bit column per source");
            ABY3G_REQUIRE(s.copy_out == nullptr, "copy_out: call aby3g_lin_copy_out first");
            const u64 off = (u64)(s.wire_rows - mem);
            ABY3G_REQUIRE(s.wire_rows >= mem && off % words == 0 && off / words < 2 * wires, "wire_rows outside mem");
            if (!s.term[0] && !s.term[1] && !s.term[2] && !s.term[3]) {
                // all zero: no LDS (aby3g_bits_to_wires_lin applies a constant
                // even without terms; this form does not)
                ABY3G_REQUIRE(s.constant == 0, "a source without terms must have a zero constant here");
                continue;
            }
            LevelInSrc& d = ls.s[nl++];
            for (int t = 0; t < 4; ++t) {
                d.term[t] = (const u64*)s.term[t];
                d.coef[t] = (u64)s.coef[t];
            }
            d.constant = (u64)s.constant;
            d.share = (u32)(off / shareStride);
            d.wire = (u32)((off % shareStride) / words);
            d.nbits = s.nbits;
            ABY3G_REQUIRE(d.wire >= in_lo && d.wire + d.nbits <= in_hi, "source wires outside [in_lo, in_hi)");
        }
        const u32 wgs = (u32)(words / kLevelWords);
        const HsPost hp = hs_post_arg(post);
        const u32 nin = in_hi - in_lo;
        const size_t lds = (size_t)nl * 64 * kLevelWords * 8;
        static const bool attr = [] {  // up to 8 sources (128 KiB) of dynamic LDS, once per process
            bool ok = true;
            for (const void* f : {(const void*)k_bin_level_in<32, true, 1>, (const void*)k_bin_level_in<32, false, 1>,
                                  (const void*)k_bin_level_in<8, true, 2>, (const void*)k_bin_level_in<8, false, 2>})
                ok = ok && hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 128 << 10) == hipSuccess;
            return ok;
        }();
        ABY3G_REQUIRE(attr || lds <= (64 << 10), "could not raise the fused level's dynamic LDS limit");
        nsrc = nl;
        if (wgs < kLevelSmallMaxWgs) {
            if (hp.flags)
                launch(PROBE_BINARY, k_bin_level_in<32, true, 1>, dim3(wgs), dim3(32 * 32), lds, S(stream), ls, nsrc,
                       (u64)rows, in_lo, nin, write_inputs, gates, batch_ends, nbatches, mem, wires, words, z, sendbuf,
                       hp);
            else
                launch(PROBE_BINARY, k_bin_level_in<32, false, 1>, dim3(wgs), dim3(32 * 32), lds, S(stream), ls, nsrc,
                       (u64)rows, in_lo, nin, write_inputs, gates, batch_ends, nbatches, mem, wires, words, z, sendbuf,
                       hp);
        } else {
            if (hp.flags)
                launch(PROBE_BINARY, k_bin_level_in<8, true, 2>, dim3(wgs), dim3(8 * 32), lds, S(stream), ls, nsrc,
                       (u64)rows, in_lo, nin, write_inputs, gates, batch_ends, nbatches, mem, wires, words, z, sendbuf,
                       hp);
            else
                launch(PROBE_BINARY, k_bin_level_in<8, false, 2>, dim3(wgs), dim3(8 * 32), lds, S(stream), ls, nsrc,
                       (u64)rows, in_lo, nin, write_inputs, gates, batch_ends, nbatches, mem, wires, words, z, sendbuf,
                       hp);
        }
    });
}

int aby3g_wires_to_bits(const uint64_t* mem_share, const uint32_t* wires, uint32_t nbits, uint64_t words, int64_t* out,
                        uint64_t rows, aby3g_stream stream) {
    return guarded([&] { wires_to_bits(mem_share, 0, 1, wires, nbits, words, out, rows, S(stream)); });
}

int aby3g_wires_to_bits2(const uint64_t* mem, uint64_t share_stride, const uint32_t* wires, uint32_t nbits,
                         uint64_t words, int64_t* out, uint64_t rows, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(words * 64 >= rows, "words too small for rows");
        if (!nbits || !rows) return;
        if (nbits <= 8) {
            launch(PROBE_OTHER, k_w2b_few, dim3((u32)((rows + 511) / 512), 2), dim3(256), 0, S(stream), mem,
                   (u64)share_stride, wires, nbits, (u64)words, out, (u64)rows);
            return;
        }
        const u64 wgs = (((rows + 63) / 64 + 63) / 64) * ((nbits + 63) / 64);
        launch(PROBE_OTHER, k_w2b_regs, dim3((u32)wgs, 2), dim3(64), 0, S(stream), mem, (u64)share_stride, wires, nbits,
               (u64)words, out, (u64)rows);
    });
}

int aby3g_bits_to_wires_map(const int64_t* in, uint64_t in_rows, uint64_t cols64, uint32_t nbits,
                            const aby3g_rowmap* map, uint64_t rows, uint64_t* wire_rows, uint64_t share_stride,
                            uint64_t words, aby3g_stream stream) {
    return aby3g_bits_to_wires_map_n(in, in_rows, cols64, nbits, map, &wire_rows, 1, rows, share_stride, words, stream);
}

int aby3g_bits_to_wires_map_n(const int64_t* in, uint64_t in_rows, uint64_t cols64, uint32_t nbits,
                              const aby3g_rowmap* maps, uint64_t* const* wire_rows, uint32_t n, uint64_t rows,
                              uint64_t share_stride, uint64_t words, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(n >= 1 && n <= 2, "one or two maps per call");
        ABY3G_REQUIRE(maps != nullptr && wire_rows != nullptr, "null argument");
        ABY3G_REQUIRE(nbits <= cols64 * 64, "nbits exceeds input columns");
        ABY3G_REQUIRE(words * 64 >= rows, "words too small for rows");
        MapPair jobs{};
        for (u32 k = 0; k < n; ++k) {
            check_map(&maps[k], rows, in_rows);
            jobs.map[k] = maps[k];
            jobs.wrows[k] = wire_rows[k];
        }
        if (!nbits || !words) return;
        const u64 tiles = ((words + kTileWords - 1) / kTileWords) * ((nbits + 63) / 64);
        launch(PROBE_OTHER, k_bits_to_wires_map, dim3((u32)tiles, 2, n), dim3(256), 0, S(stream), in, (u64)in_rows,
               (u64)cols64, nbits, jobs, (u64)rows, (u64)share_stride, (u64)words);
    });
}

int aby3g_wires_to_bits_map(const uint64_t* mem, uint64_t share_stride, const uint32_t* wires, uint32_t nbits,
                            uint64_t words, int64_t* out, uint64_t out_rows, const aby3g_rowmap* map, uint64_t rows,
                            aby3g_stream stream) {
    return aby3g_wires_to_bits_map_n(mem, share_stride, &wires, nbits, words, out, out_rows, map, 1, rows, stream);
}

int aby3g_wires_to_bits_map_n(const uint64_t* mem, uint64_t share_stride, const uint32_t* const* wires,
                              uint32_t nbits, uint64_t words, int64_t* out, uint64_t out_rows,
                              const aby3g_rowmap* maps, uint32_t n, uint64_t rows, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(n >= 1 && n <= 2, "one or two maps per call");
        ABY3G_REQUIRE(maps != nullptr && wires != nullptr, "null argument");
        ABY3G_REQUIRE(words * 64 >= rows, "words too small for rows");
        MapPair jobs{};
        for (u32 k = 0; k < n; ++k) {
            check_map(&maps[k], rows, out_rows);
            jobs.map[k] = maps[k];
            jobs.wires[k] = wires[k];
        }
        if (!nbits || !rows) return;
        const u64 tiles = (((rows + 63) / 64 + kTileWords - 1) / kTileWords) * ((nbits + 63) / 64);
        launch(PROBE_OTHER, k_wires_to_bits_map, dim3((u32)tiles, 2, n), dim3(256), 0, S(stream), mem,
               (u64)share_stride, nbits, (u64)words, out, (u64)out_rows, jobs, (u64)rows);
    });
}

}  // extern "C"
