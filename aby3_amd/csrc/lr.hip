// One SGD_Logistic iteration (aby3-ML/Regression.h:249-293) of one party as
// ONE launch of one workgroup, for three parties co-located on one device
// (aby3g_lr_iteration, include/aby3gpu.h).
//
// The op-by-op path issues ~35 launches and ~17 stream hand-offs per party
// and iteration on a batch of 256 rows: every step is a few microseconds of
// work behind a launch and a hand-off. Here the whole iteration runs inside
// one workgroup per party, phase after phase, and the parties' messages go
// through mailboxes with the in-kernel hand-off of common.h (write-through
// payload, one flag per message and epoch, polled by one lane). The
// randomness is drawn exactly where the op-by-op path draws it (stream
// positions, draw indices and OT counters come from the host), so the shares
// are bit-identical to that path's -- tests/test_lr_driver.py holds both
// against the oracle.
//
// Phases (reference lines):
//   0  AND masks of the circuit: z[k][w] = draw k * words + w of the setCir
//      keys (Sh3BinaryEvaluator.cpp:1406-1434), only the words with rows
//   1  xw = mul(XX, w) >> D: the batch rows gathered on the fly
//      (extractBatch, Regression.h:42-58), the share product
//      XX0 (w0 + w1) + XX1 w0, the truncation pair, z to P0 / P1, the
//      finalize (Sh3Evaluator.cpp:651-730)
//   2  regions = int_Sh3Piecewise_helper(xw): P0 reshares x0 + x2 to P1, the
//      inputs are bit-sliced straight into the circuit's wires, the levels
//      run with one message per level (Sh3Piecewise.cpp:381-516,
//      Sh3BinaryEvaluator.cpp:539-1196)
//   3  f = region1 * (half + slope x) [OT product, Sh3Evaluator.cpp:119-263]
//        + region2 * one [public product, :418-501]
//   4  err = f - YY; update = mulTruncate(XX^T, err, aB); w -= update
#include "common.h"

namespace aby3g {

namespace {

constexpr u32 kLrThreads = 512;
constexpr u32 kLrWaves = kLrThreads / 64;
constexpr u32 kLrMaxB = 2048;
constexpr u32 kLrMaxD = 4096;
// the circuit's engine memory and AND masks live in LDS (beside the 64 KiB
// AES table) when they fit: the levels' gate batches are chains of dependent
// word accesses, at LDS instead of L2 latency
constexpr u64 kLrDynLdsMax = 88 << 10;

// mailbox flags (one u64 each), all within a workgroup's own mailbox: F_H1 /
// F_H2 the helper workgroups' arrival counters (epoch * helpers once every
// helper published), F_ERR workgroup 0's err vector published to its helpers
// and F_P3 its start of phase 3, a hint for the helpers' polling (value =
// epoch). Between the parties there are no flags: every message word
// carries the epoch itself (msg_put / msg_get).
// (each on a 128-byte line of its own: 16 helpers poll F_ERR while block 0
// polls F_H1 / F_H2 and the helpers add to them)
enum : u32 { F_H1 = 0, F_H2 = 16, F_ERR = 32, F_P3 = 48, kLrFlags = 64 };

// Helper workgroups (blocks 1..G of the launch): the two dataset products
// gather the batch rows from all over the dataset, which one CU does at a few
// tens of GB/s; G CUs split the rows instead (kLrHelperRows each). Block 0
// runs the protocol as before and meets them through its own mailbox.
constexpr u32 kLrHelperRows = 16;
constexpr u32 kLrMaxHelpers = 32;
__host__ __device__ inline u32 lr_helpers(u32 B) {
    const u32 g = (B + kLrHelperRows - 1) / kLrHelperRows;
    return g > kLrMaxHelpers ? kLrMaxHelpers : g;
}

// The expanded AES keys of an iteration (kernel argument).
struct LrKeys {
    AesKey prev, next;      // the ShareGen streams
    AesKey zsp, zsn;        // zero-share keys
    AesKey mp, mn;          // circuit masks (setCir)
    AesKey otn, otp;        // SharedOT keys
    AesKey mp2, mn2;        // the next iteration's circuit masks (drawn ahead)
};

// Block 0 copies the schedules into LDS (AesRkLds): as kernel arguments the
// eight of them spill out of SGPRs (loaded up front, one dependent scalar load
// per 64 bytes: ~7 us at the start of every launch).
enum : u32 { kKeyPrev, kKeyNext, kKeyZsp, kKeyZsn, kKeyMp, kKeyMn, kKeyOtn, kKeyOtp, kKeyMp2, kKeyMn2, kLrKeys };
constexpr u32 kKeyWords = 44;
static_assert(sizeof(LrKeys) == kLrKeys * kKeyWords * 4, "LrKeys is the schedules in kKey order");

// Pads of the OT and public products per batch row drawn ahead (the most any
// party uses: P0's 7 OT-product words and 5 public-product words).
constexpr u64 kPads = 12;

// Mailbox and scratch layouts, in u64 words.
struct Layout {
    u64 W, Wpad;
    // mailbox: flags, then two regions (epoch parity)
    u64 flags, region;
    u64 z1, v, lvl, ots, oth, otc, pma, pmb, z2;
    // scratch
    u64 xw, a, fr, f2, yy, err, z1own, z2own, upd, reg, zmask, mem, prod, hprod, hy, hpart, total;
    // randomness drawn ahead: two slots (epoch parity), each the circuit's
    // masks, the two truncation pairs' stream words and the OT / public
    // product pads (kPads words per batch row, party-specific)
    u64 pre, preSlot, pzm, ptw1, ptw2, ppad;
    __host__ __device__ Layout(u32 B, u32 d, const aby3g_lr_circuit& c) {
        W = (B + 63) / 64;
        Wpad = 32 * (((u64)B + 2047) / 2048);
        flags = ((kLrFlags + 31) / 32) * 32;
        // messages: two {epoch, 32-bit half} granules per 64-bit word
        u64 o = 0;
        z1 = o, o += 2 * (u64)B;
        v = o, o += 2 * (u64)B;
        lvl = o, o += 2 * (u64)c.nand * W;
        ots = o, o += 4 * (u64)B;
        oth = o, o += 2 * (u64)B;
        otc = o, o += 2 * (u64)B;
        pma = o, o += 4 * (u64)B;
        pmb = o, o += 4 * (u64)B;
        z2 = o, o += 2 * (u64)d;
        region = (o + 31) / 32 * 32;
        o = 0;
        xw = o, o += 2 * (u64)B;
        a = o, o += 2 * (u64)B;
        fr = o, o += 2 * (u64)B;
        f2 = o, o += 2 * (u64)B;
        yy = o, o += 2 * (u64)B;
        err = o, o += 2 * (u64)B;
        z1own = o, o += B;
        z2own = o, o += d;
        upd = o, o += 2 * (u64)d;
        reg = o, o += 6 * (u64)B;
        zmask = o, o += (u64)c.nand * W;
        mem = o, o += 2 * (u64)c.wires * W;
        prod = o, o += (B > d ? B : d);
        hprod = o, o += B;                          // helpers: XX w products, one per batch row
        hy = o, o += 2 * (u64)B;                    // helpers: YY (both shares)
        hpart = o, o += (u64)lr_helpers(B) * d;     // helpers: partial XX^T err, one d-vector each
        pzm = 0;
        ptw1 = pzm + (u64)c.nand * W;               // next-stream words [B], prev-stream words [B]
        ptw2 = ptw1 + 2 * (u64)B;                   // the same for the second pair [d], [d]
        ppad = ptw2 + 2 * (u64)d;                   // pads [kPads][B]
        preSlot = ppad + kPads * (u64)B;
        pre = o, o += 2 * preSlot;
        total = o;
    }
    __host__ __device__ u64 mailboxWords() const { return flags + 2 * region; }
};

static_assert(kLrThreads == 512, "the XtE reduction adds eight waves' partial sums in two halves of part[]");

struct u64x2 {
    u64 x, y;
};
// p[0], p[1] (p[1] only when `pair`): one 16-byte load when p is 16-byte aligned
__device__ __forceinline__ u64x2 load_pair(const u64* p, bool pair) {
    if (pair && !((uintptr_t)p & 15)) {
        typedef u64 v2u64 __attribute__((ext_vector_type(2)));
        const v2u64 v = *reinterpret_cast<const v2u64*>(p);
        return u64x2{v.x, v.y};
    }
    return u64x2{p[0], pair ? p[1] : 0};
}

// NB AES-CTR blocks under LDS key schedules (keys[kKey...] + counters)
template <int NB>
__device__ __forceinline__ void lr_blocks(const u32* T, const u32* const (&k)[NB], const u64 (&c)[NB], u64 (&lo)[NB],
                                          u64 (&hi)[NB]) {
    aes_ctr_blocks_rk<NB>(T, threadIdx.x & 31, AesRkLds{k}, c, lo, hi);
}

// word j of PRNG(k): half (j & 1) of AES(k, j >> 1)
__device__ __forceinline__ u64 stream_word(const u32* T, const u32* k, u64 j) {
    u64 lo[1], hi[1];
    lr_blocks<1>(T, {k}, {j >> 1}, lo, hi);
    return (j & 1) ? hi[0] : lo[0];
}

// waits for a neighbour's flag `f` (one lane polls; the workgroup leaves
// together); false after a timeout
__device__ __forceinline__ bool lr_wait(const u64* box, u32 f, u64 epoch, u64* ticks, const HsStatus& status) {
    return hs_wait(HsWait{box, epoch, ticks, status}, f, f + 1);
}
// publishes this party's flag `f` after every wave's write-through stores
__device__ __forceinline__ void lr_post(u64* box, u32 f, u64 epoch) { hs_post(HsPost{box, epoch}, f, f + 1); }

// Messages between the parties in the granule form of the in-kernel hand-off
// (cdna_hip_programming.md Guideline 16, R2): word i of a message array m is
// m[2i] = {epoch, low half}, m[2i + 1] = {epoch, high half}, stored
// write-through; the reader polls the words themselves until both halves
// carry this epoch -- no drain, no flag and no second round trip for the
// payload. The mailbox regions alternate by epoch parity, so a word left from
// two epochs before never matches.
// Peers on this device (in this process or another, through an IPC mapping)
// share its L2s: agent-scope write-through stores and L1-bypassing loads.
// Peers on other GPUs read this party's mailbox over xGMI: system scope
// (aby3g_lr_iter.sys_scope), the mailboxes allocated uncached.
struct MsgTag {
    u32 tag;
    bool sys;
};
__device__ __forceinline__ void msg_store(u64* p, u64 v, bool sys) {
    if (sys)
        __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else
        hs_store(p, v);
}
__device__ __forceinline__ u64 msg_load(const u64* p, bool sys) {
    if (sys) return __hip_atomic_load((const gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return hs_load(p);
}
__device__ __forceinline__ void msg_put(u64* m, u64 i, u64 v, MsgTag tag) {
    msg_store(m + 2 * i, ((u64)tag.tag << 32) | (u32)v, tag.sys);
    msg_store(m + 2 * i + 1, ((u64)tag.tag << 32) | (u32)(v >> 32), tag.sys);
}
// A thread's reads of one receive loop: after a timeout or an abort (another
// wait timed out) it stops polling and the workgroup leaves together at
// msg_done.
struct MsgWait {
    u32 tag;
    bool sys;
    HsStatus status;
    u64 t0;
    bool ok;
};
__device__ __forceinline__ MsgWait msg_begin(MsgTag tag, const HsStatus& status) {
    return MsgWait{tag.tag, tag.sys, status, (u64)wall_clock64(), true};
}
__device__ __forceinline__ u64 msg_get(const u64* m, u64 i, MsgWait& w) {
    if (!w.ok) return 0;
    for (u32 spins = 0;;) {
        const u64 a = msg_load(m + 2 * i, w.sys), b = msg_load(m + 2 * i + 1, w.sys);
        if ((u32)(a >> 32) == w.tag && (u32)(b >> 32) == w.tag) return (u64)(u32)a | ((u64)(u32)b << 32);
        __builtin_amdgcn_s_sleep(1);
        if ((++spins & 63) == 0) {
            if (hs_failed(w.status)) break;
            if (wall_clock64() - w.t0 > w.status.limit) {
                hs_fail(w.status);
                break;
            }
        }
    }
    w.ok = false;
    return 0;
}
// the end of a receive loop (a workgroup barrier): false when any thread's
// read failed; thread 0 adds the loop's time to the wait ticks
__device__ __forceinline__ bool msg_done(const MsgWait& w, u32* bad, u64* ticks) {
    if (!w.ok) *bad = 1;
    if (threadIdx.x == 0 && ticks)
        __hip_atomic_fetch_add((gu64*)ticks, wall_clock64() - w.t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    return *bad == 0;
}

// The truncation pair over n elements (Sh3Evaluator.cpp:503-566, 667-673):
// t0 = next-stream word (nw0 + i), t1 = prev-stream word (pw0 + i);
// z = prod - (t0 >> 2) published into `out` (write-through) and kept in own,
// C = (t0 >> (d+2), t1 >> (d+2)) into c0 / c1.
// Tiles of 256 elements: an AES block holds two consecutive stream words, so
// a tile needs at most 129 blocks of each stream -- threads [0, 256) draw the
// next stream's, [256, 512) the prev stream's, one block each, into tw (512
// u64 of LDS), then the tile's elements are formed from it.
// pw: the stream words drawn ahead (pw[i] next, pw[n + i] prev), or null.
__device__ __forceinline__ void lr_trunc_pair(const u32* T, const u32* keys, u64 nw0, u64 pw0, u32 n, u32 d,
                                              const u64* prod, u64* out, MsgTag tag, u64* own, u64* c0, u64* c1,
                                              u64* tw, const u64* pw) {
    const u32 tid = threadIdx.x, half = tid >> 8, t = tid & 255;
    if (pw) {
        for (u32 i = tid; i < n; i += kLrThreads) {
            const i64 t0 = (i64)pw[i], t1 = (i64)pw[n + i];
            const u64 z = prod[i] - (u64)(t0 >> 2);
            own[i] = z;
            msg_put(out, i, z, tag);
            c0[i] = (u64)(t0 >> (d + 2));
            c1[i] = (u64)(t1 >> (d + 2));
        }
        __syncthreads();
        return;
    }
    for (u32 i0 = 0; i0 < n; i0 += 256) {
        const u32 nt = min(256u, n - i0);
        const u64 w0 = (half ? pw0 : nw0) + i0;  // this half's first stream word of the tile
        const u64 b = (w0 >> 1) + t;              // block t of it
        if (b <= ((w0 + nt - 1) >> 1)) {
            u64 lo[1], hi[1];
            lr_blocks<1>(T, {keys + (half ? kKeyPrev : kKeyNext) * kKeyWords}, {b}, lo, hi);
            const u64 j = 2 * b - w0;  // tile position of the block's low word (-1: before the tile)
            if (2 * b >= w0) tw[half * 256 + j] = lo[0];
            if (j + 1 < nt) tw[half * 256 + j + 1] = hi[0];
        }
        __syncthreads();
        if (tid < nt) {
            const u32 i = i0 + tid;
            const i64 t0 = (i64)tw[tid], t1 = (i64)tw[256 + tid];
            const u64 z = prod[i] - (u64)(t0 >> 2);
            own[i] = z;
            msg_put(out, i, z, tag);
            c0[i] = (u64)(t0 >> (d + 2));
            c1[i] = (u64)(t1 >> (d + 2));
        }
        __syncthreads();
    }
}

// Round 2 of the truncating product, parties 0 and 1 (Sh3Evaluator.cpp:
// 703-719): C[party] += (z_next + z_prev + z_own) >> d.
__device__ __forceinline__ void lr_trunc_finalize(const u64* zn, const u64* zp, const u64* own, u32 n, u32 d,
                                                  u64* cp, MsgWait& w) {
    for (u32 i = threadIdx.x; i < n; i += kLrThreads) {
        const i64 s = (i64)(msg_get(zn, i, w) + msg_get(zp, i, w) + own[i]);
        cp[i] += (u64)(s >> d);
    }
}

// An agent-scope acquire for the whole workgroup (cdna_hip_programming.md
// Guideline 16): one lane's fence drops this CU's stale L1 lines, its wait and
// the barrier put every wave's later plain loads behind it.
__device__ __forceinline__ void lr_acquire() {
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

// Every storing wave drains its write-through stores, then one lane adds 1 to
// counter f of the own mailbox (the arrival of one helper).
__device__ __forceinline__ void lr_arrive(u64* box, u32 f) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add((gu64*)box + f, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The next iteration's randomness, drawn by the helper workgroups into
// scratch slot `slot` (aby3g_lr_iter.pre_next) exactly as block 0 would draw
// it -- the circuit's masks, the stream words of the two truncation pairs and
// the OT / public-product pads of this party -- so that the next launch's
// protocol workgroup only reads it. One work item per thread, strided over
// the G helpers: a mask pair of words, a stream word, or a batch row's pads.
__device__ __forceinline__ void lr_predraw(const aby3g_lr_iter& it, const u32* T, const u32* keys, u64* slot,
                                           const Layout& L) {
    const aby3g_lr_rand& r = it.next_rand;
    const u32 B = it.B, d = it.d, G = lr_helpers(B);
    const u64 W = L.W, Wh = (W + 1) / 2;
    const int p = it.party;
    auto KL = [&](u32 key) -> const u32* { return keys + key * kKeyWords; };
    const u64 q0 = (u64)(blockIdx.x - 1) * kLrThreads + threadIdx.x, qs = (u64)G * kLrThreads;
    // masks: words 2 wp, 2 wp + 1 of AND gate k (as phase 0)
    for (u64 q = q0; q < (u64)it.cir.nand * Wh; q += qs) {
        asm volatile("" ::: "memory");  // keeps the round-key reads in the loop (hoisted, they held ~90 VGPRs)
        const u64 k = q / Wh, wp = q % Wh;
        const u64 c = (k * L.Wpad + 2 * wp) >> 1;
        u64 lo[2], hi[2];
        lr_blocks<2>(T, {KL(kKeyMp2), KL(kKeyMn2)}, {c, c}, lo, hi);
        slot[L.pzm + k * W + 2 * wp] = lo[0] ^ lo[1];
        if (2 * wp + 1 < W) slot[L.pzm + k * W + 2 * wp + 1] = hi[0] ^ hi[1];
    }
    // truncation-pair stream words: [next B | prev B] then [next d | prev d]
    for (u64 q = q0; q < 2 * ((u64)B + d); q += qs) {
        asm volatile("" ::: "memory");  // keeps the round-key reads in the loop (hoisted, they held ~90 VGPRs)
        const bool second = q >= 2 * (u64)B;
        const u64 e = second ? q - 2 * (u64)B : q;
        const u32 n = second ? d : B;
        const bool prev = e >= n;
        const u64 off = second ? (prev ? r.t2_prev_off : r.t2_next_off) : (prev ? r.t1_prev_off : r.t1_next_off);
        slot[(second ? L.ptw2 : L.ptw1) + e] = stream_word(T, KL(prev ? kKeyPrev : kKeyNext), off / 8 + (prev ? e - n : e));
    }
    // batch row i's pads (phase 3): the OT product's, then the public product's
    u64* pad = slot + L.ppad;
    for (u64 q = q0; q < B; q += qs) {
        asm volatile("" ::: "memory");  // keeps the round-key reads in the loop (hoisted, they held ~90 VGPRs)
        const u32 i = (u32)q;
        if (p == 0) {
            const u64 otw = r.ot_prev_off / 8, wz = otw + 2 * i, wc = wz + 1, wn = r.ot_next_off / 8 + i;
            u64 lo[3], hi[3];
            lr_blocks<3>(T, {KL(kKeyPrev), KL(kKeyPrev), KL(kKeyNext)}, {wz >> 1, wc >> 1, wn >> 1}, lo, hi);
            pad[0 * B + i] = (wz & 1) ? hi[0] : lo[0];
            pad[1 * B + i] = (wc & 1) ? hi[1] : lo[1];
            pad[2 * B + i] = (wn & 1) ? hi[2] : lo[2];
            u64 l2[2], h2[2];
            lr_blocks<2>(T, {KL(kKeyOtn), KL(kKeyOtn)}, {r.ot_ctr + i, r.ot_ctr + B + i}, l2, h2);
            pad[3 * B + i] = l2[0];
            pad[4 * B + i] = h2[0];
            pad[5 * B + i] = l2[1];
            pad[6 * B + i] = h2[1];
        } else if (p == 1) {
            const u64 wf = r.ot_prev_off / 8 + i, j = r.pm_draw + i;
            u64 lo[3], hi[3];
            lr_blocks<3>(T, {KL(kKeyPrev), KL(kKeyZsp), KL(kKeyZsn)}, {wf >> 1, j >> 1, j >> 1}, lo, hi);
            pad[0 * B + i] = (wf & 1) ? hi[0] : lo[0];
            pad[1 * B + i] = (j & 1) ? hi[1] - hi[2] : lo[1] - lo[2];
        } else {
            const u64 otw = r.ot_next_off / 8, wz = otw + 2 * i, wc = wz + 1;
            u64 l2[2], h2[2];
            lr_blocks<2>(T, {KL(kKeyNext), KL(kKeyNext)}, {wz >> 1, wc >> 1}, l2, h2);
            pad[0 * B + i] = (wz & 1) ? h2[0] : l2[0];
            pad[1 * B + i] = (wc & 1) ? h2[1] : l2[1];
            lr_blocks<2>(T, {KL(kKeyOtp), KL(kKeyOtp)}, {r.ot_ctr + i, r.ot_ctr + B + i}, l2, h2);
            pad[2 * B + i] = l2[0];
            pad[3 * B + i] = h2[0];
            pad[4 * B + i] = l2[1];
            pad[5 * B + i] = h2[1];
        }
    }
    for (u64 q = q0; q < B; q += qs) {
        asm volatile("" ::: "memory");  // keeps the round-key reads in the loop (hoisted, they held ~90 VGPRs)
        const u32 i = (u32)q;
        const u64 j = r.pm_draw + i;
        u64 l2[2], h2[2];
        if (p == 0) {
            lr_blocks<2>(T, {KL(kKeyZsp), KL(kKeyZsn)}, {j >> 1, j >> 1}, l2, h2);
            pad[7 * B + i] = (j & 1) ? h2[0] - h2[1] : l2[0] - l2[1];
            lr_blocks<2>(T, {KL(kKeyOtn), KL(kKeyOtp)}, {r.pm_ctr_next + i, r.pm_ctr_prev + i}, l2, h2);
            pad[8 * B + i] = l2[0];
            pad[9 * B + i] = h2[0];
            pad[10 * B + i] = l2[1];
            pad[11 * B + i] = h2[1];
        } else if (p == 1) {
            u64 l1[1], h1[1];
            lr_blocks<1>(T, {KL(kKeyOtn)}, {r.pm_ctr_next + i}, l1, h1);
            pad[2 * B + i] = l1[0];
            pad[3 * B + i] = h1[0];
        } else {
            lr_blocks<2>(T, {KL(kKeyZsp), KL(kKeyZsn)}, {j >> 1, j >> 1}, l2, h2);
            pad[6 * B + i] = (j & 1) ? h2[0] - h2[1] : l2[0] - l2[1];
            u64 l1[1], h1[1];
            lr_blocks<1>(T, {KL(kKeyOtp)}, {r.pm_ctr_prev + i}, l1, h1);
            pad[7 * B + i] = l1[0];
            pad[8 * B + i] = h1[0];
        }
    }
}

// Helper workgroup h = blockIdx.x - 1 of the launch: batch rows
// [h R, min(B, (h + 1) R)), R = ceil(B / G).
//   phase 1: hprod[i] = XX0[i] (w0 + w1) + XX1[i] w0 and hy = YY of its rows,
//            then arrives on F_H1 (block 0 waits for epoch * G);
//   phase 4: after block 0's err (F_ERR), hpart[h] = sum over its rows of
//            XX0[i] (e0 + e1)[i] + XX1[i] e0[i], then arrives on F_H2.
// A wave per row (rows wave, wave + 8, ...), lanes over k pairs (16-byte
// loads), kLrHelperUnroll rows of a wave in flight.
constexpr u32 kLrHelperUnroll = 4;
__device__ __forceinline__ void lr_helper(const u32* T0g, const aby3g_lr_iter& it, const LrKeys& K,
                                          const HsStatus& status, u64* part, u32* lds, u32* keys, bool keepRows) {
    const u32 B = it.B, d = it.d, G = lr_helpers(B), h = blockIdx.x - 1;
    const u32 tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const Layout L(B, d, it.cir);
    u64* sc = (u64*)it.scratch;
    u64* box = (u64*)it.mailbox;
    const u64 ep = it.epoch, n = it.n;
    const u64* X0 = (const u64*)it.X;
    const u64* X1 = X0 + n * d;
    const u64* Y0 = (const u64*)it.Y;
    const u64* Y1 = Y0 + n;
    const u64* w0 = (const u64*)it.w;
    const u64* w1 = w0 + d;
    const u32 R = (B + G - 1) / G, r0 = h * R, r1 = min(B, r0 + R);

    // Phase 4 reads the same rows and columns per lane as phase 1 when each
    // takes one pass (d <= 128, at most kLrWaves * kLrHelperUnroll rows):
    // phase 1's loads are then kept in registers for it instead of gathered
    // from the dataset again after block 0's err arrives.
    const bool keep = keepRows && d <= 128 && r1 - r0 <= kLrWaves * kLrHelperUnroll;
    u64x2 k0r[kLrHelperUnroll], k1r[kLrHelperUnroll];
#pragma unroll
    for (u32 u = 0; u < kLrHelperUnroll; ++u) k0r[u] = k1r[u] = u64x2{0, 0};

    // ---- phase 1 ----
    for (u32 i0 = r0 + wave; i0 < r1; i0 += kLrWaves * kLrHelperUnroll) {
        u64 acc[kLrHelperUnroll], row[kLrHelperUnroll];
#pragma unroll
        for (u32 u = 0; u < kLrHelperUnroll; ++u) {
            acc[u] = 0;
            const u32 i = i0 + u * kLrWaves;
            row[u] = it.batch[i < r1 ? i : r0];
        }
        for (u32 k = 2 * lane; k < d; k += 128) {
            const bool pair = k + 1 < d;
            const u64 ws0 = w0[k] + w1[k], wa0 = w0[k];
            const u64 ws1 = pair ? w0[k + 1] + w1[k + 1] : 0, wa1 = pair ? w0[k + 1] : 0;
            u64x2 a0[kLrHelperUnroll], a1[kLrHelperUnroll];
#pragma unroll
            for (u32 u = 0; u < kLrHelperUnroll; ++u) {
                a0[u] = load_pair(X0 + row[u] * d + k, pair);
                a1[u] = load_pair(X1 + row[u] * d + k, pair);
            }
#pragma unroll
            for (u32 u = 0; u < kLrHelperUnroll; ++u)
                acc[u] += a0[u].x * ws0 + a0[u].y * ws1 + a1[u].x * wa0 + a1[u].y * wa1;
            if (keep) {
#pragma unroll
                for (u32 u = 0; u < kLrHelperUnroll; ++u) {
                    k0r[u] = a0[u];
                    k1r[u] = a1[u];
                }
            }
        }
#pragma unroll
        for (u32 u = 0; u < kLrHelperUnroll; ++u) {
            u64 a = acc[u];
#pragma unroll
            for (int o = 32; o; o >>= 1) a += __shfl_xor(a, o, 64);
            const u32 i = i0 + u * kLrWaves;
            if (i < r1) {
                if (lane == 0) hs_store(sc + L.hprod + i, a);
                if (lane == 1) hs_store(sc + L.hy + i, Y0[row[u]]);
                if (lane == 2) hs_store(sc + L.hy + B + i, Y1[row[u]]);
            }
        }
    }
    lr_arrive(box, F_H1);

    // ---- between phases 1 and 4 (block 0 runs the protocol): the next
    // iteration's randomness, off block 0's path ----
    if (it.pre_next) {
        const u32* kw = reinterpret_cast<const u32*>(&K);
        for (u32 i = threadIdx.x; i < kLrKeys * kKeyWords; i += kLrThreads) keys[i] = kw[i];
        aes_fill_lds(lds, T0g);  // its barrier publishes the keys too
        lr_predraw(it, lds, keys, sc + L.pre + ((ep + 1) & 1) * L.preSlot, L);
    }

    // ---- phase 4 ----
    // block 0's err comes only after its circuit and products (~80 us): until
    // its F_P3 flag (phase 3) poll rarely, so that the helpers' polls do not
    // load the memory path of the parties' hand-offs; then poll closely
    if (threadIdx.x == 0) {
        const u64 t0 = wall_clock64();
        for (u32 spins = 0; __hip_atomic_load((const gu64*)box + F_P3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < ep;) {
            __builtin_amdgcn_s_sleep(32);
            if ((++spins & 15) == 0 && (hs_failed(status) || wall_clock64() - t0 > status.limit))
                break;  // the close wait below gives up too
        }
    }
    __syncthreads();
    if (!hs_wait(HsWait{box, ep, nullptr, status}, F_ERR, F_ERR + 1)) return;
    const u64* e0 = sc + L.err;
    const u64* e1 = e0 + B;
    for (u32 k0 = 0; k0 < d; k0 += 128) {
        const u32 k = k0 + 2 * lane;
        const bool kin = k < d, pair = k + 1 < d;
        u64 acc0 = 0, acc1 = 0;
        for (u32 i0 = r0 + wave; i0 < r1; i0 += kLrWaves * kLrHelperUnroll) {
            u64x2 a0[kLrHelperUnroll], a1[kLrHelperUnroll];
            u64 ev0[kLrHelperUnroll], evs[kLrHelperUnroll];
#pragma unroll
            for (u32 u = 0; u < kLrHelperUnroll; ++u) {
                const u32 i = i0 + u * kLrWaves;
                const bool in = i < r1;
                if (keep) {
                    a0[u] = kin && in ? k0r[u] : u64x2{0, 0};
                    a1[u] = kin && in ? k1r[u] : u64x2{0, 0};
                } else {
                    const u64 rw = it.batch[in ? i : r0];
                    a0[u] = kin && in ? load_pair(X0 + rw * d + k, pair) : u64x2{0, 0};
                    a1[u] = kin && in ? load_pair(X1 + rw * d + k, pair) : u64x2{0, 0};
                }
                ev0[u] = in ? hs_load(e0 + i) : 0;  // written by block 0 on another CU
                evs[u] = in ? ev0[u] + hs_load(e1 + i) : 0;
            }
#pragma unroll
            for (u32 u = 0; u < kLrHelperUnroll; ++u) {
                acc0 += a0[u].x * evs[u] + a1[u].x * ev0[u];
                acc1 += a0[u].y * evs[u] + a1[u].y * ev0[u];
            }
        }
        // waves 0-3 store, waves 4-7 add, then one sum of four per k
        if (wave < 4) {
            part[wave * 128 + 2 * lane] = acc0;
            part[wave * 128 + 2 * lane + 1] = acc1;
        }
        __syncthreads();
        if (wave >= 4) {
            part[(wave - 4) * 128 + 2 * lane] += acc0;
            part[(wave - 4) * 128 + 2 * lane + 1] += acc1;
        }
        __syncthreads();
        if (tid < 128 && k0 + tid < d)
            hs_store(sc + L.hpart + (u64)h * d + k0 + tid, part[tid] + part[128 + tid] + part[256 + tid] + part[384 + tid]);
        __syncthreads();
    }
    lr_arrive(box, F_H2);
    // the next iteration's rows into this XCD's L2 (its helper h is a
    // workgroup of the same id, dealt to the same XCD)
    if (it.next_batch) {
        const u32 k = 2 * lane;
        if (k < d) {
            u64 sink = 0;
            for (u32 i = r0 + wave; i < r1; i += kLrWaves) {
                const u64 rw = it.next_batch[i];
                const u64x2 a0 = load_pair(X0 + rw * d + k, k + 1 < d), a1 = load_pair(X1 + rw * d + k, k + 1 < d);
                sink ^= a0.x ^ a1.x;
            }
            asm volatile("" ::"v"(sink));  // the loads are kept; nothing waits for them
        }
    }
}

// phase stamps for profiling (aby3g_lr_iter.phase_ticks): wall clock of slot s
__device__ __forceinline__ void lr_stamp(u64* ticks, u32 s) {
    if (ticks && threadIdx.x == 0) ticks[s] = wall_clock64();
    // shader-clock counter beside the first and last stamps (slots 13, 14):
    // the clock the iteration actually ran at
    if (ticks && threadIdx.x == 0 && (s == 0 || s == 11)) ticks[s == 0 ? 13 : 14] = clock64();
}

// Block 0: the protocol of one party. kLds: engine memory, masks and circuit
// tables in LDS. A template rather than a run-time choice of pointers: a
// pointer that may be LDS or global memory is a flat pointer, and every flat
// access waits for the wave's outstanding global stores too -- in the levels,
// for the write-through AND shares just sent (~1 us a level).
template <bool kLds>
__device__ __forceinline__ void lr_party(const u32* T0g, const aby3g_lr_iter& it, const LrKeys& K, const HsStatus& status,
                                         u32* lds, u32* keys, u64* dyn, u64* tw) {
    u64* const PT = it.phase_ticks;
    lr_stamp(PT, 0);
    // this iteration's randomness drawn ahead by the previous launch's
    // helpers (pre_have): no AES on this workgroup at all
    const Layout L0(it.B, it.d, it.cir);
    const u64* pre = it.pre_have ? (const u64*)it.scratch + L0.pre + (it.epoch & 1) * L0.preSlot : nullptr;
    if (!pre) {
        const u32* kw = reinterpret_cast<const u32*>(&K);
        for (u32 i = threadIdx.x; i < kLrKeys * kKeyWords; i += kLrThreads) keys[i] = kw[i];
        aes_fill_lds(lds, T0g);  // its barrier publishes the keys too
    }
    lr_stamp(PT, 12);
    const u32* T = lds;
    auto KL = [&](u32 key) -> const u32* { return keys + key * kKeyWords; };
    const u32 tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int p = it.party;
    const u32 B = it.B, d = it.d;
    const aby3g_lr_circuit& cir = it.cir;
    const Layout L(B, d, cir);
    const u64 W = L.W;
    u64* sc = (u64*)it.scratch;
    u64* box = (u64*)it.mailbox;
    const u64* nbox = (const u64*)it.next_mailbox;
    const u64* pbox = (const u64*)it.prev_mailbox;
    const u64 par = (it.epoch & 1) * L.region;
    u64* my = box + L.flags + par;                   // this epoch's outgoing region
    const u64* nx = nbox + L.flags + par;            // next party's
    const u64* pv = pbox + L.flags + par;            // prev party's
    const u64 ep = it.epoch;
    u64* ticks = it.wait_ticks;
    u64* w0 = (u64*)it.w;
    u64* w1 = w0 + d;
    u64* xw0 = sc + L.xw;
    u64* xw1 = xw0 + B;
    u64* prod = sc + L.prod;

    u64* mem = kLds ? dyn : sc + L.mem;
    u64* zmw = kLds ? dyn + 2 * (u64)cir.wires * W : sc + L.zmask;
    // the gate list and the AND output wires in LDS beside the engine memory
    // (the levels read a gate descriptor per gate-word: from global memory
    // that is one L2 round trip each, 4 us per level)
    const aby3g_gate* gates = cir.gates;
    const u32* andWires = cir.and_wires;
    const aby3g_lr_level* levelsL = cir.levels;
    const u32* batchEndsL = cir.batch_ends;
    const aby3g_lr_gate_ext* extL = cir.ext;
    if (kLds) {
        u32* gl = reinterpret_cast<u32*>(zmw + (u64)cir.nand * W);
        const u32* gg = reinterpret_cast<const u32*>(cir.gates);
        const u32 gw = cir.ngates * (u32)(sizeof(aby3g_gate) / 4);
        for (u32 i = threadIdx.x; i < gw; i += kLrThreads) gl[i] = gg[i];
        u32* al = gl + gw;
        for (u32 i = threadIdx.x; i < cir.nand; i += kLrThreads) al[i] = cir.and_wires[i];
        gates = reinterpret_cast<const aby3g_gate*>(gl);
        andWires = al;
        // the level table and batch ends too: per level they were two
        // dependent loads from global memory, ~2 us of a 4 us level
        u32* lvl = al + ((cir.nand + 3) & ~3u);
        const u32* lg = reinterpret_cast<const u32*>(cir.levels);
        for (u32 i = threadIdx.x; i < cir.nlevels * (u32)(sizeof(aby3g_lr_level) / 4); i += kLrThreads) lvl[i] = lg[i];
        const aby3g_lr_level& last = cir.levels[cir.nlevels - 1];
        const u32 nbatches = last.batch_off + last.nbatch;  // <= ngates
        u32* be = lvl + cir.nlevels * (u32)(sizeof(aby3g_lr_level) / 4);
        for (u32 i = threadIdx.x; i < nbatches; i += kLrThreads) be[i] = cir.batch_ends[i];
        levelsL = reinterpret_cast<const aby3g_lr_level*>(lvl);
        batchEndsL = be;
        if (cir.ext) {  // the folded gates' operand terms (16 bytes an entry)
            u32* ex = be + ((nbatches + 3) & ~3u);
            const u32* eg = reinterpret_cast<const u32*>(cir.ext);
            for (u32 i = threadIdx.x; i < cir.next * (u32)(sizeof(aby3g_lr_gate_ext) / 4); i += kLrThreads) ex[i] = eg[i];
            extL = reinterpret_cast<const aby3g_lr_gate_ext*>(ex);
        }
        // read from the levels on, after phase 1's barriers
    }

    // ---- phase 0: the circuit's AND masks, words with rows only ----
    if (pre) {
        // drawn ahead: into LDS beside the engine memory, or read in place
        if (kLds)
            for (u64 q = tid; q < (u64)cir.nand * W; q += kLrThreads) zmw[q] = pre[L.pzm + q];
        else
            zmw = const_cast<u64*>(pre + L.pzm);
    } else {
        u64* zm = zmw;
        const u64 Wh = (W + 1) / 2;
        // two items per thread (q, q + 512), their four blocks interleaved:
        // one chain of table reads per thread (8 waves leave the LDS idle otherwise)
        const u64 items = (u64)cir.nand * Wh;
        for (u64 q = tid; q < items; q += 2 * kLrThreads) {
            const u64 q2 = q + kLrThreads < items ? q + kLrThreads : q;  // a duplicate of q when none is left
            const u64 k = q / Wh, wp = q % Wh, k2 = q2 / Wh, wp2 = q2 % Wh;
            const u64 c = (k * L.Wpad + 2 * wp) >> 1;  // Wpad is even: draws 2wp, 2wp + 1 share a block
            const u64 c2 = (k2 * L.Wpad + 2 * wp2) >> 1;
            const u32* const kk[4] = {KL(kKeyMp), KL(kKeyMn), KL(kKeyMp), KL(kKeyMn)};
            u64 lo[4], hi[4];
            lr_blocks<4>(T, kk, {c, c, c2, c2}, lo, hi);
            zm[k * W + 2 * wp] = lo[0] ^ lo[1];
            if (2 * wp + 1 < W) zm[k * W + 2 * wp + 1] = hi[0] ^ hi[1];
            zm[k2 * W + 2 * wp2] = lo[2] ^ lo[3];
            if (2 * wp2 + 1 < W) zm[k2 * W + 2 * wp2 + 1] = hi[2] ^ hi[3];
        }
    }

    lr_stamp(PT, 1);
    // ---- phase 1: xw = mul(XX, w) with truncation (shift D) ----
    // the products come from the helper workgroups (lr_helper)
    const u32 G = lr_helpers(B);
    if (!lr_wait(box, F_H1, ep * G, ticks, status)) return;
    lr_acquire();
    prod = sc + L.hprod;
    __syncthreads();
    lr_stamp(PT, 2);
    const MsgTag tag{(u32)ep, it.sys_scope != 0};
    __shared__ u32 msgBad;
    if (tid == 0) msgBad = 0;
    lr_trunc_pair(T, keys, it.t1_next_off / 8, it.t1_prev_off / 8, B, it.D, prod, my + L.z1, tag, sc + L.z1own, xw0,
                  xw1, tw, pre ? pre + L.ptw1 : nullptr);
    lr_stamp(PT, 3);
    {
        MsgWait mw = msg_begin(tag, status);
        if (p < 2) lr_trunc_finalize(nx + L.z1, pv + L.z1, sc + L.z1own, B, it.D, p == 0 ? xw0 : xw1, mw);
        if (!msg_done(mw, &msgBad, p < 2 ? ticks : nullptr)) return;
    }

    lr_stamp(PT, 4);
    // ---- phase 2: regions of the piecewise sigmoid ----
    // P0 reshares x0 + x2 (its two shares) to P1
    if (p == 0)
        for (u32 i = tid; i < B; i += kLrThreads) msg_put(my + L.v, i, xw0[i] + xw1[i], tag);
    const u64* vrecv = pv + L.v;  // P1
    MsgWait vw = msg_begin(tag, status);
    // inputs straight into the wires (setTwoInputSharing): source s in
    // {aa_0, aa_1, b}, share h; a wave transposes the bits of its 64 rows
    const u64 WS = (u64)cir.wires * W;  // share stride
    for (u32 job = wave; job < 6 * W; job += kLrWaves) {
        const u32 src = job / (2 * (u32)W), h = (job / (u32)W) & 1, w = job % (u32)W;
        const u32 r = w * 64 + lane;
        u64 val = 0;
        if (r < B) {
            if (src < 2) {
                if (p == 0 && h == 0) val = xw0[r] + xw1[r] + (u64)it.thr_off[src];
                if (p == 1 && h == 1) val = msg_get(vrecv, r, vw) + (u64)it.thr_off[src];
            } else {
                if (p == 1 && h == 0) val = xw0[r];
                if (p == 2 && h == 1) val = xw1[r];
            }
        }
        // lane b stores bit b of the wave's 64 rows (one transpose, not 64 ballots)
        mem[h * WS + ((u64)cir.in_wire[src] + lane) * W + w] = transpose64(val, lane);
    }
    if (!msg_done(vw, &msgBad, p == 1 ? ticks : nullptr)) return;
    lr_stamp(PT, 5);
    // the levels (roundCallback): unpack the previous level's received AND
    // shares (a message word per AND gate and row word), then this level's
    // batches, then publish its AND shares
    const u64* zm = zmw;
    const u32 W32 = (u32)W;
    // gate-word q -> (q / W, q % W): a shift when W is a power of two (a
    // 32-bit division is ~30 VALU ops on the levels' critical path)
    const u32 wsh = (W32 & (W32 - 1)) == 0 ? (u32)__builtin_ctz(W32) : 32u;
    auto wdiv = [&](u32 q) { return wsh < 32 ? q >> wsh : q / W32; };
    for (u32 lv = 0; lv <= cir.nlevels; ++lv) {
        if (lv > 0 && levelsL[lv - 1].nand) {
            const aby3g_lr_level pl = levelsL[lv - 1];
            const u64* grows = pv + L.lvl + 2 * (u64)pl.and_wire_off * W;
            MsgWait mw = msg_begin(tag, status);
            for (u32 q = tid; q < pl.nand * W32 && mw.ok; q += kLrThreads) {
                const u64 v = msg_get(grows, q, mw);
                const u32 j = wdiv(q), w = q - j * W32;
                if (mw.ok) mem[WS + (u64)andWires[pl.and_wire_off + j] * W + w] = v;
            }
            if (!msg_done(mw, &msgBad, ticks)) return;
            if (lv < 16) lr_stamp(PT, 96 + lv);  // level lv - 1's AND shares in (ABY3G_LR_PHASE_SLOTS)
        }
        if (lv == cir.nlevels) break;
        // by value: the engine memory's LDS stores below would otherwise
        // force a re-read of the level's fields after every gate
        const aby3g_lr_level lvr = levelsL[lv];
        u64* gsend = my + L.lvl + 2 * (u64)lvr.and_wire_off * W;
        u32 begin = 0;
        for (u32 b = 0; b < lvr.nbatch; ++b) {
            const u32 end = batchEndsL[lvr.batch_off + b];
            for (u32 q = tid; q < (end - begin) * W32; q += kLrThreads) {
                const u32 gq = wdiv(q), w = q - gq * W32;
                // a gate folded into the first batch has its operands' XOR terms
                // in ext; read beside the descriptor (one LDS round trip for both)
                const bool folded = extL && begin + gq >= lvr.fused_first;
                aby3g_lr_gate_ext e;
                if (folded) e = extL[lvr.ext_off + begin + gq - lvr.fused_first];
                const aby3g_gate g = gates[lvr.first_gate + begin + gq];
                const bool unary = g.type == ABY3G_GATE_COPY || g.type == ABY3G_GATE_INV;
                const u32 in1 = unary ? g.in0 : g.in1;
                u64 x0 = mem[(u64)g.in0 * W + w], x1 = mem[WS + (u64)g.in0 * W + w];
                u64 y0 = mem[(u64)in1 * W + w], y1 = mem[WS + (u64)in1 * W + w];
                if (folded) {
#pragma unroll
                    for (int t = 0; t < 3; ++t) {
                        if (e.x[t] != 0xFFFF) {
                            x0 ^= mem[(u64)e.x[t] * W + w];
                            x1 ^= mem[WS + (u64)e.x[t] * W + w];
                        }
                        if (e.y[t] != 0xFFFF) {
                            y0 ^= mem[(u64)e.y[t] * W + w];
                            y1 ^= mem[WS + (u64)e.y[t] * W + w];
                        }
                    }
                    if (e.flags & 1) x0 = ~x0, x1 = ~x1;
                    if (e.flags & 2) y0 = ~y0, y1 = ~y1;
                }
                if (gate_is_and(g.type)) {
                    const u64 r = gate_and_share(g.type, x0, x1, y0, y1) ^ zm[(u64)g.z_row * W + w];
                    mem[(u64)g.out * W + w] = r;
                    msg_put(gsend, (u64)g.send_row * W + w, r, tag);
                } else {
                    u64 o0, o1;
                    gate_local(g.type, x0, x1, y0, y1, o0, o1);
                    mem[(u64)g.out * W + w] = o0;
                    mem[WS + (u64)g.out * W + w] = o1;
                }
            }
            if (lv < 8 && b < 4) lr_stamp(PT, 64 + 4 * lv + b);
            __syncthreads();
            if (lv < 8 && b < 4) lr_stamp(PT, 32 + 4 * lv + b);
            begin = end;
        }
        if (lv < 16) lr_stamp(PT, 16 + lv);
    }
    lr_stamp(PT, 6);
    // regions (getOutput, 1 bit each): reg[t][h][i]
    u64* reg = sc + L.reg;
    for (u32 i = tid; i < B; i += kLrThreads)
        for (u32 t = 0; t < 3; ++t)
            for (u32 h = 0; h < 2; ++h)
                reg[(2 * t + h) * B + i] = (mem[h * WS + (u64)cir.out_wire[t] * W + (i >> 6)] >> (i & 63)) & 1;
    __syncthreads();

    // ---- phase 3: f = region1 (half + slope x) + region2 one ----
    u64* A0 = sc + L.a;
    u64* A1 = A0 + B;
    u64* fr0 = sc + L.fr;
    u64* fr1 = fr0 + B;
    u64* g0 = sc + L.f2;
    u64* g1 = g0 + B;
    const u64* r1a = reg + 2 * B;  // region 1, share 0 / 1
    const u64* r1b = reg + 3 * B;
    const u64* r2a = reg + 4 * B;  // region 2
    const u64* r2b = reg + 5 * B;
    for (u32 i = tid; i < B; i += kLrThreads) {  // getFunctionValues (Sh3Piecewise.cpp:518-567)
        A0[i] = (u64)it.slope * xw0[i] + (p == 0 ? (u64)it.half : 0);
        A1[i] = (u64)it.slope * xw1[i] + (p == 1 ? (u64)it.half : 0);
    }
    __syncthreads();
    lr_stamp(PT, 7);
    const u64 otw = p == 0 ? it.ot_prev_off / 8 : p == 1 ? it.ot_prev_off / 8 : it.ot_next_off / 8;
    const u64* pad = pre ? pre + L.ppad : nullptr;  // the pads drawn ahead
    // Each send loop splits its AES blocks over all 512 threads (the OT part
    // on threads [0, B), the public-product part on [B, 2B)) and interleaves a
    // thread's blocks in one lr_blocks<NB> call: one wave of dependent
    // table reads per round instead of NB of them.
    if (p == 0) {
        const u64 nw = it.ot_next_off / 8;
        for (u32 q = tid; q < 2 * B; q += kLrThreads) {
            if (q < B) {
                // OT product, sender + helper (Sh3Evaluator.cpp:132-163)
                const u32 i = q;
                u64 lo[5], hi[5], zr, c1, c0;
                if (pad) {
                    zr = pad[0 * B + i], c1 = pad[1 * B + i], c0 = pad[2 * B + i];
                    lo[3] = pad[3 * B + i], hi[3] = pad[4 * B + i], lo[4] = pad[5 * B + i], hi[4] = pad[6 * B + i];
                } else {
                    const u64 wz = otw + 2 * i, wc = wz + 1, wn = nw + i;
                    const u32* const k[5] = {KL(kKeyPrev), KL(kKeyPrev), KL(kKeyNext), KL(kKeyOtn), KL(kKeyOtn)};
                    const u64 c[5] = {wz >> 1, wc >> 1, wn >> 1, it.ot_ctr + i, it.ot_ctr + B + i};
                    lr_blocks<5>(T, k, c, lo, hi);
                    zr = (wz & 1) ? hi[0] : lo[0], c1 = (wc & 1) ? hi[1] : lo[1], c0 = (wn & 1) ? hi[2] : lo[2];
                }
                fr0[i] = c0;
                fr1[i] = c1;
                const u32 bb0 = (u32)((r1a[i] ^ r1b[i]) & 1), bb1 = (u32)(r1a[i] & 1);
                const u64 zz = 0 - (c0 + c1) - zr;
                u64 s[2];
                s[bb0] = zz;
                s[bb0 ^ 1] = A0[i] + A1[i] + zz;
                msg_put(my + L.ots, 2 * i, lo[3] ^ s[0], tag);
                msg_put(my + L.ots, 2 * i + 1, hi[3] ^ s[1], tag);
                msg_put(my + L.oth, i, bb1 ? hi[4] : lo[4], tag);
            } else {
                // public product (Sh3Evaluator.cpp:430-447)
                const u32 i = q - B;
                u64 lo[4], hi[4], zs;
                if (pad) {
                    zs = pad[7 * B + i];
                    lo[2] = pad[8 * B + i], hi[2] = pad[9 * B + i], lo[3] = pad[10 * B + i], hi[3] = pad[11 * B + i];
                } else {
                    const u64 j = it.pm_draw + i;
                    const u32* const k[4] = {KL(kKeyZsp), KL(kKeyZsn), KL(kKeyOtn), KL(kKeyOtp)};
                    const u64 c[4] = {j >> 1, j >> 1, it.pm_ctr_next + i, it.pm_ctr_prev + i};
                    lr_blocks<4>(T, k, c, lo, hi);
                    zs = (j & 1) ? hi[0] - hi[1] : lo[0] - lo[1];
                }
                const u32 bb = (u32)((r2a[i] ^ r2b[i]) & 1);
                u64 t[2];
                t[bb] = zs;
                t[bb ^ 1] = (u64)it.one + zs;
                msg_put(my + L.pma, 2 * i, lo[2] ^ t[0], tag);
                msg_put(my + L.pma, 2 * i + 1, hi[2] ^ t[1], tag);
                msg_put(my + L.pmb, 2 * i, lo[3] ^ t[0], tag);
                msg_put(my + L.pmb, 2 * i + 1, hi[3] ^ t[1], tag);
            }
        }
        if (tid == 0) hs_store(box + F_P3, ep);  // sends done: the helpers poll for err closely from here
        MsgWait mw = msg_begin(tag, status);
        for (u32 i = tid; i < B; i += kLrThreads) {
            g0[i] = msg_get(nx + L.pmb, i, mw);  // P1's share of the product
            g1[i] = msg_get(pv + L.pmb, i, mw);  // P2's
        }
        if (!msg_done(mw, &msgBad, ticks)) return;
    } else if (p == 1) {
        for (u32 q = tid; q < 2 * B; q += kLrThreads) {
            if (q < B) {
                // OT receiver's share 1 (:165-200); public product, helper (:452-487)
                const u32 i = q;
                u64 zs;
                if (pad) {
                    fr1[i] = pad[0 * B + i];
                    zs = pad[1 * B + i];
                } else {
                    const u64 wf = otw + i, j = it.pm_draw + i;
                    const u32* const k[3] = {KL(kKeyPrev), KL(kKeyZsp), KL(kKeyZsn)};
                    const u64 c[3] = {wf >> 1, j >> 1, j >> 1};
                    u64 lo[3], hi[3];
                    lr_blocks<3>(T, k, c, lo, hi);
                    fr1[i] = (wf & 1) ? hi[0] : lo[0];
                    zs = (j & 1) ? hi[1] - hi[2] : lo[1] - lo[2];
                }
                g1[i] = zs;
                msg_put(my + L.pmb, i, zs, tag);  // mine -> P0
            } else {
                const u32 i = q - B;
                u64 lo[1], hi[1];
                if (pad)
                    lo[0] = pad[2 * B + i], hi[0] = pad[3 * B + i];
                else
                    lr_blocks<1>(T, {KL(kKeyOtn)}, {it.pm_ctr_next + i}, lo, hi);
                msg_put(my + L.pma, i, (r2a[i] & 1) ? hi[0] : lo[0], tag);  // help -> P2
            }
        }
        if (tid == 0) hs_store(box + F_P3, ep);  // sends done: the helpers poll for err closely from here
        MsgWait mw = msg_begin(tag, status);
        for (u32 i = tid; i < B; i += kLrThreads) {
            // c0 = recv(P2's send, P0's help; choice b1) + recv(P0's send, P2's help; choice b0)
            const u64 m1 = msg_get(nx + L.ots, 2 * i + (r1b[i] & 1), mw) ^ msg_get(pv + L.oth, i, mw);
            const u64 m0 = msg_get(pv + L.ots, 2 * i + (r1a[i] & 1), mw) ^ msg_get(nx + L.oth, i, mw);
            fr0[i] = m1 + m0;
            msg_put(my + L.otc, i, m1 + m0, tag);  // -> P2
        }
        for (u32 i = tid; i < B; i += kLrThreads)
            g0[i] = msg_get(pv + L.pma, 2 * i + (r2a[i] & 1), mw) ^ msg_get(nx + L.pma, i, mw);
        if (!msg_done(mw, &msgBad, ticks)) return;
    } else {
        for (u32 q = tid; q < 2 * B; q += kLrThreads) {
            if (q < B) {
                // OT product, sender + helper (:202-240)
                const u32 i = q;
                u64 lo[4], hi[4], zr, c0;
                if (pad) {
                    zr = pad[0 * B + i], c0 = pad[1 * B + i];
                    lo[2] = pad[2 * B + i], hi[2] = pad[3 * B + i], lo[3] = pad[4 * B + i], hi[3] = pad[5 * B + i];
                } else {
                    const u64 wz = otw + 2 * i, wc = wz + 1;
                    const u32* const k[4] = {KL(kKeyNext), KL(kKeyNext), KL(kKeyOtp), KL(kKeyOtp)};
                    const u64 c[4] = {wz >> 1, wc >> 1, it.ot_ctr + i, it.ot_ctr + B + i};
                    lr_blocks<4>(T, k, c, lo, hi);
                    zr = (wz & 1) ? hi[0] : lo[0], c0 = (wc & 1) ? hi[1] : lo[1];
                }
                fr0[i] = c0;
                const u32 bb0 = (u32)(r1b[i] & 1), bb1 = (u32)((r1a[i] ^ r1b[i]) & 1);
                u64 s[2];
                s[bb1] = zr;
                s[bb1 ^ 1] = A1[i] + zr;
                msg_put(my + L.oth, i, bb0 ? hi[2] : lo[2], tag);
                msg_put(my + L.ots, 2 * i, lo[3] ^ s[0], tag);
                msg_put(my + L.ots, 2 * i + 1, hi[3] ^ s[1], tag);
            } else {
                // public product, helper
                const u32 i = q - B;
                u64 lo[3], hi[3], zs;
                if (pad) {
                    zs = pad[6 * B + i];
                    lo[2] = pad[7 * B + i], hi[2] = pad[8 * B + i];
                } else {
                    const u64 j = it.pm_draw + i;
                    const u32* const k[3] = {KL(kKeyZsp), KL(kKeyZsn), KL(kKeyOtp)};
                    const u64 c[3] = {j >> 1, j >> 1, it.pm_ctr_prev + i};
                    lr_blocks<3>(T, k, c, lo, hi);
                    zs = (j & 1) ? hi[0] - hi[1] : lo[0] - lo[1];
                }
                g0[i] = zs;
                msg_put(my + L.pma, i, (r2b[i] & 1) ? hi[2] : lo[2], tag);  // help -> P1
                msg_put(my + L.pmb, i, zs, tag);                            // mine -> P0
            }
        }
        if (tid == 0) hs_store(box + F_P3, ep);  // sends done: the helpers poll for err closely from here
        MsgWait mw = msg_begin(tag, status);
        for (u32 i = tid; i < B; i += kLrThreads) {
            fr1[i] = msg_get(pv + L.otc, i, mw);
            g1[i] = msg_get(nx + L.pmb, 2 * i + (r2b[i] & 1), mw) ^ msg_get(pv + L.pma, i, mw);
        }
        if (!msg_done(mw, &msgBad, ticks)) return;
    }
    __syncthreads();

    lr_stamp(PT, 8);
    // ---- phase 4: err = f - YY; update = mulTruncate(XX^T, err); w -= update ----
    u64* e0 = sc + L.err;
    u64* e1 = e0 + B;
    const u64* hy = sc + L.hy;
    for (u32 i = tid; i < B; i += kLrThreads) {
        // write-through: the helpers on other CUs read err
        hs_store(e0 + i, fr0[i] + g0[i] - hy[i]);
        hs_store(e1 + i, fr1[i] + g1[i] - hy[B + i]);
    }
    lr_post(box, F_ERR, ep);
    // prod = XX^T err: the helpers' partial sums over their rows
    prod = sc + L.prod;
    if (!lr_wait(box, F_H2, ep * G, ticks, status)) return;
    lr_acquire();
    for (u32 k = tid; k < d; k += kLrThreads) {
        u64 v = 0;
#pragma unroll 16
        for (u32 h = 0; h < G; ++h) v += sc[L.hpart + (u64)h * d + k];  // the loads of 16 go out together
        prod[k] = v;
    }
    __syncthreads();
    lr_stamp(PT, 9);
    const u32 sh2 = it.D + it.aB;
    u64* u0 = sc + L.upd;
    u64* u1 = u0 + d;
    lr_trunc_pair(T, keys, it.t2_next_off / 8, it.t2_prev_off / 8, d, sh2, prod, my + L.z2, tag, sc + L.z2own, u0, u1, tw,
                  pre ? pre + L.ptw2 : nullptr);
    lr_stamp(PT, 10);
    {
        MsgWait mw = msg_begin(tag, status);
        if (p < 2) lr_trunc_finalize(nx + L.z2, pv + L.z2, sc + L.z2own, d, sh2, p == 0 ? u0 : u1, mw);
        if (!msg_done(mw, &msgBad, p < 2 ? ticks : nullptr)) return;
    }
    for (u32 k = tid; k < d; k += kLrThreads) {
        w0[k] -= u0[k];
        w1[k] -= u1[k];
    }
    lr_stamp(PT, 11);
}

__global__ void __launch_bounds__(kLrThreads, 1) k_lr_iter(const u32* __restrict__ T0g, aby3g_lr_iter it, LrKeys K,
                                                           HsStatus status, int memInLds, int keepRows) {
    __shared__ u32 lds[kAesLdsWords];
    __shared__ u64 part[kLrThreads];
    __shared__ __attribute__((aligned(16))) u32 keys[kLrKeys * kKeyWords];
    extern __shared__ __attribute__((aligned(16))) u64 dyn[];  // [2][wires][W] engine memory, then [nand][W] masks
    if (blockIdx.x > 0)
        lr_helper(T0g, it, K, status, part, lds, keys, keepRows != 0);
    else if (memInLds)
        lr_party<true>(T0g, it, K, status, lds, keys, dyn, part);
    else
        lr_party<false>(T0g, it, K, status, lds, keys, dyn, part);
}

}  // namespace

}  // namespace aby3g

using namespace aby3g;

// ABY3G_LR_KEEP_ROWS=0: the helpers gather their batch rows again for the
// XX^T err product (A/B runs); default: kept from the XX w product
static bool keep_rows() {
    static const bool on = [] {
        const char* e = getenv("ABY3G_LR_KEEP_ROWS");
        return !e || e[0] != '0';
    }();
    return on;
}

extern "C" {

uint64_t aby3g_lr_mailbox_bytes(uint32_t B, uint32_t d, const aby3g_lr_circuit* cir) {
    return cir ? Layout(B, d, *cir).mailboxWords() * 8 : 0;
}

uint64_t aby3g_lr_scratch_bytes(uint32_t B, uint32_t d, const aby3g_lr_circuit* cir) {
    return cir ? Layout(B, d, *cir).total * 8 : 0;
}

int aby3g_lr_iteration(const aby3g_lr_iter* it, aby3g_stream stream) {
    return guarded([&] {
        ABY3G_REQUIRE(it != nullptr, "null argument");
        ABY3G_REQUIRE(it->party >= 0 && it->party <= 2, "party out of range");
        ABY3G_REQUIRE(it->B >= 1 && it->B <= kLrMaxB && it->d >= 1 && it->d <= kLrMaxD, "shape outside the fused form");
        ABY3G_REQUIRE(it->D + it->aB + 2 < 64, "shift too large");
        ABY3G_REQUIRE(it->epoch >= 1, "epochs start at 1");
        ABY3G_REQUIRE(it->X && it->Y && it->w && it->batch && it->scratch && it->mailbox && it->next_mailbox &&
                          it->prev_mailbox && it->cir.gates && it->cir.levels,
                      "null pointer");
        ABY3G_REQUIRE(!it->cir.ext || it->cir.wires < 0xFFFF, "folded gate terms address wires by 16 bits");
        ABY3G_REQUIRE(it->t1_next_off % 8 == 0 && it->t1_prev_off % 8 == 0 && it->t2_next_off % 8 == 0 &&
                          it->t2_prev_off % 8 == 0 && it->ot_next_off % 8 == 0 && it->ot_prev_off % 8 == 0,
                      "stream offsets must be multiples of 8");
        LrKeys K;
        K.prev = expand_key(it->prev_seed);
        K.next = expand_key(it->next_seed);
        K.zsp = expand_key(it->zs_prev);
        K.zsn = expand_key(it->zs_next);
        K.mp = expand_key(it->mask_prev);
        K.mn = expand_key(it->mask_next);
        K.otn = expand_key(it->ot_next_key);
        K.otp = expand_key(it->ot_prev_key);
        if (it->pre_next) {
            ABY3G_REQUIRE(it->next_rand.t1_next_off % 8 == 0 && it->next_rand.t1_prev_off % 8 == 0 &&
                              it->next_rand.t2_next_off % 8 == 0 && it->next_rand.t2_prev_off % 8 == 0 &&
                              it->next_rand.ot_next_off % 8 == 0 && it->next_rand.ot_prev_off % 8 == 0,
                          "stream offsets must be multiples of 8");
            K.mp2 = expand_key(it->next_rand.mask_prev);
            K.mn2 = expand_key(it->next_rand.mask_next);
        }
        const Layout L(it->B, it->d, it->cir);
        // engine memory, masks, gates, AND wires (padded to 4), level table, batch ends (<= ngates, padded
        // to 4), folded gates' operand terms
        const u64 dynBytes = (2 * (u64)it->cir.wires + it->cir.nand) * L.W * 8 +
                             (u64)it->cir.ngates * sizeof(aby3g_gate) + 4 * (((u64)it->cir.nand + 3) & ~3ull) +
                             (u64)it->cir.nlevels * sizeof(aby3g_lr_level) + 4 * (((u64)it->cir.ngates + 3) & ~3ull) +
                             (it->cir.ext ? (u64)it->cir.next * sizeof(aby3g_lr_gate_ext) : 0);
        const int inLds = dynBytes <= kLrDynLdsMax;
        static const bool attr = [] {  // dynamic LDS beyond the default limit, once per process
            return hipFuncSetAttribute((const void*)k_lr_iter, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)kLrDynLdsMax) == hipSuccess;
        }();
        ABY3G_REQUIRE(attr || !inLds, "could not raise the fused iteration's dynamic LDS limit");
        // block 0 runs the protocol, blocks 1..G help with the dataset products
        launch(PROBE_OTHER, k_lr_iter, dim3(1 + lr_helpers(it->B)), dim3(kLrThreads), inLds ? dynBytes : 0, S(stream),
               aes_table(), *it, K, hs_status(), inLds, keep_rows() ? 1 : 0);
    });
}

}  // extern "C"
