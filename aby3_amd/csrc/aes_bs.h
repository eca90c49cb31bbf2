// Bitsliced AES-128 in counter mode: 32 blocks per thread, one u32 bit
// plane per state bit (plane i, bit j = bit i of block j), VALU only -- no
// LDS tables.
//
// MEASURED AND NOT USED BY THE KERNELS (round 1): on gfx950 this runs at
// 38 G blocks/s for 16M-block batches (~1030 VALU ops per block with this
// 161-gate S-box, 303 VGPRs -> one wave per SIMD) against 50 G blocks/s for
// the LDS T-table kernels, and a 32-block-per-thread batch leaves most of
// the chip idle below ~8M blocks. Kept, with its host test, as the base for
// a smaller S-box (113-gate class) that could tip the balance.
//
// Blocks of a thread: counter(j) = base + lane + 64 * j, j = 0..31, with
// base a multiple of 2048, so the plaintext planes (LE64(counter) || 0^64,
// SURVEY.md Appendix A) are constants: bits 0..5 come from the lane, bits
// 6..10 from j (the usual 0xAAAAAAAA ... 0xFFFF0000 patterns), the rest
// from base. The S-box is the 161-gate tower-field circuit generated and
// exhaustively checked by tools/gen_sbox.py. Host and device compile the
// same code; tests/cpp/test_aes_bs.cpp checks it against the oracle's AES.
#pragma once
#include <cstdint>
#include "aes_bs_sbox.h"

#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define ABY3G_HD __host__ __device__ __forceinline__
#else
#define ABY3G_HD inline
#endif

namespace aby3g {
namespace bs {

using u32 = uint32_t;
using u64 = uint64_t;

// plaintext planes of counters base + lane + 64 j (base % 2048 == 0)
ABY3G_HD void load_counters(u32 st[128], u64 base, u32 lane) {
    const u32 jmask[5] = {0xAAAAAAAAu, 0xCCCCCCCCu, 0xF0F0F0F0u, 0xFF00FF00u, 0xFFFF0000u};
#pragma unroll
    for (int i = 0; i < 6; ++i) st[i] = ((lane >> i) & 1) ? ~0u : 0u;
#pragma unroll
    for (int i = 6; i < 11; ++i) st[i] = jmask[i - 6];
#pragma unroll
    for (int i = 11; i < 64; ++i) st[i] = ((base >> i) & 1) ? ~0u : 0u;
#pragma unroll
    for (int i = 64; i < 128; ++i) st[i] = 0u;
}

// round key r, bit i: bit (i % 32) of rk[4r + i / 32] (LE column words)
ABY3G_HD void add_round_key(u32 st[128], const u32* rk, int r) {
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const u32 k = rk[4 * r + w];
#pragma unroll
        for (int b = 0; b < 32; ++b) st[32 * w + b] ^= 0u - ((k >> b) & 1u);
    }
}

ABY3G_HD void sub_bytes(u32 st[128]) {
#pragma unroll
    for (int byte = 0; byte < 16; ++byte) {
        u32* x = st + 8 * byte;
        u32 y[8];
        ABY3G_AES_BS_SBOX(u32, x, y);
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = y[k];
    }
}

// byte b = row + 4 col; after ShiftRows new[r + 4c] = old[r + 4((c + r) % 4)]
ABY3G_HD void shift_rows(u32 st[128]) {
    u32 t[128];
#pragma unroll
    for (int i = 0; i < 128; ++i) t[i] = st[i];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int k = 0; k < 8; ++k) st[8 * (r + 4 * c) + k] = t[8 * (r + 4 * ((c + r) & 3)) + k];
}

// out_i = 2 (a_i ^ a_{i+1}) ^ (a_0 ^ a_1 ^ a_2 ^ a_3) ^ a_i per column
ABY3G_HD void mix_columns(u32 st[128]) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        u32* a0 = st + 8 * (4 * c + 0);
        u32* a1 = st + 8 * (4 * c + 1);
        u32* a2 = st + 8 * (4 * c + 2);
        u32* a3 = st + 8 * (4 * c + 3);
        u32 tmp[8], in[4][8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            in[0][k] = a0[k];
            in[1][k] = a1[k];
            in[2][k] = a2[k];
            in[3][k] = a3[k];
            tmp[k] = a0[k] ^ a1[k] ^ a2[k] ^ a3[k];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            u32 s[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) s[k] = in[i][k] ^ in[(i + 1) & 3][k];
            // xtime(s): (s << 1) ^ (s7 ? 0x1b : 0)
            const u32 x[8] = {s[7], s[0] ^ s[7], s[1], s[2] ^ s[7], s[3] ^ s[7], s[4], s[5], s[6]};
            u32* o = st + 8 * (4 * c + i);
#pragma unroll
            for (int k = 0; k < 8; ++k) o[k] = x[k] ^ tmp[k] ^ in[i][k];
        }
    }
}

ABY3G_HD void encrypt(u32 st[128], const u32* rk) {
    add_round_key(st, rk, 0);
#pragma unroll 1
    for (int r = 1; r < 10; ++r) {
        sub_bytes(st);
        shift_rows(st);
        mix_columns(st);
        add_round_key(st, rk, r);
    }
    sub_bytes(st);
    shift_rows(st);
    add_round_key(st, rk, 10);
}

// In-place 32 x 32 bit transpose of a[0..31]: afterwards bit t of a[j] is
// what bit j of a[t] was.
ABY3G_HD void transpose32(u32 a[32]) {
    u32 m = 0x0000FFFFu;
#pragma unroll
    for (int j = 16; j != 0; j >>= 1, m ^= m << j) {
#pragma unroll
        for (int k = 0; k < 32; k = (k + j + 1) & ~j) {
            // swap bits c + j of a[k] with bits c of a[k + j] (bit j of c clear)
            const u32 t = ((a[k] >> j) ^ a[k + j]) & m;
            a[k + j] ^= t;
            a[k] ^= t << j;
        }
    }
}

// planes -> per block: after this, st[4 j + w] = 32-bit word w of block j
// (word w = bytes 4w .. 4w+3 of the ciphertext, little-endian)
ABY3G_HD void planes_to_blocks(u32 st[128]) {
    u32 tmp[128];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        u32 a[32];
#pragma unroll
        for (int t = 0; t < 32; ++t) a[t] = st[32 * w + t];
        transpose32(a);
#pragma unroll
        for (int j = 0; j < 32; ++j) tmp[4 * j + w] = a[j];
    }
#pragma unroll
    for (int i = 0; i < 128; ++i) st[i] = tmp[i];
}

}  // namespace bs
}  // namespace aby3g
