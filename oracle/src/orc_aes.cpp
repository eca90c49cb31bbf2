// TEST INFRASTRUCTURE ONLY -- CPU oracle. See orc_aes.h.
#include "orc_aes.h"
#include <cstring>
#include <wmmintrin.h>
#include <emmintrin.h>
#include <cpuid.h>
#include <vector>

namespace orc {

namespace {

// FIPS-197 S-box computed from its definition (multiplicative inverse in
// GF(2^8) followed by the affine map), not from a pasted table.
struct SBox {
    u8 s[256];
    SBox() {
        auto gmul = [](u8 a, u8 b) {
            u8 p = 0;
            for (int i = 0; i < 8; ++i) {
                if (b & 1) p ^= a;
                u8 hi = a & 0x80;
                a <<= 1;
                if (hi) a ^= 0x1b;
                b >>= 1;
            }
            return p;
        };
        for (int x = 0; x < 256; ++x) {
            u8 inv = 0;
            if (x)
                for (int y = 1; y < 256; ++y)
                    if (gmul((u8)x, (u8)y) == 1) { inv = (u8)y; break; }
            u8 b = inv, r = 0x63;
            for (int i = 0; i < 8; ++i) {
                u8 bit = ((b >> i) ^ (b >> ((i + 4) & 7)) ^ (b >> ((i + 5) & 7)) ^
                          (b >> ((i + 6) & 7)) ^ (b >> ((i + 7) & 7))) & 1;
                r ^= (u8)(bit << i);
            }
            s[x] = r;
        }
    }
};
const SBox& sbox() {
    static SBox b;
    return b;
}

inline u8 xtime(u8 a) { return (u8)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

void expand(const u8 key[16], u8 rk[11][16]) {
    const u8* S = sbox().s;
    memcpy(rk[0], key, 16);
    u8 rcon = 1;
    for (int r = 1; r <= 10; ++r) {
        const u8* p = rk[r - 1];
        u8 t[4] = {S[p[13]], S[p[14]], S[p[15]], S[p[12]]};  // SubWord(RotWord(w[i-1]))
        t[0] ^= rcon;
        rcon = xtime(rcon);
        for (int j = 0; j < 4; ++j) rk[r][j] = p[j] ^ t[j];
        for (int j = 4; j < 16; ++j) rk[r][j] = p[j] ^ rk[r][j - 4];
    }
}

}  // namespace

void AesRef::setKey(const u8 key[16]) { expand(key, rk); }

void AesRef::encrypt(const u8 in[16], u8 out[16]) const {
    const u8* S = sbox().s;
    u8 st[16];
    for (int i = 0; i < 16; ++i) st[i] = in[i] ^ rk[0][i];
    for (int r = 1; r <= 10; ++r) {
        u8 t[16];
        // SubBytes + ShiftRows: state byte (row, col) lives at 4*col+row.
        for (int c = 0; c < 4; ++c)
            for (int row = 0; row < 4; ++row) t[4 * c + row] = S[st[4 * ((c + row) & 3) + row]];
        if (r != 10) {
            for (int c = 0; c < 4; ++c) {
                u8* col = t + 4 * c;
                u8 a0 = col[0], a1 = col[1], a2 = col[2], a3 = col[3];
                u8 all = a0 ^ a1 ^ a2 ^ a3;
                col[0] = a0 ^ all ^ xtime(a0 ^ a1);
                col[1] = a1 ^ all ^ xtime(a1 ^ a2);
                col[2] = a2 ^ all ^ xtime(a2 ^ a3);
                col[3] = a3 ^ all ^ xtime(a3 ^ a0);
            }
        }
        for (int i = 0; i < 16; ++i) st[i] = t[i] ^ rk[r][i];
    }
    memcpy(out, st, 16);
}

Block AesRef::encrypt(Block b) const {
    Block o;
    encrypt(reinterpret_cast<const u8*>(&b), reinterpret_cast<u8*>(&o));
    return o;
}

void AesNI::setKey(const u8 key[16]) { expand(key, rk); }

__attribute__((target("aes,sse2"))) Block AesNI::encrypt(Block b) const {
    __m128i s = _mm_loadu_si128((const __m128i*)&b);
    s = _mm_xor_si128(s, _mm_load_si128((const __m128i*)rk[0]));
    for (int r = 1; r < 10; ++r) s = _mm_aesenc_si128(s, _mm_load_si128((const __m128i*)rk[r]));
    s = _mm_aesenclast_si128(s, _mm_load_si128((const __m128i*)rk[10]));
    Block o;
    _mm_storeu_si128((__m128i*)&o, s);
    return o;
}

__attribute__((target("aes,sse2"))) void AesNI::ctr(u64 base, u64 n, Block* out) const {
    __m128i k[11];
    for (int r = 0; r < 11; ++r) k[r] = _mm_load_si128((const __m128i*)rk[r]);
    u64 i = 0;
    for (; i + 8 <= n; i += 8) {
        __m128i s[8];
        for (int j = 0; j < 8; ++j) s[j] = _mm_xor_si128(_mm_set_epi64x(0, (long long)(base + i + j)), k[0]);
        for (int r = 1; r < 10; ++r)
            for (int j = 0; j < 8; ++j) s[j] = _mm_aesenc_si128(s[j], k[r]);
        for (int j = 0; j < 8; ++j) _mm_storeu_si128((__m128i*)&out[i + j], _mm_aesenclast_si128(s[j], k[10]));
    }
    for (; i < n; ++i) {
        __m128i s = _mm_xor_si128(_mm_set_epi64x(0, (long long)(base + i)), k[0]);
        for (int r = 1; r < 10; ++r) s = _mm_aesenc_si128(s, k[r]);
        _mm_storeu_si128((__m128i*)&out[i], _mm_aesenclast_si128(s, k[10]));
    }
}

bool aesni_available() {
    static const bool has = [] {  // cpuid traps under virtualisation: ask once
        unsigned a, b, c, d;
        if (!__get_cpuid(1, &a, &b, &c, &d)) return false;
        return (c & bit_AES) != 0;
    }();
    return has;
}

void prng_bytes(const u8 seed[16], u64 byte_off, u64 nbytes, u8* out) {
    if (!nbytes) return;
    AesNI aes;
    aes.setKey(seed);
    u64 first = byte_off / 16, last = (byte_off + nbytes - 1) / 16;
    std::vector<Block> tmp(last - first + 1);
    if (aesni_available()) {
        aes.ctr(first, tmp.size(), tmp.data());
    } else {
        AesRef r;
        r.setKey(seed);
        for (u64 i = 0; i < tmp.size(); ++i) tmp[i] = r.encrypt(toBlock(first + i));
    }
    memcpy(out, reinterpret_cast<u8*>(tmp.data()) + (byte_off % 16), nbytes);
}

}  // namespace orc
