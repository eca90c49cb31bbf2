// TEST INFRASTRUCTURE ONLY -- part of the CPU oracle (see oracle/README.md).
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
// anything under oracle/. The product (aby3_amd/) never links it.
//
// AES-128 restated from FIPS-197 as cryptoTools' oc::AES uses it
// (call sites: aby3/sh3/Sh3ShareGen.h:19-20,52-53; aby3/OT/SharedOT.cpp:15,64,73;
// aby3/sh3/Sh3BinaryEvaluator.cpp:76,1420-1421). Two implementations:
//   * orc::AesRef  -- byte-oriented textbook cipher (the specification),
//   * orc::AesNI   -- AES-NI path, what cryptoTools runs on x86 and what the
//                     CPU baseline must use to be a fair restatement.
// Both are checked against the FIPS-197 known-answer vectors and against each
// other in tests/test_oracle_aes.py.
#pragma once
#include <cstdint>
#include <cstddef>

namespace orc {

using u8 = uint8_t;
using u32 = uint32_t;
using u64 = uint64_t;
using i64 = int64_t;

// A 16-byte block; byte order is memory order. cryptoTools' toBlock(hi, lo)
// = LE64(lo) || LE64(hi) (Appendix A of SURVEY.md).
struct Block {
    u64 lo, hi;
};
inline Block toBlock(u64 hi, u64 lo) { return Block{lo, hi}; }
inline Block toBlock(u64 lo) { return Block{lo, 0}; }

struct AesRef {
    u8 rk[11][16];
    void setKey(const u8 key[16]);
    void encrypt(const u8 in[16], u8 out[16]) const;
    Block encrypt(Block b) const;
};

struct AesNI {
    alignas(16) u8 rk[11][16];
    void setKey(const u8 key[16]);
    // out[i] = AES(key, LE64(base+i) || 0^8) -- oc::AES::ecbEncCounterMode
    void ctr(u64 base, u64 n, Block* out) const;
    Block encrypt(Block b) const;
};

bool aesni_available();

// Byte stream of cryptoTools' PRNG(seed): S[b] = AES(seed, b/16)[b%16]
// (PRNG::SetSeed + refillBuffer = ecbEncCounterMode from block 0).
void prng_bytes(const u8 seed[16], u64 byte_off, u64 nbytes, u8* out);

}  // namespace orc
