// Correlated randomness state of one party (aby3/sh3/Sh3ShareGen.h).
//
// The reference keeps two oc::PRNG streams (mPrevCommon / mNextCommon) and
// two AES-CTR zero-share buffers. Every draw is a pure function of (key,
// position), so the host keeps only keys and positions and the GPU produces
// the bytes where they are consumed:
//   * stream positions: byte offsets into PRNG(prevSeed) / PRNG(nextSeed);
//   * zero-share draw index j: draw j = half (j & 1) of AES(k, j >> 1).
#pragma once
#include "Channel.h"

namespace aby3 {

struct Sh3ShareGen {
    block mPrevSeed, mNextSeed;  // seeds of mPrevCommon / mNextCommon
    u64 mPrevOff = 0, mNextOff = 0;
    block mKeyPrev, mKeyNext;  // mShareGen[0] / mShareGen[1] keys
    u64 mDrawIdx = 0;

    // Sh3ShareGen::init(prevSeed, nextSeed) (Sh3ShareGen.h:9-23)
    void init(block prevSeed, block nextSeed);
    // seed exchange (Sh3ShareGen.h:25-31): send own seed to next, receive prev's
    void init(CommPkg& comm, block seed);

    // 16 bytes of a stream, computed on the host CPU (key derivation only)
    block getPrevBlock();
    block getNextBlock();

    // Reserve nbytes of a stream; returns the starting byte offset.
    u64 takePrev(u64 nbytes) {
        u64 o = mPrevOff;
        mPrevOff += nbytes;
        return o;
    }
    u64 takeNext(u64 nbytes) {
        u64 o = mNextOff;
        mNextOff += nbytes;
        return o;
    }
    // Reserve n zero-share draws; returns the first draw index.
    u64 takeDraws(u64 n) {
        u64 j = mDrawIdx;
        mDrawIdx += n;
        return j;
    }

    aby3g_zero_share zeroShare(u64 drawBase) const;
};

block streamBlock(const block& seed, u64 byteOff);  // PRNG(seed) bytes [off, off+16), off % 8 == 0

}  // namespace aby3
