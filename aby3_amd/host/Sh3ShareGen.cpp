#include "Sh3ShareGen.h"

namespace aby3 {

block streamBlock(const block& seed, u64 byteOff) {
    if (byteOff % 8) throw std::runtime_error("stream offsets are multiples of 8 bytes");
    u8 a[16], b[16];
    GPU_CALL(aby3g_aes_block_host(seed.data(), byteOff / 16, a));
    block r;
    if (byteOff % 16 == 0) {
        std::memcpy(&r, a, 16);
    } else {
        GPU_CALL(aby3g_aes_block_host(seed.data(), byteOff / 16 + 1, b));
        std::memcpy(r.data(), a + 8, 8);
        std::memcpy(r.data() + 8, b, 8);
    }
    return r;
}

void Sh3ShareGen::init(block prevSeed, block nextSeed) {
    mPrevSeed = prevSeed;
    mNextSeed = nextSeed;
    mPrevOff = mNextOff = 0;
    mKeyPrev = getPrevBlock();  // mShareGen[0].setKey(mPrevCommon.get<block>())
    mKeyNext = getNextBlock();  // mShareGen[1].setKey(mNextCommon.get<block>())
    mDrawIdx = 0;
}

void Sh3ShareGen::init(CommPkg& comm, block seed) {
    comm.mNext.asyncSendCopy(seed);
    block prevSeed;
    comm.mPrev.recv(prevSeed);
    init(prevSeed, seed);
}

block Sh3ShareGen::getPrevBlock() {
    block b = streamBlock(mPrevSeed, mPrevOff);
    mPrevOff += 16;
    return b;
}
block Sh3ShareGen::getNextBlock() {
    block b = streamBlock(mNextSeed, mNextOff);
    mNextOff += 16;
    return b;
}

aby3g_zero_share Sh3ShareGen::zeroShare(u64 drawBase) const {
    aby3g_zero_share z;
    std::memcpy(z.k_prev, mKeyPrev.data(), 16);
    std::memcpy(z.k_next, mKeyNext.data(), 16);
    z.draw_base = drawBase;
    return z;
}

}  // namespace aby3
