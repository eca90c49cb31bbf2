#include "Link.h"
#include "Device.h"
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <fcntl.h>
#include <sys/mman.h>
#include <thread>
#include <unistd.h>

namespace aby3 {

struct LinkEnd::Hdr {
    std::atomic<u64> magic;
    std::atomic<u64> senderPid, receiverPid;
    std::atomic<u64> head, tail;  // ring bytes written / consumed, ever
    std::atomic<u64> posted[kMaxSlots];
};

namespace {
constexpr size_t kPage = 4096;
constexpr u64 kMagic = 0x6c696e6b61627933ull;  // "aby3link"
static_assert(sizeof(std::atomic<u64>) == 8, "lock-free 64-bit atomics in shared memory");
static_assert((8 + LinkEnd::kMaxSlots) * 8 <= kPage, "signal words fit one page");
}  // namespace

double LinkEnd::timeoutS() {
    static const double t = [] {
        const char* e = getenv("ABY3_LINK_TIMEOUT_S");
        return e ? atof(e) : 300.0;
    }();
    return t;
}

// Spins briefly, then sleeps in short steps; a peer that never answers is an
// error after timeoutS() (a crashed party must not hang the others forever).
void LinkEnd::waitFor(const char* what, const std::atomic<u64>& w, u64 atLeast) const {
    if (w.load(std::memory_order_acquire) >= atLeast) return;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 2000; ++i) {
        for (int j = 0; j < 32; ++j) __builtin_ia32_pause();
        if (w.load(std::memory_order_acquire) >= atLeast) return;
    }
    const auto limit = std::chrono::duration<double>(timeoutS());
    while (w.load(std::memory_order_acquire) < atLeast) {
        if (std::chrono::steady_clock::now() - t0 > limit)
            throw std::runtime_error("link " + mName + ": timed out waiting for the peer (" + what + ")");
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

LinkEnd::LinkEnd(const std::string& name, bool sender, int device) : mName(name), mSender(sender) {
    mBytes = 2 * kPage + kRingBytes;
    // Both ends create-or-open; a fresh segment is zero-filled, which is the
    // initial state, so neither end has to come first.
    int fd = shm_open(name.c_str(), O_CREAT | O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("link " + name + ": shm_open failed");
    if (ftruncate(fd, (off_t)mBytes) != 0) {
        close(fd);
        throw std::runtime_error("link " + name + ": ftruncate failed");
    }
    void* p = mmap(nullptr, mBytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("link " + name + ": mmap failed");
    mBase = (u8*)p;
    mHdr = reinterpret_cast<Hdr*>(mBase + kPage);
    mRing = mBase + 2 * kPage;
    static_assert(sizeof(Hdr) <= kPage, "header fits one page");
    try {
        GPU_CALL(aby3g_set_device(device));
        void* dev = nullptr;
        GPU_CALL(aby3g_host_register(mBase, kPage, &dev));
        mRegistered = true;
        mSigDev = (u64*)dev;
        // attach handshake: announce this end, wait for the other
        u64 expect = 0;
        mHdr->magic.compare_exchange_strong(expect, kMagic);
        if (mHdr->magic.load() != kMagic) throw std::runtime_error("link " + name + ": not an aby3 link segment");
        (sender ? mHdr->senderPid : mHdr->receiverPid).store((u64)getpid(), std::memory_order_release);
        waitFor("attach", sender ? mHdr->receiverPid : mHdr->senderPid, 1);
        // both ends mapped it: the name is no longer needed
        shm_unlink(name.c_str());
    } catch (...) {
        if (mRegistered) aby3g_host_unregister(mBase);
        munmap(mBase, mBytes);
        shm_unlink(name.c_str());
        throw;
    }
}

LinkEnd::~LinkEnd() {
    if (mRegistered) aby3g_host_unregister(mBase);
    if (mBase) munmap(mBase, mBytes);
}

std::atomic<u64>& LinkEnd::posted(u32 slot) { return mHdr->posted[slot]; }

void LinkEnd::waitPosted(u32 slot, u64 seq) const { waitFor("a free staging slot", mHdr->posted[slot], seq); }

u64 LinkEnd::consumed(u32 slot) const {
    return __atomic_load_n(reinterpret_cast<const u64*>(mBase) + 8 + slot, __ATOMIC_ACQUIRE);
}

bool LinkEnd::waitConsumed(u32 slot, u64 seq, double maxS) const {
    const auto t0 = std::chrono::steady_clock::now();
    const auto limit = std::chrono::duration<double>(maxS);
    while (consumed(slot) < seq) {
        if (std::chrono::steady_clock::now() - t0 > limit) return false;
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    return true;
}

void LinkEnd::write(const void* src, size_t n) {
    const u8* s = (const u8*)src;
    u64 head = mHdr->head.load(std::memory_order_relaxed);
    while (n) {
        // room: the receiver has consumed up to tail
        waitFor("ring space", mHdr->tail, head + 1 > kRingBytes ? head + 1 - kRingBytes : 0);
        const u64 tail = mHdr->tail.load(std::memory_order_acquire);
        const size_t room = kRingBytes - (size_t)(head - tail);
        const size_t pos = (size_t)(head % kRingBytes);
        const size_t k = std::min({n, room, kRingBytes - pos});
        std::memcpy(mRing + pos, s, k);
        head += k;
        s += k;
        n -= k;
        mHdr->head.store(head, std::memory_order_release);
    }
}

void LinkEnd::read(void* dst, size_t n) {
    u8* d = (u8*)dst;
    u64 tail = mHdr->tail.load(std::memory_order_relaxed);
    while (n) {
        waitFor("message", mHdr->head, tail + 1);
        const u64 head = mHdr->head.load(std::memory_order_acquire);
        const size_t pos = (size_t)(tail % kRingBytes);
        const size_t k = std::min({n, (size_t)(head - tail), kRingBytes - pos});
        std::memcpy(d, mRing + pos, k);
        tail += k;
        d += k;
        n -= k;
        mHdr->tail.store(tail, std::memory_order_release);
    }
}

}  // namespace aby3
