#include "Link.h"
#include "Device.h"
#include <algorithm>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <mutex>
#include <signal.h>
#include <sys/mman.h>
#include <thread>
#include <unistd.h>
#include <vector>

namespace aby3 {

struct LinkEnd::Hdr {
    std::atomic<u64> magic;
    std::atomic<u64> senderPid, receiverPid;
    std::atomic<u64> head, tail;  // ring bytes written / consumed, ever
    std::atomic<u64> abortPid;    // a process that failed (abortAll): its pid, abortMsg written before
    std::atomic<u64> senderClosed, receiverClosed;  // the end left normally (closeAll)
    char abortMsg[160];
    std::atomic<u64> posted[kMaxSlots];
};

namespace {
constexpr size_t kPage = 4096;
constexpr u64 kMagic = 0x6c696e6b61627933ull;  // "aby3link"
static_assert(sizeof(std::atomic<u64>) == 8, "lock-free 64-bit atomics in shared memory");
static_assert((8 + LinkEnd::kMaxSlots) * 8 <= kPage, "signal words fit one page");

// Every live link end of this process, and the watchdog that looks at their
// peers while any exists. The watchdog never throws: it records the first
// failure and keeps every signal word released (~0), so that the streams of
// this process -- and of the peers, which map the same pages -- drain instead
// of waiting on a party that is gone; the host code throws at its next link
// wait or stream sync (failed()).
std::mutex gMu;
std::vector<LinkEnd*> gLinks;
std::thread gWatch;
bool gWatchStop = false;
std::atomic<bool> gFailed{false};
std::string gWhy;

double nowS() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// a process that still runs (a zombie -- exited, not yet reaped by its
// parent -- counts as gone)
bool processAlive(u64 pid) {
    if (!pid) return true;  // not attached yet
    if (kill((pid_t)pid, 0) != 0 && errno == ESRCH) return false;
    char path[64];
    std::snprintf(path, sizeof path, "/proc/%llu/stat", (unsigned long long)pid);
    FILE* f = std::fopen(path, "r");
    if (!f) return true;  // no procfs: trust kill()
    char buf[256] = {0};
    const size_t n = std::fread(buf, 1, sizeof buf - 1, f);
    std::fclose(f);
    const char* rp = n ? std::strrchr(buf, ')') : nullptr;  // "pid (comm) S ..."
    return !(rp && rp[1] == ' ' && (rp[2] == 'Z' || rp[2] == 'X'));
}
}  // namespace

void LinkEnd::releaseWords() {
    // callers hold gMu
    for (LinkEnd* l : gLinks) {
        u64* w = reinterpret_cast<u64*>(l->mBase);
        for (u32 i = 0; i < 8 + kMaxSlots; ++i) __atomic_store_n(w + i, ~0ull, __ATOMIC_RELEASE);
    }
}

bool LinkEnd::peerFailed(std::string& why) const {
    const u64 me = (u64)getpid();
    const u64 ab = mHdr->abortPid.load(std::memory_order_acquire);
    if (ab && ab != me) {
        char msg[sizeof mHdr->abortMsg + 1];
        std::memcpy(msg, mHdr->abortMsg, sizeof mHdr->abortMsg);
        msg[sizeof mHdr->abortMsg] = 0;
        why = "peer process " + std::to_string(ab) + " failed: " + msg;
        return true;
    }
    const double t = nowS();
    if (t < mNextAliveCheck) return false;
    mNextAliveCheck = t + 0.02;
    const u64 peer = (mSender ? mHdr->receiverPid : mHdr->senderPid).load(std::memory_order_acquire);
    const bool closed = (mSender ? mHdr->receiverClosed : mHdr->senderClosed).load(std::memory_order_acquire) != 0;
    if (!closed && !processAlive(peer)) {
        why = "peer process " + std::to_string(peer) + " exited without closing link " + mName;
        return true;
    }
    return false;
}

void LinkEnd::watchdog() {
    for (;;) {
        // a plain sleep, not a timed condition-variable wait: the sanitizers
        // of this toolchain do not see the unlock inside a steady-clock
        // timed wait (pthread_cond_clockwait) and report false races
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
        std::lock_guard<std::mutex> lk(gMu);
        if (gWatchStop) break;
        if (!gFailed.load(std::memory_order_relaxed)) {
            std::string why;
            for (LinkEnd* l : gLinks)
                if (l->peerFailed(why)) {
                    gWhy = why;
                    gFailed.store(true, std::memory_order_release);
                    break;
                }
        }
        // a stream still running may write a smaller value after the release
        if (gFailed.load(std::memory_order_relaxed)) releaseWords();
    }
}

void LinkEnd::abortAll(const std::string& why) {
    std::lock_guard<std::mutex> lk(gMu);
    const u64 me = (u64)getpid();
    for (LinkEnd* l : gLinks) {
        u64 expect = 0;
        if (l->mHdr->abortPid.load(std::memory_order_acquire) == 0) {
            std::strncpy(l->mHdr->abortMsg, why.c_str(), sizeof l->mHdr->abortMsg - 1);
            l->mHdr->abortPid.compare_exchange_strong(expect, me, std::memory_order_acq_rel);
        }
    }
    if (!gFailed.load(std::memory_order_relaxed)) {
        gWhy = why;
        gFailed.store(true, std::memory_order_release);
    }
    releaseWords();
}

void LinkEnd::closeAll() {
    std::lock_guard<std::mutex> lk(gMu);
    for (LinkEnd* l : gLinks) (l->mSender ? l->mHdr->senderClosed : l->mHdr->receiverClosed).store(1, std::memory_order_release);
}

bool LinkEnd::failed() { return gFailed.load(std::memory_order_acquire); }

std::string LinkEnd::failure() {
    if (!failed()) return std::string();
    std::lock_guard<std::mutex> lk(gMu);
    return gWhy;
}

double LinkEnd::timeoutS() {
    static const double t = [] {
        const char* e = getenv("ABY3_LINK_TIMEOUT_S");
        return e ? atof(e) : 300.0;
    }();
    return t;
}

// Spins briefly, then sleeps in short steps. A failed process (this one or a
// peer: abort word, or gone without closing -- the watchdog's finding) is an
// error at once; a peer that never answers is an error after timeoutS().
void LinkEnd::waitFor(const char* what, const std::atomic<u64>& w, u64 atLeast) const {
    if (w.load(std::memory_order_acquire) >= atLeast) return;
    auto fail = [&] {
        throw std::runtime_error("link " + mName + ": gave up waiting for the peer (" + what + "): " + failure());
    };
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 2000; ++i) {
        for (int j = 0; j < 32; ++j) __builtin_ia32_pause();
        if (w.load(std::memory_order_acquire) >= atLeast) return;
        if ((i & 63) == 0 && failed()) fail();
    }
    const auto limit = std::chrono::duration<double>(timeoutS());
    while (w.load(std::memory_order_acquire) < atLeast) {
        if (failed()) fail();
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
        std::lock_guard<std::mutex> lk(gMu);
        gLinks.push_back(this);
        if (!gWatch.joinable()) {
            gWatchStop = false;
            gWatch = std::thread(&LinkEnd::watchdog);
        }
    } catch (...) {
        if (mRegistered) aby3g_host_unregister(mBase);
        munmap(mBase, mBytes);
        shm_unlink(name.c_str());
        throw;
    }
}

LinkEnd::~LinkEnd() {
    std::thread stop;
    {
        std::lock_guard<std::mutex> lk(gMu);
        gLinks.erase(std::remove(gLinks.begin(), gLinks.end(), this), gLinks.end());
        if (gLinks.empty()) {
            if (gWatch.joinable()) {
                gWatchStop = true;  // seen within the watchdog's 2 ms tick
                stop = std::move(gWatch);
            }
            // the ring is gone: a later one in this process starts clean
            gFailed.store(false, std::memory_order_release);
            gWhy.clear();
        }
    }
    if (stop.joinable()) stop.join();
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
