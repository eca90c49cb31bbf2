// One direction of a cross-process channel (one party per process, the
// reference's deployment: Eval/dis_exec.sh:10-12 starts three processes whose
// CommPkg channels run over TCP, Sh3Types.h:32-34). The processes share a
// POSIX shared-memory segment per direction:
//   page 0   signal words, registered with each end's device: `ready` (written
//            by the sender's stream after a payload landed in its staging slot)
//            and `consumed[slot]` (written by the receiver's stream after it
//            copied a slot out) -- stream-ordered, no host round trip;
//   page 1   host control words: ring head / tail, per-slot "copy-out
//            enqueued" marks, the two ends' pids (attach handshake);
//   ring     the ordered message stream (descriptors and host payloads),
//            written in pieces so messages larger than the ring stream through.
// Device payloads themselves stay in device memory: the sender's staging
// slots are exported through IPC handles and the receiver copies out of them
// (a peer read over xGMI when the parties sit on different GPUs).
#pragma once
#include "Defines.h"
#include <aby3gpu.h>
#include <atomic>
#include <string>

namespace aby3 {

class LinkEnd {
public:
    static constexpr u32 kMaxSlots = 480;      // staging slots per direction
    static constexpr size_t kMaxStagedBytes = 2ull << 30;  // device bytes of staging per direction
    static constexpr size_t kRingBytes = 4u << 20;

    // name: the segment's shm name ("/aby3.<link>.<from>.<to>"); both ends
    // open it and wait (up to timeoutS) until the other end has attached.
    LinkEnd(const std::string& name, bool sender, int device);
    ~LinkEnd();
    LinkEnd(const LinkEnd&) = delete;
    LinkEnd& operator=(const LinkEnd&) = delete;

    bool sender() const { return mSender; }
    // ring bytes (blocking while the ring is full / empty)
    void write(const void* p, size_t n);
    void read(void* p, size_t n);

    // device-visible addresses of the signal words (this end's registration)
    u64* readyDev() const { return mSigDev; }
    u64* consumedDev(u32 slot) const { return mSigDev + 8 + slot; }
    // host words: the receiver has enqueued the copy-out of slot k's message `seq`
    std::atomic<u64>& posted(u32 slot);
    // blocks (up to timeoutS()) until posted(slot) >= seq
    void waitPosted(u32 slot, u64 seq) const;
    // host view of consumed[slot] (written by the receiver's stream once its
    // copy-out of the slot's message `seq` finished)
    u64 consumed(u32 slot) const;
    // waits (up to maxS seconds, no error) until consumed(slot) >= seq; false on timeout
    bool waitConsumed(u32 slot, u64 seq, double maxS) const;

    static double timeoutS();

    // ---- failing fast (the reference's Channel fails a pending receive when
    // the peer's session closes) ----
    // This process failed: every live link's header carries the abort word
    // (this pid) and the message, and every signal word of every live link is
    // set to ~0 so that no stream of any party stays parked on a wait this
    // process will never satisfy. Idempotent; the first message is kept.
    static void abortAll(const std::string& why);
    // This process is leaving normally (after the closing token exchange): a
    // peer that sees it exit does not take that for a failure.
    static void closeAll();
    // The first failure seen by this process (its own abort, a peer's abort
    // word, or a peer process gone without closing), or "" -- once set, every
    // link wait throws with it and the watchdog keeps the signal words released.
    static std::string failure();
    static bool failed();

private:
    static void releaseWords();
    static void watchdog();
    // one watchdog pass: a peer's abort word or a peer gone without closing
    bool peerFailed(std::string& why) const;
    void waitFor(const char* what, const std::atomic<u64>& w, u64 atLeast) const;
    std::string mName;
    bool mSender;
    u8* mBase = nullptr;
    size_t mBytes = 0;
    u64* mSigDev = nullptr;
    bool mRegistered = false;
    struct Hdr;
    Hdr* mHdr = nullptr;
    u8* mRing = nullptr;
    mutable double mNextAliveCheck = 0;  // watchdog: when to look at the peer's pid next
};

}  // namespace aby3
