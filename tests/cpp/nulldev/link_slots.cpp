// The staging-slot rules of the cross-process links (Channel.cpp) under
// asynchronous streams (the null device with ND_ASYNC=1: every stream a
// thread that runs its copies, signal-word writes and waits in order, some
// after a random delay, so the host runs ahead of its streams as on a GPU).
// Three forked processes, one party each, exchange 1200 device messages per
// direction whose sizes wander across the slots' 2 MiB steps (so slots are
// reused, outgrown, retired and re-mapped), by the three send forms --
// staged copies (asyncSendDevice), zero-copy sends that stage a copy
// (asyncSendShared) and payloads produced straight into a reserved slot
// (linkSendBuffer) -- and complete each receive a few messages after it was
// posted, in a shuffled order (futures completed out of ticket order, as the
// protocols' tasks do), so copy-outs are in flight while slots are reused.
// The null device copies for real, so every message's bytes are checked:
// a slot reused before its copy-out finished, a copy-out before its copy-in,
// or a mapping closed under a pending copy (which the null device also traps)
// shows up as wrong bytes or an abort. Run by tests/test_host_asan.py under
// AddressSanitizer.
#include "Channel.h"
#include "Device.h"
#include <algorithm>
#include <cstdio>
#include <random>
#include <string>
#include <sys/wait.h>
#include <unistd.h>
#include <vector>

extern "C" int nulldev_shared_arena(size_t bytes);
extern "C" size_t nulldev_arena_used();

using namespace aby3;

// a message's bytes: one value per (sender, message), written by a stream
// memset (no host copy, which would drain the stream)
static int byteOf(int from, int msg) { return (from * 89 + msg * 7 + 1) % 251; }

static size_t msgBytes(int msg) {
    // eight sizes either side of the slots' 2 MiB steps, in a pseudo-random
    // walk (few sizes: the pools cache by size class and never trim mid-run)
    static const size_t sizes[] = {8, 4096, (64u << 10) + 8, 1u << 20, (2u << 20) + 8, 3u << 20, (4u << 20) + 8, 6u << 20};
    std::mt19937_64 r((u64)msg * 7919 + 17);
    const int band = (msg / 37) % 3;  // runs of small, mixed and large messages
    const u64 v = r();
    return sizes[band == 0 ? v % 4 : band == 1 ? v % 8 : 4 + v % 4];
}

static int party_main(int p, const std::string& tag) {
    const int kMsgs = 1200, kLag = 3, kCheck = 16;
    Gpu g(0);
    g.bind();
    CommPkg c = makeProcessRing(p, tag, 0, false, true);  // the cross-GPU branches: every device message staged
    const int from = (p + 2) % 3;
    std::mt19937 shuf(1234 + p);
    std::vector<std::shared_ptr<DeviceBuffer>> keep(kMsgs), dst(kMsgs), got(kMsgs);
    std::vector<RecvFuture> fut(kMsgs);
    std::vector<int> pending;  // posted receives not yet completed
    int checked = 0;
    auto check = [&](int upTo) {
        g.sync();
        for (; checked < upTo; ++checked) {
            const int m = checked;
            const size_t bytes = msgBytes(m);
            std::vector<u8> h(bytes);
            toHost(h.data(), got[m]->data(), bytes, g);
            for (size_t i = 0; i < h.size(); ++i)
                if (h[i] != (u8)byteOf(from, m)) {
                    std::printf("FAIL party %d: message %d (%zu bytes) byte %zu: %d, expected %d\n", p, m, bytes, i,
                                h[i], byteOf(from, m));
                    return false;
                }
            got[m].reset();
            dst[m].reset();
            keep[m].reset();
            fut[m] = RecvFuture();  // a completed future holds its received buffer
        }
        return true;
    };
    for (int m = 0; m < kMsgs; ++m) {
        const size_t bytes = msgBytes(m);
        const int form = m % 3;
        if (form == 2) {
            keep[m] = c.mNext.linkSendBuffer(g, bytes);  // produced in place
            GPU_CALL(aby3g_memset(keep[m]->data(), byteOf(p, m), bytes, g.stream()));
            c.mNext.asyncSendShared(keep[m], bytes, g);
        } else {
            keep[m] = std::make_shared<DeviceBuffer>(g, bytes);
            GPU_CALL(aby3g_memset(keep[m]->data(), byteOf(p, m), bytes, g.stream()));
            if (form == 0)
                c.mNext.asyncSendDevice(keep[m]->data(), bytes, g);
            else
                c.mNext.asyncSendShared(keep[m], bytes, g);
        }
        // post the matching receive now, complete receives a few messages
        // later and out of order, so copy-outs are in flight on this stream
        // while the sender reuses, outgrows and retires slots
        if (form == 0) {
            dst[m] = std::make_shared<DeviceBuffer>(g, bytes);
            fut[m] = c.mPrev.asyncRecvDevice(dst[m]->data(), bytes, g);
        } else {
            fut[m] = c.mPrev.asyncRecvShared(bytes, g);
        }
        pending.push_back(m);
        while ((int)pending.size() > kLag || (m == kMsgs - 1 && !pending.empty())) {
            const size_t pick = shuf() % pending.size();
            const int k = pending[pick];
            pending.erase(pending.begin() + (long)pick);
            if (dst[k]) {
                fut[k].get();
                got[k] = dst[k];
            } else {
                got[k] = fut[k].getShared();
            }
        }
        // verify the completed prefix now and then (a sync: everything enqueued so far lands)
        if (m % kCheck == kCheck - 1) {
            int done = checked;
            while (done < m && got[done]) ++done;
            if (!check(done)) return 1;
        }
    }
    if (!check(kMsgs)) return 1;
    // leave together: no process unmaps a slot its peer still copies out of
    const u64 token = 7;
    u64 a = 0, b = 0;
    c.mNext.asyncSendCopy(token);
    c.mPrev.asyncSendCopy(token);
    c.mNext.recv(a);
    c.mPrev.recv(b);
    return 0;
}

int main() {
    if (nulldev_shared_arena((size_t)4 << 30)) return 2;
    const std::string tag = "s" + std::to_string(getpid());
    pid_t kids[3];
    for (int p = 0; p < 3; ++p) {
        kids[p] = fork();
        if (kids[p] == 0) {
            int rc;
            try {
                rc = party_main(p, tag);
            } catch (const std::exception& e) {
                std::printf("party %d: %s\n", p, e.what());
                rc = 3;
            }
            std::fflush(stdout);  // _exit does not flush
            _exit(rc);
        }
    }
    int bad = 0;
    for (int p = 0; p < 3; ++p) {
        int st = 0;
        waitpid(kids[p], &st, 0);
        if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) {
            std::printf("party %d exited with status %d\n", p, st);
            bad = 1;
        }
    }
    if (!bad) std::printf("link_slots: ok (%.1f MiB of the null arena)\n", nulldev_arena_used() / 1048576.0);
    return bad;
}
