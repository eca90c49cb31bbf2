// Cross-process links (Link.h, makeProcessRing): a cyclic exchange of host
// payloads larger than a link's 4 MiB ring. Every party sends 12 MiB to the
// next party before it receives from the previous one, three times, then a
// mixed round of small and large messages; with the ring written inline by
// the sending thread this cycle waited on itself until the link timeout.
// Three forked processes on the null device (gen_nulldev.py), built with
// -fsanitize=address by tests/test_host_asan.py.
#include "Channel.h"
#include <cstdio>
#include <cstring>
#include <string>
#include <sys/wait.h>
#include <unistd.h>
#include <vector>

extern "C" int nulldev_shared_arena(size_t bytes);

using namespace aby3;

static int party_main(int p, const std::string& tag) {
    CommPkg c = makeProcessRing(p, tag, 0);
    const size_t big = 12u << 20;
    std::vector<u8> out(big), in(big);
    for (int round = 0; round < 3; ++round) {
        for (size_t i = 0; i < big; ++i) out[i] = (u8)(i * 7 + p * 31 + round);
        c.mNext.asyncSendCopy(out.data(), big);  // returns before the peer reads
        c.mPrev.recv(in.data(), big);
        const int q = (p + 2) % 3;
        for (size_t i = 0; i < big; i += 4099)
            if (in[i] != (u8)(i * 7 + q * 31 + round)) {
                std::printf("FAIL party %d round %d: byte %zu\n", p, round, i);
                return 1;
            }
    }
    // order across sizes: small, large, small to next; the same back from prev
    const u64 a = 1000 + p;
    c.mNext.asyncSendCopy(a);
    c.mNext.asyncSendCopy(out.data(), big);
    c.mNext.asyncSendCopy(a + 1);
    u64 x = 0, y = 0;
    c.mPrev.recv(x);
    c.mPrev.recv(in.data(), big);
    c.mPrev.recv(y);
    const u64 e = 1000 + (p + 2) % 3;
    if (x != e || y != e + 1) {
        std::printf("FAIL party %d: small messages %llu %llu\n", p, (unsigned long long)x, (unsigned long long)y);
        return 1;
    }
    return 0;
}

int main() {
    if (nulldev_shared_arena((size_t)1 << 28)) return 2;
    const std::string tag = "x" + std::to_string(getpid());
    pid_t kids[3];
    for (int p = 0; p < 3; ++p) {
        kids[p] = fork();
        if (kids[p] == 0) _exit(party_main(p, tag));
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
    if (!bad) std::printf("link_exchange: ok\n");
    return bad;
}
