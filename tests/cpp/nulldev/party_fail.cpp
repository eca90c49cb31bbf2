// Failing fast between party processes (ADVICE/VERDICT r05: a party that
// failed its setup left a peer spinning for the whole link timeout and
// another blocked in a stream sync until the harness killed it). On the null
// device: three forked processes, one party each, running the C2-shaped
// multiplication job; party 1 fails -- (1) a copy of its setup fails, as a
// faulted device's next call does, (2) its process exits right after the
// ring is built, without closing. Both peers must exit non-zero within 2 s
// of party 1's exit, each naming the cause (the LinkEnd abort word / the
// watchdog's dead-peer check, Link.cpp). Built with -fsanitize=address by
// tests/test_host_asan.py.
#include <aby3.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <sys/wait.h>
#include <unistd.h>
#include <vector>

extern "C" int nulldev_shared_arena(size_t bytes);
extern "C" void nulldev_fail_nth_memcpy(long n);

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int party_main(int party, const std::string& link, int mode) {
    std::vector<uint64_t> p = {64, 48, 80, 16, 1};
    if (party == 1 && mode == 1) nulldev_fail_nth_memcpy(1);
    aby3h_session* s = aby3h_party_create(ABY3H_JOB_MUL_TRUNC, p.data(), (int)p.size(), party, 0, link.c_str(), 2, 0);
    if (!s) {
        std::printf("party %d: create failed: %s\n", party, aby3h_last_error());
        std::fflush(stdout);
        return 3;
    }
    if (party == 1 && mode == 2) _exit(7);  // gone without closing its links
    if (aby3h_session_run(s, 3)) {
        std::printf("party %d: run failed: %s\n", party, aby3h_last_error());
        std::fflush(stdout);
        aby3h_session_destroy(s);
        return 4;
    }
    // the revealed check needs every party (a party that only sends can finish
    // its steps without its peer)
    if (aby3h_session_check(s) == 2) {
        std::printf("party %d: check failed: %s\n", party, aby3h_last_error());
        std::fflush(stdout);
        aby3h_session_destroy(s);
        return 5;
    }
    aby3h_session_destroy(s);
    std::printf("party %d: finished without noticing the failure\n", party);
    std::fflush(stdout);
    return 0;
}

int main() {
    if (nulldev_shared_arena((size_t)1 << 28)) return 2;
    int bad = 0;
    for (int mode = 1; mode <= 2; ++mode) {
        const std::string link = "pf" + std::to_string(getpid()) + "m" + std::to_string(mode);
        pid_t kids[3];
        for (int q = 0; q < 3; ++q) {
            kids[q] = fork();
            if (kids[q] == 0) _exit(party_main(q, link, mode));
        }
        double tExit[3] = {0, 0, 0};
        int st[3] = {0, 0, 0};
        for (int left = 3; left > 0; --left) {
            int s = 0;
            const pid_t w = waitpid(-1, &s, 0);
            for (int q = 0; q < 3; ++q)
                if (kids[q] == w) {
                    tExit[q] = now();
                    st[q] = s;
                }
        }
        for (int q = 0; q < 3; ++q) {
            const bool ok = WIFEXITED(st[q]) && WEXITSTATUS(st[q]) != 0;
            if (!ok) {
                std::printf("mode %d: party %d ended with status %d (expected a non-zero exit)\n", mode, q, st[q]);
                bad = 1;
            }
        }
        for (int q : {0, 2}) {
            const double lag = tExit[q] - tExit[1];
            std::printf("mode %d: party %d exited %.3f s after party 1\n", mode, q, lag);
            if (lag > 2.0) bad = 1;
        }
    }
    if (!bad) std::printf("party_fail: ok\n");
    return bad;
}
