// One party per process on the null device: the driver forks three
// processes, each runs aby3h_party_create for its party (shared-memory links,
// "IPC" slots in a shared arena) and steps / checks / destroys every job.
// Built with -fsanitize=address by tests/test_host_asan.py. Compute results
// are meaningless here; the test covers the cross-process transport's
// message order, sizes, slot reuse and teardown.
#include <aby3.h>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <sys/wait.h>
#include <unistd.h>
#include <vector>

extern "C" int nulldev_shared_arena(size_t bytes);
extern "C" void nulldev_stats(unsigned* peer_bits, unsigned long* kind3_copies);
extern "C" unsigned long nulldev_blocking_calls();

// ownDevice: party p on device p (the north-star layout, three GPUs): the
// receiver's copy out of the sender's staging slot is then a peer copy
// forceRemote: one device, every cross-GPU branch taken (colocated = 2)
static int party_main(int party, const std::string& tag, bool ownDevice, bool forceRemote = false) {
    struct J {
        int job;
        std::vector<uint64_t> p;
        int steps;
    } jobs[] = {
        {ABY3H_JOB_MUL_TRUNC, {64, 48, 80, 16, 1}, 3}, {ABY3H_JOB_MUL_TRUNC, {64, 64, 64, 8, 0}, 3},
        {ABY3H_JOB_MUL, {32, 16, 8, 1}, 3},            {ABY3H_JOB_MSB, {3000}, 2},
        {ABY3H_JOB_LR, {2048, 16, 64, 16, 11}, 3},     {ABY3H_JOB_SORT, {512}, 1},
        {ABY3H_JOB_A2B, {1000}, 2},                    {ABY3H_JOB_BITINJ, {300, 20}, 2},
    };
    int k = 0;
    for (auto& j : jobs) {
        const std::string link = tag + "." + std::to_string(k++);
        aby3h_session* s = aby3h_party_create(j.job, j.p.data(), (int)j.p.size(), party, ownDevice ? party : 0,
                                              link.c_str(), ownDevice ? 0 : (forceRemote ? 2 : 1), 0);
        if (!s) {
            std::printf("FAIL party %d create job %d: %s\n", party, j.job, aby3h_last_error());
            return 1;
        }
        const unsigned long b0 = nulldev_blocking_calls();
        if (aby3h_session_run(s, j.steps)) {
            std::printf("FAIL party %d job %d: %s\n", party, j.job, aby3h_last_error());
            return 1;
        }
        // no device-wide wait while the parties run (a host blocked in one
        // cannot enqueue what a peer's waiting kernel needs)
        if (nulldev_blocking_calls() != b0) {
            std::printf("FAIL party %d job %d: %lu device-wide waits inside session_run\n", party, j.job,
                        nulldev_blocking_calls() - b0);
            return 1;
        }
        if (aby3h_session_check(s) == 2) {
            std::printf("FAIL party %d job %d: %s\n", party, j.job, aby3h_last_error());
            return 1;
        }
        double info[ABY3H_INFO_COUNT];
        aby3h_session_info(s, info, ABY3H_INFO_COUNT);
        aby3h_session_destroy(s);
    }
    if (ownDevice) {
        unsigned peers = 0;
        unsigned long kind3 = 0;
        nulldev_stats(&peers, &kind3);
        if (!kind3) {
            std::printf("FAIL party %d: no peer copy on its own device\n", party);
            return 1;
        }
    }
    return 0;
}

int main(int argc, char** argv) {
    if (nulldev_shared_arena((size_t)4 << 30)) return 2;
    // `party_procs <party> <tag>`: one party only, started by a launcher
    // (tests/test_dist.py: three gloo ranks, one party each, sharing the
    // named arena ND_ARENA)
    if (argc == 3) return party_main(atoi(argv[1]), argv[2], false);
    int bad = 0;
    // one device, a device per party, one device with the cross-GPU branches
    for (int own = 0; own < 3 && !bad; ++own) {
        const std::string tag = "t" + std::to_string(getpid()) + "d" + std::to_string(own);
        pid_t kids[3];
        for (int p = 0; p < 3; ++p) {
            kids[p] = fork();
            if (kids[p] == 0) _exit(party_main(p, tag, own == 1, own == 2));
        }
        for (int p = 0; p < 3; ++p) {
            int st = 0;
            waitpid(kids[p], &st, 0);
            if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) {
                std::printf("party %d exited with status %d (%s)\n", p, st, own == 1 ? "own devices" : own == 2 ? "one device, remote branches" : "one device");
                bad = 1;
            }
        }
    }
    if (!bad) std::printf("party_procs: ok\n");
    return bad;
}
