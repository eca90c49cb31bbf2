// TEST INFRASTRUCTURE ONLY (bench.py's C1 cpu_baseline leg): the oracle's
// asyncMul of BASELINE configs[0] -- "Sh3Evaluator asyncMul on 128x128
// si64Matrix, 3 CPU processes over localhost" -- as three processes, one
// party each, as the reference deploys them (aby3-Basic/BuildingBlocks.cpp:
// 150-179 sets up the three parties' sessions; Eval/dis_exec.sh starts one
// process per party). Each party computes its local product and zero share
// (orc::localProduct + ShareGen, Sh3Evaluator.cpp:92-116 / :651-673) and
// sends its share to the next party, which receives it as its second share
// (the reshare round, Sh3Evaluator.cpp:104-111). The reference's channel is a
// localhost TCP socket; here each direction is a shared-memory mailbox with
// a sequence word (a copy in, a copy out, as through a socket's buffer), so
// the transport adds no more than localhost TCP would.
//
// usage: orc_c1_procs <mode 0 hadamard | 1 gemm> <M> <K> <N> <reps>
// prints one JSON line {"secs": wall seconds of the reps, "reps": reps}
#include "orc_core.h"
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sys/mman.h>
#include <sys/wait.h>
#include <thread>
#include <unistd.h>

using namespace orc;

namespace {
struct alignas(128) Word {
    std::atomic<uint64_t> v;
};
struct Ctl {
    Word ready, start, done;
    Word sent[3], taken[3];  // mailbox p: party p -> party p + 1
};

void spinUntil(const std::atomic<uint64_t>& w, uint64_t atLeast) {
    while (w.load(std::memory_order_acquire) < atLeast) std::this_thread::yield();
}

int party(int p, int mode, u64 M, u64 K, u64 N, int reps, Ctl* ctl, int64_t* box) {
    auto ev = makeEvaluators(1);  // every party's generator; party p uses its own
    std::array<SMat, 3> A, B;
    u64 x = 43;  // the inputs of orc_bench_mul, party by party
    auto rnd = [&](SMat& m, u64 r, u64 c) {
        m = SMat(r, c);
        for (int s = 0; s < 2; ++s)
            for (auto& v : m.s[s].v) {
                x ^= x << 13;
                x ^= x >> 7;
                x ^= x << 17;
                v = (i64)x;
            }
    };
    for (int q = 0; q < 3; ++q) {
        rnd(A[q], M, K);
        rnd(B[q], mode == MUL_GEMM ? K : M, mode == MUL_GEMM ? N : K);
    }
    const u64 n = M * (mode == MUL_GEMM ? N : K);
    const int prev = (p + 2) % 3;
    ctl->ready.v.fetch_add(1, std::memory_order_acq_rel);
    spinUntil(ctl->start.v, 1);
    SMat C;
    for (int r = 0; r < reps; ++r) {
        Mat c0;
        localProduct((MulMode)mode, A[p], B[p], c0);
        for (u64 k = 0; k < c0.size(); ++k) c0.v[k] = (i64)((u64)c0.v[k] + (u64)ev[p].gen.getShare());
        // send: the next party took the previous message out of the mailbox
        spinUntil(ctl->taken[p].v, (uint64_t)r);
        std::memcpy(box + (size_t)p * n, c0.v.data(), n * 8);
        ctl->sent[p].v.store((uint64_t)r + 1, std::memory_order_release);
        // receive the previous party's share
        spinUntil(ctl->sent[prev].v, (uint64_t)r + 1);
        Mat c1 = c0;
        std::memcpy(c1.v.data(), box + (size_t)prev * n, n * 8);
        ctl->taken[prev].v.store((uint64_t)r + 1, std::memory_order_release);
        C.s[0] = std::move(c0);
        C.s[1] = std::move(c1);
    }
    ctl->done.v.fetch_add(1, std::memory_order_acq_rel);
    return 0;
}
}  // namespace

int main(int argc, char** argv) {
    if (argc != 6) {
        std::fprintf(stderr, "usage: %s mode M K N reps\n", argv[0]);
        return 2;
    }
    const int mode = atoi(argv[1]);
    const u64 M = strtoull(argv[2], nullptr, 10), K = strtoull(argv[3], nullptr, 10),
              N = strtoull(argv[4], nullptr, 10);
    const int reps = atoi(argv[5]);
    if ((mode != MUL_GEMM && mode != MUL_HADAMARD) || !M || !K || !N || reps < 1) return 2;
    const u64 n = M * (mode == MUL_GEMM ? N : K);
    const size_t bytes = sizeof(Ctl) + 3 * n * 8;
    void* mem = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    if (mem == MAP_FAILED) return 3;
    Ctl* ctl = new (mem) Ctl{};
    int64_t* box = (int64_t*)((char*)mem + sizeof(Ctl));
    pid_t kids[3];
    for (int p = 0; p < 3; ++p) {
        kids[p] = fork();
        if (kids[p] < 0) return 4;
        if (kids[p] == 0) _exit(party(p, mode, M, K, N, reps, ctl, box));
    }
    spinUntil(ctl->ready.v, 3);
    const auto t0 = std::chrono::steady_clock::now();
    ctl->start.v.store(1, std::memory_order_release);
    spinUntil(ctl->done.v, 3);
    const auto t1 = std::chrono::steady_clock::now();
    int bad = 0;
    for (int p = 0; p < 3; ++p) {
        int st = 0;
        waitpid(kids[p], &st, 0);
        bad |= !WIFEXITED(st) || WEXITSTATUS(st) != 0;
    }
    if (bad) return 5;
    std::printf("{\"secs\": %.9f, \"reps\": %d}\n", std::chrono::duration<double>(t1 - t0).count(), reps);
    return 0;
}
