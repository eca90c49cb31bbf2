// Host-runtime memory-safety driver: sessions of every job created, stepped,
// checked and destroyed back to back, plus the three-party sim entry points,
// linked against the null device (gen_nulldev.py) and built with
// -fsanitize=address by tests/test_host_asan.py. Compute results are
// meaningless here; only the host code's memory behaviour is under test.
#include <aby3.h>
#include <cstdio>
#include <cstring>
#include <vector>

extern "C" void nulldev_stats(unsigned* peer_bits, unsigned long* kind3_copies);
extern "C" unsigned long nulldev_blocking_calls();

static int fail(const char* what) {
    std::printf("FAIL %s: %s\n", what, aby3h_last_error());
    return 1;
}

int main() {
    const int dev[3] = {0, 0, 0};
    struct J {
        int job;
        std::vector<uint64_t> p;
        int steps;
    } jobs[] = {
        {ABY3H_JOB_MUL_TRUNC, {64, 48, 80, 16, 1}, 3}, {ABY3H_JOB_MUL_TRUNC, {64, 64, 64, 8, 0}, 3},
        {ABY3H_JOB_MUL, {32, 32, 32, 0}, 3},           {ABY3H_JOB_MUL, {32, 16, 8, 1}, 3},
        {ABY3H_JOB_MSB, {3000}, 2},                    {ABY3H_JOB_LR, {2048, 16, 64, 16, 11}, 3},
        {ABY3H_JOB_SORT, {4096}, 1},                  {ABY3H_JOB_MUL_TRUNC, {64, 48, 80, 16, 1}, 2},
        // row splits (rows [32, 64) of 64; rows [42, 63) of 63)
        {ABY3H_JOB_MUL_TRUNC, {64, 48, 80, 16, 1, 1, 1, 2}, 2}, {ABY3H_JOB_MUL_TRUNC, {63, 48, 80, 16, 1, 1, 2, 3}, 2},
        {ABY3H_JOB_MSB, {5000, 1, 2}, 2},  // rows [2048, 5000) of 5000
        {ABY3H_JOB_MSB, {1000, 0, 2}, 2},  // an empty slice
    };
    // rounds 0 / 1: the three parties on one device, without and with probes;
    // round 2: each on its own device (the north-star layout inside one
    // process): peer access both ways and peer copies of staged messages
    const int dev3[3] = {0, 1, 2};
    for (int round = 0; round < 3; ++round)
        for (auto& j : jobs) {
            aby3h_session* s =
                aby3h_session_create(j.job, j.p.data(), (int)j.p.size(), round == 2 ? dev3 : dev, round == 1);
            if (!s) return fail("create");
            // no device-wide wait while the parties run (the r04h
            // hand-off timeouts): setup may synchronise, a step may not
            const unsigned long b0 = nulldev_blocking_calls();
            if (aby3h_session_run(s, j.steps)) return fail("run");
            if (nulldev_blocking_calls() != b0) {
                std::printf("FAIL job %d round %d: %lu device-wide waits (sync / free / signal-word zeroing) "
                            "inside session_run\n", j.job, round, nulldev_blocking_calls() - b0);
                return 1;
            }
            if (aby3h_session_check(s) == 2) return fail("check");
            if (j.job == ABY3H_JOB_MUL_TRUNC) {  // the result's shares: the slice's rows x N
                const uint64_t S = j.p.size() > 7 ? j.p[7] : 1, k = j.p.size() > 7 ? j.p[6] : 0;
                const uint64_t want = (j.p[0] * (k + 1) / S - j.p[0] * k / S) * j.p[2];
                std::vector<int64_t> r(want + 1);
                uint64_t n = 0;
                if (aby3h_session_result(s, 1, 1, r.data(), r.size(), &n)) return fail("result");
                if (n != want) {
                    std::printf("FAIL job params %zu: result of %lu elements, expected %lu\n", j.p.size(),
                                (unsigned long)n, (unsigned long)want);
                    return 1;
                }
            }
            double ms;
            uint64_t n;
            aby3h_session_probe(s, 0, &ms, &n);
            aby3h_session_destroy(s);
        }
    unsigned peers = 0;
    unsigned long kind3 = 0;
    nulldev_stats(&peers, &kind3);
    if (peers != 0xEEu) {  // every ordered pair of distinct devices
        std::printf("FAIL peer access enabled for pairs 0x%x, expected 0xee\n", peers);
        return 1;
    }
    if (!kind3) {
        std::printf("FAIL no copy between devices on three devices\n");
        return 1;
    }
    std::printf("cross-device: peer pairs 0x%x, %lu copies between devices\n", peers, kind3);
    std::vector<int64_t> a(64 * 48, 3), b(48 * 80, 5), sh(6 * 64 * 80), pl(64 * 80);
    // row splits the jobs refuse: a shard past the last, a split Hadamard product
    for (const auto& bad : {std::vector<uint64_t>{64, 64, 64, 16, 1, 1, 2, 2}, {64, 64, 64, 16, 0, 1, 0, 2}}) {
        if (aby3h_session* s = aby3h_session_create(ABY3H_JOB_MUL_TRUNC, bad.data(), (int)bad.size(), dev, 0)) {
            aby3h_session_destroy(s);
            std::printf("FAIL a bad row split was accepted\n");
            return 1;
        }
        if (!std::strstr(aby3h_last_error(), "row split")) {
            std::printf("FAIL bad row split: unexpected error '%s'\n", aby3h_last_error());
            return 1;
        }
    }
    if (aby3h_sim_mul(0, 1, 1, 16, a.data(), b.data(), 64, 48, 80, sh.data(), pl.data())) return fail("sim_mul");
    // empty shapes: no rows, no inner dimension (a zero product, then truncated), no columns
    for (const auto& s3 : {std::vector<uint64_t>{0, 5, 7}, {5, 0, 7}, {5, 7, 0}}) {
        for (int trunc = 0; trunc < 2; ++trunc)
            if (aby3h_sim_mul(0, 1, trunc, 16, a.data(), b.data(), s3[0], s3[1], s3[2], sh.data(), pl.data()))
                return fail("sim_mul (empty shape)");
    }
    std::vector<int64_t> x(300, 1), y(300, 2), o(300), osh(6 * 300);
    if (aby3h_sim_cipher_gt(0, x.data(), y.data(), 300, o.data(), osh.data())) return fail("sim_cipher_gt");
    // the merge network: general shapes (padding, explicit row lists) and
    // the high-dimensional forms
    const uint64_t lens[] = {5, 7, 8, 3, 2, 6};
    std::vector<int64_t> keys(31, 1), sorted(31), msh(6 * 31);
    for (int mode = 0; mode < 4; ++mode) {
        const uint64_t n = mode == 3 ? 4 : 6, dim = mode >= 2 ? 2 : 0;
        if (aby3h_sim_merge(0, mode, lens, n, dim, keys.data(), sorted.data(), msh.data())) return fail("sim_merge");
    }
    std::vector<int64_t> lx(500 * 8, 1 << 16), ly(500, 0), wsh(6 * 8), wpl(8);
    std::vector<uint64_t> lb(2 * 64);
    if (aby3h_lr_batches(500, 64, 2, lb.data())) return fail("lr_batches");
    if (aby3h_sim_lr(0, 500, 8, 64, 16, 11, 2, lx.data(), ly.data(), lb.data(), wsh.data(), wpl.data()))
        return fail("sim_lr");
    std::printf("session_asan: ok\n");
    return 0;
}
