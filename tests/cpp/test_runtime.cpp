// Scheduler / Sh3Runtime contract, restating the reference's
// Task_schedule_test and Sh3_Runtime_schedule_test
// (aby3_tests/Sh3RuntimeTests.cpp:15-154, 156-266): exact execution order.
// CPU-only (the runtime is created without a device).
#include "Channel.h"
#include "Sh3Runtime.h"
#include <cstdio>
#include <functional>

using namespace aby3;

static int failures = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) throw std::runtime_error("check failed: " #c " @" LOCATION); \
    } while (0)

static void run(const char* name, std::function<void()> f) {
    try {
        f();
        std::printf("PASS %s\n", name);
    } catch (const std::exception& e) {
        ++failures;
        std::printf("FAIL %s: %s\n", name, e.what());
    }
}

static void task_schedule_test() {
    Scheduler rt;
    const i64 base = -1;
    i64 task0 = rt.addTask(TaskType::Round, {base});
    i64 task1 = rt.addTask(TaskType::Round, {base});
    i64 task2 = rt.addTask(TaskType::Round, {task0, task1});
    i64 task1b = rt.addTask(TaskType::Round, {base});
    i64 task2b = rt.addTask(TaskType::Round, {task2});
    i64 close1 = rt.addClosure({task2});
    i64 task3 = rt.addTask(TaskType::Round, {close1});

    CHECK(rt.currentTask() == task0);
    rt.popTask();
    CHECK(rt.currentTask() == task1);
    rt.popTask();
    CHECK(rt.currentTask() == task1b);
    rt.popTask();
    CHECK(rt.currentTask() == task2);
    i64 task2c = rt.addTask(TaskType::Round, {task2});
    rt.popTask();
    CHECK(rt.currentTask() == task2b);
    rt.popTask();
    CHECK(rt.currentTask() == task2c);
    rt.popTask();
    CHECK(rt.currentTask() == task3);
    rt.popTask();
}

static void runtime_schedule_test() {
    Sh3Runtime rt;
    CommPkg comm;
    rt.init(0, comm, -1);
    int counter = 0;
    auto base = rt.noDependencies();

    auto task0 = base.then([&](CommPkg&, Sh3Task) { CHECK(counter++ == 0); }, "task0");
    auto task1 = base.then([&](CommPkg&, Sh3Task) { CHECK(counter++ == 1); }, "task1");
    auto task2 = (task0 && task1)
                     .then(
                         [&](CommPkg&, Sh3Task self) {
                             CHECK(counter++ == 2);
                             self.then([&](CommPkg&, Sh3Task) { CHECK(counter++ == 5); }, "task2-sub1")
                                 .then([&](CommPkg&, Sh3Task) { CHECK(counter++ == 6); }, "task2-sub2");
                         },
                         "task2");
    task2.then([&](Sh3Task) { CHECK(counter++ == 4); }, "task2-cont.");
    auto task3 = task2.getClosure().then([&](CommPkg&, Sh3Task) { CHECK(counter++ == 7); }, "task3");

    task2.get();
    CHECK(counter++ == 3);
    task3.get();
    CHECK(counter++ == 8);

    base.then([&](CommPkg&, Sh3Task self) {
        CHECK(counter++ == 9);
        self.then([&](CommPkg&, Sh3Task) { CHECK(counter++ == 12); });
    });
    base.then([&](CommPkg&, Sh3Task self) {
        CHECK(counter++ == 10);
        self.then([&](CommPkg&, Sh3Task) { CHECK(counter++ == 13); });
    });
    rt.runOneRound();
    CHECK(counter++ == 11);
    rt.runOneRound();
    CHECK(counter++ == 14);
    rt.runAll();
    CHECK(counter++ == 15);
}

static void reentrancy_test() {
    Sh3Runtime rt;
    CommPkg comm;
    rt.init(0, comm, -1);
    bool threw = false;
    rt.noDependencies().then([&](CommPkg&, Sh3Task self) {
        auto inner = self.then([](CommPkg&, Sh3Task) {});
        try {
            inner.get();  // Sh3Runtime.cpp:274-275 forbids this
        } catch (const std::runtime_error&) {
            threw = true;
        }
    });
    rt.runAll();
    CHECK(threw);
}

// A task chained on an inner closure inside a task (asyncEvaluate(self,
// ...).then(getOutput), Sh3Converter.cpp:111) completes before the outer
// closure does.
static void nested_closure_test() {
    Sh3Runtime rt;
    CommPkg comm;
    rt.init(0, comm, -1);
    int counter = 0;
    auto outer = rt.noDependencies()
                     .then([&](CommPkg&, Sh3Task self) {
                         auto inner = self.then([&](CommPkg&, Sh3Task s2) {
                             s2.then([&](CommPkg&, Sh3Task s3) {
                                 s3.then([&](CommPkg&, Sh3Task) { CHECK(counter++ == 0); }, "round-3");
                             }, "round-2");
                         }, "round-1");
                         inner.getClosure().then([&](Sh3Task) { CHECK(counter++ == 1); }, "output");
                     })
                     .getClosure();
    outer.get();
    CHECK(counter == 2);
}

// The in-kernel hand-off residency rule (Channel.h): two spinning consumer
// launches + the other spinners must leave the producer a CU.
static void handoff_residency_test() {
    // MI355X as measured: 256 CUs, one 32-slot workgroup (16 waves) or five
    // 8-slot workgroups per CU (94 VGPRs), four hardware queues
    HandoffResidency r{256, 1, 5, 128, 4};
    CHECK(handoffResidencyOk(r, 1));
    CHECK(handoffResidencyOk(r, 64));    // light levels (C3's last five)
    CHECK(handoffResidencyOk(r, 125));   // 2 * 125 + 4 + 1 = 255
    CHECK(!handoffResidencyOk(r, 126));  // 257 CUs: a small-form consumer pair could fill the chip
    CHECK(handoffResidencyOk(r, 128));   // the large form: 2 * 26 + 5
    CHECK(handoffResidencyOk(r, 512));   // 2^20 rows: 2 * 103 + 5 = 211
    CHECK(handoffResidencyOk(r, 625));
    CHECK(!handoffResidencyOk(r, 626));
    // a register regression to 4 waves per SIMD: the 2^20-row messages go back
    // to the stream hand-off (2 * 128 + 5 > 256), smaller ones stay
    r.perCuLarge = 4;
    CHECK(!handoffResidencyOk(r, 512));
    CHECK(handoffResidencyOk(r, 500));
    CHECK(!handoffResidencyOk(r, 501));
    // a part with fewer CUs: the small form's limit drops below the large form's
    HandoffResidency s{80, 1, 5, 128, 4};
    CHECK(handoffResidencyOk(s, 37));
    CHECK(!handoffResidencyOk(s, 38));
    CHECK(!handoffResidencyOk(s, 100));  // small form (16-wave workgroups), 2 * 100 + 5 > 80
    CHECK(handoffResidencyOk(s, 185));   // large form: 2 * 37 + 5 = 79
    // three processes on one GPU (the IPC arenas): three processes' queues of
    // stream-op waits, 2 * 103 + 12 + 1 = 219 CUs for 2^20-row messages
    r = HandoffResidency{256, 1, 5, 128, 4};
    CHECK(handoffResidencyOk(r, 512, 3));
    CHECK(handoffResidencyOk(r, 500, 3));
    CHECK(handoffResidencyOk(r, 605, 3));   // 2 * 121 + 13 = 255
    CHECK(!handoffResidencyOk(r, 606, 3));
    r.perCuLarge = 4;
    CHECK(!handoffResidencyOk(r, 500, 3));  // 2 * 125 + 13 > 256
    CHECK(handoffResidencyOk(r, 484, 3));   // 2 * 121 + 13 = 255
    CHECK(!handoffResidencyOk(r, 485, 3));
    r.perCuLarge = 5;
    CHECK(!handoffResidencyOk(r, 512, 0));  // no process count, no hand-off
    // a kernel that cannot be resident at all never hands off in-kernel
    HandoffResidency z{256, 0, 0, 128, 4};
    CHECK(!handoffResidencyOk(z, 1));
    CHECK(!handoffResidencyOk(r, 0));
}

int main() {
    run("handoff_residency_test", handoff_residency_test);
    run("Task_schedule_test", task_schedule_test);
    run("Sh3_Runtime_schedule_test", runtime_schedule_test);
    run("Sh3_Runtime_reentrancy_test", reentrancy_test);
    run("nested_closure_test", nested_closure_test);
    return failures ? 1 : 0;
}
