// Round-based task scheduler of one party (aby3/Common/Task.h,
// aby3/sh3/Sh3Runtime.h/.cpp), restated. Contract kept from the reference and
// pinned by tests/cpp/test_runtime.cpp (Sh3RuntimeTests.cpp:15-266):
//   * then(f) runs f after its dependency completes; a task whose dependency
//     completed is queued for the NEXT round (Task.h:240-247) -- for round
//     functions and continuations alike (both are added as rounds,
//     Sh3Runtime.cpp:91,118);
//   * getClosure() completes when the task and everything it spawned through
//     self.then(...) complete (Task.h:157-200,250-271);
//   * a && b joins; get() drives runNext() until the task completes;
//   * runNext() is not re-entrant (Sh3Runtime.cpp:274-275).
// One Sh3Runtime per party, driven by one host thread; it also owns the
// party's Gpu (device + stream) so every kernel of the party is stream-ordered.
#pragma once
#include "Channel.h"
#include <functional>
#include <list>
#include <map>
#include <type_traits>
#include <unordered_map>

namespace aby3 {

// Move-only callable (the reference uses fu2::unique_function).
template <class Sig>
class UniqueFunction;
template <class R, class... A>
class UniqueFunction<R(A...)> {
    struct Base {
        virtual ~Base() = default;
        virtual R call(A... a) = 0;
    };
    template <class F>
    struct Impl : Base {
        F f;
        explicit Impl(F&& x) : f(std::move(x)) {}
        R call(A... a) override { return f(std::forward<A>(a)...); }
    };
    std::unique_ptr<Base> mImpl;

public:
    UniqueFunction() = default;
    template <class F, class = std::enable_if_t<std::is_invocable_r_v<R, F&, A...> &&
                                                !std::is_same_v<std::decay_t<F>, UniqueFunction>>>
    UniqueFunction(F f) : mImpl(new Impl<F>(std::move(f))) {}
    UniqueFunction(UniqueFunction&&) = default;
    UniqueFunction& operator=(UniqueFunction&&) = default;
    explicit operator bool() const { return (bool)mImpl; }
    R operator()(A... a) { return mImpl->call(std::forward<A>(a)...); }
};

enum class TaskType { Round, Continuation };

class Scheduler {
public:
    struct Node {
        TaskType type;
        std::vector<i64> up, down, closures;
    };
    i64 mTaskIdx = 0;
    std::unordered_map<i64, Node> mTasks;
    std::list<i64> mReady, mNextRound;

    i64 addTask(TaskType t, const std::vector<i64>& deps);
    i64 addClosure(const std::vector<i64>& deps);
    i64 currentTask();
    void popTask();
    void removeTask(i64 idx);

private:
    void addReady(i64 idx);
    void addNextRound(i64 idx);
};

class Sh3Runtime;

class Sh3Task {
public:
    using RoundFunc = UniqueFunction<void(CommPkg& comm, Sh3Task& self)>;
    using ContinuationFunc = UniqueFunction<void(Sh3Task& self)>;

    Sh3Runtime& getRuntime() const { return *mRuntime; }

    // schedules a task that runs in the round after this task completes
    Sh3Task then(RoundFunc task, std::string name = {}) const;
    // a continuation (in the reference it is scheduled exactly like a round)
    Sh3Task then(ContinuationFunc task, std::string name = {}) const;

    Sh3Task getClosure() const;
    Sh3Task operator&&(const Sh3Task& o) const;
    Sh3Task operator&=(const Sh3Task& o);
    void get() const;
    bool isCompleted() const;

    bool operator==(const Sh3Task& t) const { return mRuntime == t.mRuntime && mIdx == t.mIdx; }
    bool operator!=(const Sh3Task& t) const { return !(*this == t); }

    Sh3Runtime* mRuntime = nullptr;
    i64 mIdx = -1;
};

class Sh3Runtime {
public:
    Sh3Runtime() = default;
    Sh3Runtime(u64 partyIdx, CommPkg& comm, int device = 0) { init(partyIdx, comm, device); }
    ~Sh3Runtime();
    Sh3Runtime(const Sh3Runtime&) = delete;
    Sh3Runtime& operator=(const Sh3Runtime&) = delete;

    // Binds this party to `device` on the calling thread (creates its stream).
    void init(u64 partyIdx, CommPkg& comm, int device = 0);

    const Sh3Task& noDependencies() const { return mNullTask; }
    operator Sh3Task() const { return noDependencies(); }

    Sh3Task addTask(const std::vector<Sh3Task>& deps, Sh3Task::RoundFunc&& f, std::string&& name);
    Sh3Task addTask(const std::vector<Sh3Task>& deps, Sh3Task::ContinuationFunc&& f, std::string&& name);
    Sh3Task addClosure(Sh3Task dep);
    Sh3Task addAnd(const std::vector<Sh3Task>& deps, std::string&& name);

    void runUntilTaskCompletes(Sh3Task task);
    void runNext();
    void runAll();
    void runOneRound();

    Gpu& gpu() { return *mGpu; }

    u64 mPartyIdx = (u64)-1;
    CommPkg mComm;
    bool mIsActive = false;
    Scheduler mSched;
    Sh3Task mNullTask;

private:
    struct TaskFn {
        int kind = 0;  // 0 round, 1 continuation, 2 and
        Sh3Task::RoundFunc round;
        Sh3Task::ContinuationFunc cont;
        std::string name;
    };
    std::unordered_map<i64, TaskFn> mFns;
    std::unique_ptr<Gpu> mGpu;
};

}  // namespace aby3
