#include "Sh3Runtime.h"
#include <algorithm>
#include <iostream>

namespace aby3 {

// ----------------------------------------------------------------- Scheduler
void Scheduler::addReady(i64 idx) {
    auto it = mTasks.find(idx);
    if (idx > mTaskIdx || it == mTasks.end() || !it->second.up.empty()) throw RTE_LOC;
    mReady.push_back(idx);
}
void Scheduler::addNextRound(i64 idx) {
    auto it = mTasks.find(idx);
    if (idx > mTaskIdx || it == mTasks.end() || !it->second.up.empty()) throw RTE_LOC;
    mNextRound.push_back(idx);
}

static void addUnique(std::vector<i64>& v, i64 x) {
    if (std::find(v.begin(), v.end(), x) == v.end()) v.push_back(x);
}
static void removeOne(std::vector<i64>& v, i64 x) {
    auto it = std::find(v.begin(), v.end(), x);
    if (it == v.end()) throw RTE_LOC;
    std::swap(*it, v.back());
    v.pop_back();
}

i64 Scheduler::addTask(TaskType t, const std::vector<i64>& deps) {
    const i64 idx = mTaskIdx++;
    Node& n = mTasks.emplace(idx, Node{t, {}, {}, {}}).first->second;
    for (i64 d : deps) {
        if (d != -1 && d >= idx) throw RTE_LOC;
        auto db = mTasks.find(d);
        if (db != mTasks.end()) {  // dependency still pending
            addUnique(db->second.down, idx);
            addUnique(n.up, d);
        }
    }
    if (n.up.empty()) addReady(idx);
    return idx;
}

i64 Scheduler::addClosure(const std::vector<i64>& deps) {
    const i64 idx = mTaskIdx++;
    Node n{TaskType::Continuation, {}, {}, {}};
    for (i64 d : deps) {
        if (d != -1 && d >= idx) throw RTE_LOC;
        auto db = mTasks.find(d);
        if (db != mTasks.end()) {
            addUnique(db->second.closures, idx);
            addUnique(n.up, d);
        }
    }
    // a closure over completed tasks is itself complete
    if (!n.up.empty()) mTasks.emplace(idx, std::move(n));
    return idx;
}

i64 Scheduler::currentTask() {
    if (mReady.empty()) std::swap(mReady, mNextRound);
    if (mReady.empty()) throw std::runtime_error("no task is ready (a dependency can never complete) " LOCATION);
    return mReady.front();
}

void Scheduler::popTask() {
    if (mReady.empty()) throw RTE_LOC;
    const i64 idx = mReady.front();
    removeTask(idx);
    mReady.pop_front();
}

void Scheduler::removeTask(i64 idx) {
    auto it = mTasks.find(idx);
    if (it == mTasks.end() || !it->second.up.empty()) throw RTE_LOC;
    const std::vector<i64> down = it->second.down;
    const std::vector<i64> closures = it->second.closures;
    for (i64 d : down) {
        auto ds = mTasks.find(d);
        if (ds == mTasks.end()) throw RTE_LOC;
        removeOne(ds->second.up, idx);
        if (ds->second.up.empty()) {
            if (ds->second.type == TaskType::Round)
                addNextRound(d);
            else
                addReady(d);
        }
        // closures watching this task now also watch what it spawned
        for (i64 c : closures) {
            auto cc = mTasks.find(c);
            if (cc == mTasks.end()) throw RTE_LOC;
            addUnique(ds->second.closures, c);
            addUnique(cc->second.up, d);
        }
    }
    // Innermost closure first (the latest created): a task chained on an inner
    // closure -- asyncEvaluate(self, ...).then(getOutput) inside a task whose
    // closure the caller waits on (Sh3Converter.cpp:111) -- belongs to the
    // outer closure too, so every outer closure also waits on the inner ones
    // and through them on what is chained after them. (The reference's
    // Task.h:263-271 releases both at once and can leave that task behind.)
    std::vector<i64> cl = closures;
    std::sort(cl.begin(), cl.end(), std::greater<i64>());
    for (size_t a = 0; a < cl.size(); ++a) {
        auto cc = mTasks.find(cl[a]);
        if (cc == mTasks.end()) continue;
        for (size_t b = a + 1; b < cl.size(); ++b) {
            auto outer = mTasks.find(cl[b]);
            if (outer == mTasks.end()) continue;
            addUnique(cc->second.closures, cl[b]);
            addUnique(outer->second.up, cl[a]);
        }
        removeOne(cc->second.up, idx);
        if (cc->second.up.empty()) removeTask(cl[a]);
    }
    mTasks.erase(idx);
}

// ------------------------------------------------------------------- Sh3Task
Sh3Task Sh3Task::then(RoundFunc task, std::string name) const {
    return getRuntime().addTask({*this}, std::move(task), std::move(name));
}
Sh3Task Sh3Task::then(ContinuationFunc task, std::string name) const {
    return getRuntime().addTask({*this}, std::move(task), std::move(name));
}
Sh3Task Sh3Task::getClosure() const { return getRuntime().addClosure(*this); }
Sh3Task Sh3Task::operator&&(const Sh3Task& o) const { return getRuntime().addAnd({*this, o}, {}); }
Sh3Task Sh3Task::operator&=(const Sh3Task& o) {
    *this = *this && o;
    return *this;
}
void Sh3Task::get() const { getRuntime().runUntilTaskCompletes(*this); }
bool Sh3Task::isCompleted() const { return mRuntime->mSched.mTasks.find(mIdx) == mRuntime->mSched.mTasks.end(); }

// ---------------------------------------------------------------- Sh3Runtime
Sh3Runtime::~Sh3Runtime() {
    if (!mSched.mTasks.empty()) std::cerr << "~~~~~~~~~~~~~~~~ Runtime not empty!!! ~~~~~~~~~~~~~~~~" << std::endl;
}

void Sh3Runtime::init(u64 partyIdx, CommPkg& comm, int device) {
    mPartyIdx = partyIdx;
    mComm = comm;
    mNullTask.mRuntime = this;
    mNullTask.mIdx = -1;
    if (device >= 0) {
        mGpu = std::make_unique<Gpu>(device);
        mGpu->bind();
    }
}

static std::vector<i64> depIdx(const std::vector<Sh3Task>& deps) {
    std::vector<i64> v;
    v.reserve(deps.size());
    for (auto& d : deps) v.push_back(d.mIdx);
    return v;
}

Sh3Task Sh3Runtime::addTask(const std::vector<Sh3Task>& deps, Sh3Task::RoundFunc&& f, std::string&& name) {
    if (!f) throw std::runtime_error("empty task (round function) " LOCATION);
    i64 idx = mSched.addTask(TaskType::Round, depIdx(deps));
    TaskFn& t = mFns[idx];
    t.kind = 0;
    t.round = std::move(f);
    t.name = std::move(name);
    return {this, idx};
}

Sh3Task Sh3Runtime::addTask(const std::vector<Sh3Task>& deps, Sh3Task::ContinuationFunc&& f, std::string&& name) {
    if (!f) throw std::runtime_error("empty task (continuation) " LOCATION);
    // Sh3Runtime.cpp:118 adds continuations as Type::Round as well
    i64 idx = mSched.addTask(TaskType::Round, depIdx(deps));
    TaskFn& t = mFns[idx];
    t.kind = 1;
    t.cont = std::move(f);
    t.name = std::move(name);
    return {this, idx};
}

Sh3Task Sh3Runtime::addClosure(Sh3Task dep) { return {this, mSched.addClosure({dep.mIdx})}; }

Sh3Task Sh3Runtime::addAnd(const std::vector<Sh3Task>& deps, std::string&& name) {
    i64 idx = mSched.addTask(TaskType::Round, depIdx(deps));
    TaskFn& t = mFns[idx];
    t.kind = 2;
    t.name = std::move(name);
    return {this, idx};
}

void Sh3Runtime::runUntilTaskCompletes(Sh3Task task) {
    while (!task.isCompleted()) runNext();
}

void Sh3Runtime::runAll() {
    while (!mFns.empty()) runNext();
}

void Sh3Runtime::runOneRound() {
    if (mSched.mTasks.empty()) return;
    mSched.currentTask();
    while (!mSched.mReady.empty()) runNext();
}

void Sh3Runtime::runNext() {
    if (mIsActive)
        throw std::runtime_error(
            "The runtime is currently running a different task. Do not call Sh3Task.get() recursively. " LOCATION);
    const i64 idx = mSched.currentTask();
    auto it = mFns.find(idx);
    if (it == mFns.end()) throw RTE_LOC;
    TaskFn fn = std::move(it->second);  // the body may add tasks (rehash)
    mFns.erase(it);
    Sh3Task self{this, idx};
    if (mGpu) mGpu->bind();
    mIsActive = true;
    try {
        if (fn.kind == 0)
            fn.round(mComm, self);
        else if (fn.kind == 1)
            fn.cont(self);
    } catch (...) {
        mIsActive = false;
        throw;
    }
    mIsActive = false;
    mSched.popTask();
}

}  // namespace aby3
