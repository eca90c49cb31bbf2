#include "Device.h"
#include "Link.h"
#include <mutex>
#include <vector>
#include <map>

namespace aby3 {

namespace {
thread_local Gpu* t_current = nullptr;

size_t sizeClass(size_t bytes) {
    if (bytes <= 512) return 512;
    // round up to 1/8 of the next power of two to bound internal waste
    size_t p = 1;
    while (p < bytes) p <<= 1;
    size_t step = p / 8;
    return (bytes + step - 1) / step * step;
}
}  // namespace

void gpuCheck(int rc, const char* what) {
    if (rc == 0) return;
    std::string m = std::string(what) + ": " + aby3g_last_error();
    if (rc == ABY3G_EHIP) {
        // an error of the HIP runtime may be a device fault of earlier work
        char recent[1024];
        if (aby3g_recent_calls(recent, sizeof recent) == 0 && recent[0]) m += " [recent calls, newest first: " + std::string(recent) + "]";
    }
    throw std::runtime_error(m);
}

// Events are recycled: a protocol round creates several (message readiness,
// buffer fences) and creating + destroying a HIP event costs two runtime
// calls. An Event is only destroyed after every wait on it was enqueued, and
// a wait refers to the record preceding it, so re-recording a recycled event
// cannot affect earlier waits.
namespace {
struct EventCache {
    std::mutex mu;
    std::map<int, std::vector<aby3g_event>> free;  // per device
};
EventCache& eventCache() {
    static EventCache* c = new EventCache;  // never destroyed: events may die during static teardown
    return *c;
}
constexpr size_t kEventCacheMax = 4096;
}  // namespace

Event::Event() {
    GPU_CALL(aby3g_get_device(&mDevice));
    {
        EventCache& c = eventCache();
        std::lock_guard<std::mutex> lk(c.mu);
        auto& v = c.free[mDevice];
        if (!v.empty()) {
            mEv = v.back();
            v.pop_back();
            return;
        }
    }
    GPU_CALL(aby3g_event_create(&mEv));
}
Event::~Event() {
    if (!mEv) return;
    {
        EventCache& c = eventCache();
        std::lock_guard<std::mutex> lk(c.mu);
        auto& v = c.free[mDevice];
        if (v.size() < kEventCacheMax) {
            v.push_back(mEv);
            return;
        }
    }
    aby3g_event_destroy(mEv);
}
void Event::record(aby3g_stream s) { GPU_CALL(aby3g_event_record(mEv, s)); }
void Event::sync() { GPU_CALL(aby3g_event_sync(mEv)); }
bool Event::done() const {
    int d = 0;
    GPU_CALL(aby3g_event_query(mEv, &d));
    return d != 0;
}

Gpu::Gpu(int device) : mDevice(device) {
    GPU_CALL(aby3g_set_device(device));
    GPU_CALL(aby3g_stream_create(&mStream));
    mPool = std::make_shared<Pool>();
    mPool->device = device;
    mPool->stream = mStream;
}

Gpu::~Gpu() {
    aby3g_set_device(mDevice);
    aby3g_stream_sync(mStream);
    if (mAux) aby3g_stream_sync(mAux);
    if (mDraw) aby3g_stream_sync(mDraw->s);  // draws into this party's buffers
    mAttach.clear();
    trim();
    {
        // buffers still alive elsewhere now free straight to the driver
        std::lock_guard<std::mutex> lk(mPool->mu);
        mPool->stream = nullptr;
    }
    mForkEv.reset();
    mAuxEv.reset();
    if (mAux && !mAuxAliased) aby3g_stream_destroy(mAux);
    if (mWaitTicks) aby3g_free(mWaitTicks);
    aby3g_stream_destroy(mStream);
    if (t_current == this) t_current = nullptr;
}

Gpu::SharedStream::SharedStream(int dev) : device(dev) {
    GPU_CALL(aby3g_set_device(dev));
    GPU_CALL(aby3g_stream_create(&s));
}
Gpu::SharedStream::~SharedStream() {
    aby3g_set_device(device);
    aby3g_stream_sync(s);
    aby3g_stream_destroy(s);
}

void Gpu::bind() {
    GPU_CALL(aby3g_set_device(mDevice));
    t_current = this;
}

void Gpu::sync() {
    GPU_CALL(aby3g_stream_sync(mStream));
    if (mAux) GPU_CALL(aby3g_stream_sync(mAux));
    // one party per process: a failed peer's waits were released (~0 signal
    // words, LinkEnd's watchdog), so the stream drained on garbage -- an error
    if (LinkEnd::failed()) throw std::runtime_error("stream drained after a party failure: " + LinkEnd::failure());
}

u64* Gpu::waitTicks() {
    if (!mWaitTicks) {
        GPU_CALL(aby3g_set_device(mDevice));
        void* p = nullptr;
        GPU_CALL(aby3g_malloc(&p, 8));
        // zeroed in this stream's order: only this party's kernels add to it
        GPU_CALL(aby3g_memset(p, 0, 8, mStream));
        mWaitTicks = (u64*)p;
    }
    return mWaitTicks;
}

double Gpu::waitUs() {
    if (!mWaitTicks) return 0.0;
    u64 t = 0;
    toHost(&t, mWaitTicks, 8, *this);
    return (double)t * 0.01;  // 100 MHz wall clock
}

aby3g_stream Gpu::aux() {
    if (!mAux) {
        GPU_CALL(aby3g_set_device(mDevice));
        if (mAuxAliased)
            mAux = mStream;
        else
            GPU_CALL(aby3g_stream_create(&mAux));
        mForkEv = std::make_unique<Event>();
        mAuxEv = std::make_unique<Event>();
    }
    return mAux;
}

void Gpu::forkAux() {
    aby3g_stream a = aux();
    if (mAuxAliased) return;  // one stream: already in order
    mForkEv->record(mStream);
    GPU_CALL(aby3g_stream_wait_event(a, mForkEv->get()));
}

void Gpu::aliasAux() {
    if (mAux && !mAuxAliased) throw std::runtime_error("Gpu::aliasAux after the auxiliary stream was created");
    mAuxAliased = true;
}

aby3g_event Gpu::recordAux() {
    aux();
    mAuxEv->record(mAux);
    return mAuxEv->get();
}

void Gpu::joinAux() {
    if (aux() == mStream) return;
    GPU_CALL(aby3g_stream_wait_event(mStream, recordAux()));
}

void* Gpu::alloc(size_t bytes) {
    size_t cls = sizeClass(bytes);
    {
        std::lock_guard<std::mutex> lk(mPool->mu);
        auto it = mPool->free.find(cls);
        if (it != mPool->free.end()) {
            void* p = it->second.ptr;
            for (auto& ev : it->second.fences) GPU_CALL(aby3g_stream_wait_event(mStream, ev->get()));
            mPool->free.erase(it);
            mPool->cached -= cls;
            return p;
        }
    }
    void* p = nullptr;
    GPU_CALL(aby3g_set_device(mDevice));
    if (aby3g_malloc(&p, cls) != 0) {
        // Out of memory. No recovery here: returning the cache to the driver
        // (hipFree) waits for the whole device, and mid-protocol that wait can
        // block on a peer's kernel that waits for this party's next launch.
        // The session trims the pools between runs instead, once a party's
        // cache passes ABY3_POOL_TRIM_MB (aby3h_session_run, Session.cpp).
        size_t cached;
        {
            std::lock_guard<std::mutex> lk(mPool->mu);
            cached = mPool->cached;
        }
        throw std::runtime_error(std::string("device out of memory allocating ") + std::to_string(cls) +
                                 " bytes (" + std::to_string(cached) + " bytes cached by this party's pool; " +
                                 "runs trim it past ABY3_POOL_TRIM_MB): " + aby3g_last_error());
    }
    return p;
}

void Gpu::Pool::release(void* p, size_t bytes, std::vector<std::unique_ptr<Event>>&& fences) {
    if (!p) return;
    const size_t cls = sizeClass(bytes);
    std::unique_lock<std::mutex> lk(mu);
    if (stream) {
        free.emplace(cls, FreeBlock{p, std::move(fences)});
        cached += cls;
        return;
    }
    lk.unlock();
    // the owner is gone: wait for the other streams' last uses, then free
    for (auto& ev : fences) ev->sync();
    aby3g_set_device(device);
    aby3g_device_sync();
    aby3g_free(p);
}

void Gpu::trim() {
    std::lock_guard<std::mutex> lk(mPool->mu);
    bool fenced = false;
    for (auto& kv : mPool->free) fenced = fenced || !kv.second.fences.empty();
    if (fenced) aby3g_device_sync();  // fenced blocks may still be read by other streams
    for (auto& kv : mPool->free) aby3g_free(kv.second.ptr);
    mPool->free.clear();
    mPool->cached = 0;
}

std::shared_ptr<void> Gpu::attachment(u64 key, const std::function<std::shared_ptr<void>()>& make) {
    std::lock_guard<std::mutex> lk(mAttachMu);
    auto it = mAttach.find(key);
    if (it != mAttach.end()) return it->second;
    auto v = make();
    mAttach.emplace(key, v);
    return v;
}

Gpu& Gpu::current() {
    if (!t_current) throw std::runtime_error("no current Gpu on this thread (call Gpu::bind / Sh3Runtime::init)");
    return *t_current;
}
bool Gpu::hasCurrent() { return t_current != nullptr; }

void DeviceBuffer::reset(Gpu& gpu, size_t bytes) {
    free();
    mGpu = &gpu;
    mPool = gpu.pool();
    mBytes = bytes;
    mPtr = gpu.alloc(bytes ? bytes : 8);
    mFences = std::make_unique<Fences>();  // created here: fence() may race from several consumer threads
}

std::shared_ptr<DeviceBuffer> DeviceBuffer::view(const std::shared_ptr<DeviceBuffer>& parent, size_t off,
                                                 size_t bytes) {
    if (!parent || off + bytes > parent->mBytes) throw std::runtime_error("DeviceBuffer::view out of range");
    auto v = std::make_shared<DeviceBuffer>();
    v->mGpu = parent->mGpu;
    v->mPtr = static_cast<char*>(parent->mPtr) + off;
    v->mBytes = bytes;
    v->mParent = parent;
    return v;
}

std::shared_ptr<DeviceBuffer> DeviceBuffer::borrow(void* ptr, size_t bytes, Gpu* gpu) {
    auto v = std::make_shared<DeviceBuffer>();
    v->mGpu = gpu;
    v->mPtr = ptr;
    v->mBytes = bytes;
    v->mFences = std::make_unique<Fences>();
    return v;
}

void DeviceBuffer::fence(aby3g_stream s) {
    if (mParent) {
        mParent->fence(s);
        return;
    }
    if (!mPtr) return;
    if (mPool) {
        // the owner's stream: the pool reuses blocks in that stream's order anyway
        std::lock_guard<std::mutex> lk(mPool->mu);
        if (mPool->stream == s) return;
    }
    auto ev = std::make_unique<Event>();
    ev->record(s);
    std::lock_guard<std::mutex> lk(mFences->mu);
    mFences->events.push_back(std::move(ev));
}

void DeviceBuffer::free() {
    if (mParent) {
        mParent.reset();
        mPtr = nullptr;
        mGpu = nullptr;
        mBytes = 0;
        return;
    }
    if (mPtr && mPool) {
        std::vector<std::unique_ptr<Event>> fences;
        if (mFences) fences = std::move(mFences->events);
        mPool->release(mPtr, mBytes ? mBytes : 8, std::move(fences));
    }
    mFences.reset();
    mPool.reset();
    mPtr = nullptr;
    mGpu = nullptr;
    mBytes = 0;
}

u32 handoffTimeouts(int device) {
    u32 n = 0;
    GPU_CALL(aby3g_set_device(device));
    GPU_CALL(aby3g_handoff_status(&n));
    return n;
}
int liveStreams(int device) {
    int n = 0;
    GPU_CALL(aby3g_stream_count(device, &n));
    return n;
}

void toDevice(void* dst, const void* src, size_t bytes, Gpu& gpu) {
    GPU_CALL(aby3g_memcpy(dst, src, bytes, 0, gpu.stream()));
    // the host source may be reused by the caller right away
    gpu.sync();
}
void toHost(void* dst, const void* src, size_t bytes, Gpu& gpu) {
    GPU_CALL(aby3g_memcpy(dst, src, bytes, 1, gpu.stream()));
    gpu.sync();
}
void d2d(void* dst, const void* src, size_t bytes, Gpu& gpu) {
    // both buffers are this party's (its device): the copy-kernel path
    GPU_CALL(aby3g_memcpy(dst, src, bytes, 2, gpu.stream()));
}

}  // namespace aby3
