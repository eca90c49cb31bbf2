#include "Device.h"

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
    if (rc != 0) throw std::runtime_error(std::string(what) + ": " + aby3g_last_error());
}

Event::Event() { GPU_CALL(aby3g_event_create(&mEv)); }
Event::~Event() {
    if (mEv) aby3g_event_destroy(mEv);
}
void Event::record(aby3g_stream s) { GPU_CALL(aby3g_event_record(mEv, s)); }
void Event::sync() { GPU_CALL(aby3g_event_sync(mEv)); }

Gpu::Gpu(int device) : mDevice(device) {
    GPU_CALL(aby3g_set_device(device));
    GPU_CALL(aby3g_stream_create(&mStream));
}

Gpu::~Gpu() {
    aby3g_set_device(mDevice);
    aby3g_stream_sync(mStream);
    trim();
    aby3g_stream_destroy(mStream);
    if (t_current == this) t_current = nullptr;
}

void Gpu::bind() {
    GPU_CALL(aby3g_set_device(mDevice));
    t_current = this;
}

void Gpu::sync() { GPU_CALL(aby3g_stream_sync(mStream)); }

void* Gpu::alloc(size_t bytes) {
    size_t cls = sizeClass(bytes);
    std::lock_guard<std::mutex> lk(mMu);
    auto it = mFree.find(cls);
    if (it != mFree.end()) {
        void* p = it->second;
        mFree.erase(it);
        mCached -= cls;
        return p;
    }
    void* p = nullptr;
    GPU_CALL(aby3g_set_device(mDevice));
    int rc = aby3g_malloc(&p, cls);
    if (rc != 0) {
        // out of memory: drop the cache (after the stream drains) and retry once
        sync();
        for (auto& kv : mFree) aby3g_free(kv.second);
        mFree.clear();
        mCached = 0;
        GPU_CALL(aby3g_malloc(&p, cls));
    }
    return p;
}

void Gpu::release(void* p, size_t bytes) {
    if (!p) return;
    size_t cls = sizeClass(bytes);
    std::lock_guard<std::mutex> lk(mMu);
    mFree.emplace(cls, p);
    mCached += cls;
}

void Gpu::trim() {
    std::lock_guard<std::mutex> lk(mMu);
    for (auto& kv : mFree) aby3g_free(kv.second);
    mFree.clear();
    mCached = 0;
}

Gpu& Gpu::current() {
    if (!t_current) throw std::runtime_error("no current Gpu on this thread (call Gpu::bind / Sh3Runtime::init)");
    return *t_current;
}
bool Gpu::hasCurrent() { return t_current != nullptr; }

void DeviceBuffer::reset(Gpu& gpu, size_t bytes) {
    free();
    mGpu = &gpu;
    mBytes = bytes;
    mPtr = gpu.alloc(bytes ? bytes : 8);
}

void DeviceBuffer::free() {
    if (mPtr && mGpu) mGpu->release(mPtr, mBytes ? mBytes : 8);
    mPtr = nullptr;
    mGpu = nullptr;
    mBytes = 0;
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
    GPU_CALL(aby3g_memcpy(dst, src, bytes, 3, gpu.stream()));
}

}  // namespace aby3
