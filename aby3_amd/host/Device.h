// The host runtime's view of the GPU: one `Gpu` per party (device + in-order
// stream + stream-ordered caching allocator). Everything goes through the
// C-ABI of include/aby3gpu.h; this layer never calls HIP directly.
#pragma once
#include "Defines.h"
#include <aby3gpu.h>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

namespace aby3 {

// Throws std::runtime_error carrying aby3g_last_error() when rc != 0.
void gpuCheck(int rc, const char* what);
#define GPU_CALL(expr) ::aby3::gpuCheck((expr), #expr)

class Event {
public:
    Event();
    ~Event();
    Event(const Event&) = delete;
    Event& operator=(const Event&) = delete;
    void record(aby3g_stream s);
    void sync();
    aby3g_event get() const { return mEv; }

private:
    aby3g_event mEv = nullptr;
};

// One party's device context. Allocations are cached per size class and
// reused in stream order: a block freed after work was enqueued on this
// party's stream can be handed out again to later work on the same stream.
class Gpu {
public:
    explicit Gpu(int device = 0);
    ~Gpu();
    Gpu(const Gpu&) = delete;
    Gpu& operator=(const Gpu&) = delete;

    int device() const { return mDevice; }
    aby3g_stream stream() const { return mStream; }
    void bind();  // makes this the calling thread's current device/Gpu
    void sync();

    void* alloc(size_t bytes);
    void release(void* p, size_t bytes);
    size_t cachedBytes() const { return mCached; }
    void trim();  // return cached blocks to the driver

    // thread-local current Gpu (set by bind(), e.g. by Sh3Runtime::init)
    static Gpu& current();
    static bool hasCurrent();

private:
    int mDevice;
    aby3g_stream mStream = nullptr;
    std::mutex mMu;
    std::multimap<size_t, void*> mFree;
    size_t mCached = 0;
};

// Owning device allocation from a party's pool (move-only).
class DeviceBuffer {
public:
    DeviceBuffer() = default;
    DeviceBuffer(Gpu& gpu, size_t bytes) { reset(gpu, bytes); }
    explicit DeviceBuffer(size_t bytes) { reset(Gpu::current(), bytes); }
    ~DeviceBuffer() { free(); }
    DeviceBuffer(DeviceBuffer&& o) noexcept { *this = std::move(o); }
    DeviceBuffer& operator=(DeviceBuffer&& o) noexcept {
        if (this != &o) {
            free();
            mGpu = o.mGpu;
            mPtr = o.mPtr;
            mBytes = o.mBytes;
            o.mGpu = nullptr;
            o.mPtr = nullptr;
            o.mBytes = 0;
        }
        return *this;
    }
    DeviceBuffer(const DeviceBuffer&) = delete;
    DeviceBuffer& operator=(const DeviceBuffer&) = delete;

    void reset(Gpu& gpu, size_t bytes);
    void free();
    void* data() const { return mPtr; }
    template <class T>
    T* as() const { return static_cast<T*>(mPtr); }
    size_t bytes() const { return mBytes; }
    Gpu* gpu() const { return mGpu; }

private:
    Gpu* mGpu = nullptr;
    void* mPtr = nullptr;
    size_t mBytes = 0;
};

// Convenience copies on the current Gpu's stream.
void toDevice(void* dst, const void* src, size_t bytes, Gpu& gpu);
void toHost(void* dst, const void* src, size_t bytes, Gpu& gpu);  // synchronizes the stream
void d2d(void* dst, const void* src, size_t bytes, Gpu& gpu);

}  // namespace aby3
