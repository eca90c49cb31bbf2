// The host runtime's view of the GPU: one `Gpu` per party (device + in-order
// stream + stream-ordered caching allocator). Everything goes through the
// C-ABI of include/aby3gpu.h; this layer never calls HIP directly.
#pragma once
#include "Defines.h"
#include <aby3gpu.h>
#include <functional>
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
    bool done() const;  // the last recorded work completed (never blocks)
    aby3g_event get() const { return mEv; }

private:
    aby3g_event mEv = nullptr;
    int mDevice = 0;
};

// One party's device context. Allocations are cached per size class and
// reused in stream order: a block freed after work was enqueued on this
// party's stream can be handed out again to later work on the same stream.
// The cache (Pool) is shared with every buffer drawn from it, so a buffer
// that outlives its Gpu (a matrix declared outside the party's scope, a
// zero-copy message held by another party) is still freed correctly: after
// the Gpu is gone it goes straight back to the driver.
class Gpu {
public:
    explicit Gpu(int device = 0);
    ~Gpu();
    Gpu(const Gpu&) = delete;
    Gpu& operator=(const Gpu&) = delete;

    int device() const { return mDevice; }
    aby3g_stream stream() const { return mStream; }
    void bind();  // makes this the calling thread's current device/Gpu
    void sync();  // drains the main and the auxiliary stream

    // A second in-order stream of this party for work that overlaps the main
    // stream (e.g. the truncation pair's AES beside the share GEMM).
    aby3g_stream aux();
    void forkAux();             // aux waits for all work enqueued so far on the main stream
    aby3g_event recordAux();    // event: all work enqueued so far on aux
    void joinAux();             // main waits for all work enqueued so far on aux
    // Make aux() the main stream itself (fork/join become no-ops in effect);
    // for co-located parties, whose extra streams would share hardware queues.
    void aliasAux();
    bool auxAliased() const { return mAuxAliased; }

    // A stream shared by the co-located parties of one device, for work with
    // no inputs of the party's stream that should overlap it (the binary
    // engine's AND-mask draws): with three parties on a device it is the
    // fourth stream, so every stream keeps a hardware queue of its own.
    // Destroyed with the last Gpu holding it; null: such work goes to aux().
    struct SharedStream {
        aby3g_stream s = nullptr;
        int device = 0;
        explicit SharedStream(int device);
        ~SharedStream();
    };
    void setDrawStream(std::shared_ptr<SharedStream> s) { mDraw = std::move(s); }
    aby3g_stream drawStream() const { return mDraw ? mDraw->s : nullptr; }

    struct FreeBlock {
        void* ptr;
        std::vector<std::unique_ptr<Event>> fences;  // other streams' last uses
    };
    struct Pool {
        std::mutex mu;
        int device = 0;
        aby3g_stream stream = nullptr;  // owner's stream; null once the Gpu is gone
        std::multimap<size_t, FreeBlock> free;
        size_t cached = 0;
        // returns a block: cached while the owner lives, else freed at once
        void release(void* p, size_t bytes, std::vector<std::unique_ptr<Event>>&& fences);
    };

    void* alloc(size_t bytes);
    const std::shared_ptr<Pool>& pool() const { return mPool; }
    size_t cachedBytes() const {
        std::lock_guard<std::mutex> lk(mPool->mu);  // other parties' threads release late buffers into it
        return mPool->cached;
    }
    void trim();  // return cached blocks to the driver

    // Per-Gpu cache of derived device data (uploaded circuits, tables): the
    // object made by `make` on the first call with `key`, released with the Gpu.
    std::shared_ptr<void> attachment(u64 key, const std::function<std::shared_ptr<void>()>& make);

    // Device-side time this party's kernels spent waiting for peers inside
    // the kernels (in-kernel hand-offs: aby3g_handoff.wait_ticks), a device
    // counter in 100 MHz ticks written only by kernels on this party's stream.
    u64* waitTicks();
    double waitUs();  // reads the counter (synchronizes this party's stream)

    // thread-local current Gpu (set by bind(), e.g. by Sh3Runtime::init)
    static Gpu& current();
    static bool hasCurrent();

private:
    int mDevice;
    aby3g_stream mStream = nullptr;
    aby3g_stream mAux = nullptr;
    bool mAuxAliased = false;  // aliasAux(): the auxiliary stream is the main stream
    std::unique_ptr<Event> mForkEv, mAuxEv;
    std::shared_ptr<Pool> mPool;
    std::mutex mAttachMu;
    std::map<u64, std::shared_ptr<void>> mAttach;
    std::shared_ptr<SharedStream> mDraw;
    u64* mWaitTicks = nullptr;
};

// Owning device allocation from a party's pool (move-only). A buffer handed
// to another party's stream (zero-copy messages) is fenced by each consumer
// after it enqueued its last use; the block returns to the owner's pool
// behind those fences.
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
            mPool = std::move(o.mPool);
            mPtr = o.mPtr;
            mBytes = o.mBytes;
            mFences = std::move(o.mFences);
            mParent = std::move(o.mParent);
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
    Gpu* gpu() const { return mGpu; }  // valid while the allocating Gpu lives
    // records "stream s is done with this buffer as of now" (thread-safe)
    void fence(aby3g_stream s);
    // [off, off + bytes) of `parent` as a buffer of its own: keeps the parent
    // alive, and its fences are the parent's (one fence after the last use
    // of any view covers them all)
    static std::shared_ptr<DeviceBuffer> view(const std::shared_ptr<DeviceBuffer>& parent, size_t off, size_t bytes);
    // memory this buffer does not own (e.g. a region of an IPC-mapped arena):
    // fence() works, nothing is freed
    static std::shared_ptr<DeviceBuffer> borrow(void* ptr, size_t bytes, Gpu* gpu);

private:
    struct Fences {
        std::mutex mu;
        std::vector<std::unique_ptr<Event>> events;
    };
    Gpu* mGpu = nullptr;  // the allocating party (informational; may be gone)
    std::shared_ptr<Gpu::Pool> mPool;
    void* mPtr = nullptr;
    size_t mBytes = 0;
    std::unique_ptr<Fences> mFences;
    std::shared_ptr<DeviceBuffer> mParent;  // views only
};

// The device's count of in-kernel hand-off timeouts so far (aby3g_handoff_status):
// compare before and after a run.
u32 handoffTimeouts(int device);
// Streams of this process currently alive on `device` (aby3g_stream_count).
int liveStreams(int device);

// Convenience copies on the current Gpu's stream.
void toDevice(void* dst, const void* src, size_t bytes, Gpu& gpu);
void toHost(void* dst, const void* src, size_t bytes, Gpu& gpu);  // synchronizes the stream
void d2d(void* dst, const void* src, size_t bytes, Gpu& gpu);

}  // namespace aby3
