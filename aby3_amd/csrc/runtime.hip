// Runtime plumbing of the C-ABI: errors, device memory, streams, events, the
// kernel-timing probe, and the host half of AES (key schedule, T-table).
#include "common.h"
#include <atomic>
#include <cstring>
#include <mutex>
#include <map>

namespace aby3g {

thread_local double t_api_us = 0;
thread_local u64 t_api_calls = 0;

namespace {
thread_local std::string t_err;

struct ProbeRec {
    hipEvent_t a, b;
    int family;
};
struct Probe {
    bool on = false;
    u32 mask = 0;  // families bracketed
    hipEvent_t pending = nullptr;
    std::vector<ProbeRec> recs;
    double ms[8] = {0};
    u64 launches[8] = {0};
    std::vector<hipEvent_t> pool;
    hipEvent_t get() {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        hipEvent_t e;
        ABY3G_CHECK_HIP(hipEventCreate(&e));
        return e;
    }
    void drain() {
        for (auto& r : recs) {
            ABY3G_CHECK_HIP(hipEventSynchronize(r.b));
            float t = 0;
            ABY3G_CHECK_HIP(hipEventElapsedTime(&t, r.a, r.b));
            ms[r.family] += t;
            launches[r.family] += 1;
            pool.push_back(r.a);
            pool.push_back(r.b);
        }
        recs.clear();
    }
};
thread_local Probe t_probe;

// FIPS-197 S-box from its definition (inverse in GF(2^8), then the affine
// map), evaluated at compile time: the host keeps a copy and the T-table is a
// device global initialised by the code object's loader, so no copy -- and no
// null-stream operation -- is needed to get it onto a device (a null-stream
// memcpy at the first AES launch would create the null stream's hardware
// queue mid-run and could block behind a spinning kernel).
constexpr u8 gf_mul(u8 a, u8 b) {
    u8 p = 0;
    for (int i = 0; i < 8; ++i) {
        if (b & 1) p ^= a;
        const bool hi = a & 0x80;
        a = (u8)(a << 1);
        if (hi) a ^= 0x1b;
        b >>= 1;
    }
    return p;
}
constexpr u8 gf_inv(u8 x) {  // x^254 (0 -> 0)
    u8 r = 1, base = x;
    for (unsigned e = 254; e; e >>= 1) {
        if (e & 1) r = gf_mul(r, base);
        base = gf_mul(base, base);
    }
    return x ? r : 0;
}
struct Tables {
    u8 sbox[256];
    u32 T0[256];
};
constexpr Tables make_tables() {
    Tables t{};
    for (int x = 0; x < 256; ++x) {
        const u8 inv = gf_inv((u8)x);
        u8 r = 0x63;
        for (int i = 0; i < 8; ++i) {
            const int bit = ((inv >> i) ^ (inv >> ((i + 4) & 7)) ^ (inv >> ((i + 5) & 7)) ^ (inv >> ((i + 6) & 7)) ^
                             (inv >> ((i + 7) & 7))) & 1;
            r ^= (u8)(bit << i);
        }
        t.sbox[x] = r;
        const u8 s2 = gf_mul(r, 2), s3 = gf_mul(r, 3);
        t.T0[x] = (u32)s2 | ((u32)r << 8) | ((u32)r << 16) | ((u32)s3 << 24);
    }
    return t;
}
constexpr Tables kTables = make_tables();
static_assert(kTables.sbox[0] == 0x63 && kTables.sbox[1] == 0x7c && kTables.sbox[0x53] == 0xed, "FIPS-197 S-box");
const Tables& tables() { return kTables; }

std::mutex g_tab_mu;
std::map<int, u32*> g_tab_dev;
std::map<int, u32*> g_status_dev;  // per device: in-kernel hand-off timeouts (under g_tab_mu)
}  // namespace

// The AES T-table as a device global, initialised by the code object's loader
// from the compile-time table (externally linked and writable: the runtime
// registers such a variable; a const one in an anonymous namespace was folded
// into read-only data and could not be found by hipGetSymbolAddress).
struct AesT0Table {
    u32 v[256];
};
constexpr AesT0Table make_aes_t0() {
    AesT0Table t{};
    for (int i = 0; i < 256; ++i) t.v[i] = kTables.T0[i];
    return t;
}
__device__ AesT0Table aby3g_aes_t0_dev = make_aes_t0();

// Pinned host memory, so neither the kernels' timeout path nor the host's
// reads need a stream: HIP's null stream is never touched (it would take one
// of the process's hardware queues and make two party streams share one).
u32* handoff_status_word() {
    const int dev = current_device();
    std::lock_guard<std::mutex> lk(g_tab_mu);
    auto it = g_status_dev.find(dev);
    if (it != g_status_dev.end()) return it->second;
    void* p = nullptr;
    ABY3G_CHECK_HIP(hipHostMalloc(&p, 256, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(p, 0, 256);
    g_status_dev[dev] = (u32*)p;
    return (u32*)p;
}

static std::atomic<u64> g_handoff_timeout_ticks{kHandoffTimeoutTicks};
u64 handoff_timeout_ticks() { return g_handoff_timeout_ticks.load(std::memory_order_relaxed); }

void set_error(const std::string& msg) { t_err = msg; }
thread_local int t_device = -1;

void probe_begin(int family, hipStream_t s) {
    if (!t_probe.on || !((t_probe.mask >> family) & 1)) return;
    t_probe.pending = t_probe.get();
    ABY3G_CHECK_HIP(hipEventRecord(t_probe.pending, s));
}
void probe_end(int family, hipStream_t s) {
    if (!t_probe.on || !t_probe.pending) return;
    hipEvent_t b = t_probe.get();
    ABY3G_CHECK_HIP(hipEventRecord(b, s));
    t_probe.recs.push_back(ProbeRec{t_probe.pending, b, family});
    t_probe.pending = nullptr;
    if (t_probe.recs.size() > 4096) t_probe.drain();
}

AesKey expand_key(const u8 key[16]) {
    const u8* S = tables().sbox;
    AesKey k;
    for (int c = 0; c < 4; ++c)
        k.rk[c] = (u32)key[4 * c] | ((u32)key[4 * c + 1] << 8) | ((u32)key[4 * c + 2] << 16) |
                  ((u32)key[4 * c + 3] << 24);
    u32 rcon = 1;
    for (int i = 4; i < 44; ++i) {
        u32 t = k.rk[i - 1];
        if (i % 4 == 0) {
            t = (t >> 8) | (t << 24);  // RotWord on a little-endian word
            t = (u32)S[t & 0xff] | ((u32)S[(t >> 8) & 0xff] << 8) | ((u32)S[(t >> 16) & 0xff] << 16) |
                ((u32)S[t >> 24] << 24);
            t ^= rcon;
            rcon = (rcon << 1) ^ ((rcon & 0x80) ? 0x11b : 0);
        }
        k.rk[i] = k.rk[i - 4] ^ t;
    }
    return k;
}

int current_device() {
    if (t_device < 0) ABY3G_CHECK_HIP(hipGetDevice(&t_device));
    return t_device;
}

const u32* aes_table() {
    const int dev = current_device();
    std::lock_guard<std::mutex> lk(g_tab_mu);
    auto it = g_tab_dev.find(dev);
    if (it != g_tab_dev.end()) return it->second;
    void* p = nullptr;
    ABY3G_CHECK_HIP(hipGetSymbolAddress(&p, HIP_SYMBOL(aby3g_aes_t0_dev)));
    g_tab_dev[dev] = (u32*)p;
    return (u32*)p;
}

static std::atomic<u64> g_call_n{0};
static std::atomic<const char*> g_calls[32];
void note_call(const char* name) {
    g_calls[g_call_n.fetch_add(1, std::memory_order_relaxed) & 31].store(name, std::memory_order_relaxed);
}

namespace {
// dst[0, n) <- src[0, n) in 16-byte pieces (both 16-byte aligned), grid-stride
__global__ void __launch_bounds__(256) k_copy16(uint4* __restrict__ dst, const uint4* __restrict__ src, u64 n) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) dst[i] = src[i];
}
__global__ void __launch_bounds__(256) k_copy1(u8* __restrict__ dst, const u8* __restrict__ src, u64 n) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) dst[i] = src[i];
}
}  // namespace

void launch_copy(void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (!bytes) return;
    const bool aligned = (((uintptr_t)dst | (uintptr_t)src | bytes) & 15) == 0;
    const u64 n = aligned ? bytes / 16 : bytes;
    const u32 grid = (u32)std::min<u64>((n + 255) / 256, 2048);
    if (aligned)
        launch(PROBE_OTHER, k_copy16, dim3(grid), dim3(256), 0, s, (uint4*)dst, (const uint4*)src, n);
    else
        launch(PROBE_OTHER, k_copy1, dim3(grid), dim3(256), 0, s, (u8*)dst, (const u8*)src, n);
}

}  // namespace aby3g

using namespace aby3g;

extern "C" {

const char* aby3g_last_error(void) { return t_err.c_str(); }
int aby3g_recent_calls(char* out, size_t cap) {
    if (!out || !cap) return ABY3G_EINVAL;
    std::string r;
    const u64 n = g_call_n.load(std::memory_order_relaxed);
    for (u64 k = 0; k < 32 && k < n; ++k) {
        const char* c = g_calls[(n - 1 - k) & 31].load(std::memory_order_relaxed);
        if (!c) continue;
        if (!r.empty()) r += " < ";
        r += c;
    }
    std::strncpy(out, r.c_str(), cap - 1);
    out[cap - 1] = 0;
    return ABY3G_OK;
}
int aby3g_version(void) { return 1; }

int aby3g_device_count(int* n) {
    return guarded([&] { ABY3G_CHECK_HIP(hipGetDeviceCount(n)); });
}
int aby3g_set_device(int device) {
    // hipSetDevice / hipGetDevice are not free (they serialise with the other
    // threads' launches: 15-100 us per call measured with three party
    // threads); the library remembers the device it last set on this thread
    // and skips the call when it is unchanged
    return guarded([&] {
        if (t_device == device) return;
        ABY3G_CHECK_HIP(hipSetDevice(device));
        t_device = device;
    });
}
int aby3g_api_time(double* us, uint64_t* calls) {
    *us = t_api_us;
    *calls = t_api_calls;
    return 0;
}
int aby3g_get_device(int* device) {
    return guarded([&] { *device = current_device(); });
}

int aby3g_malloc(void** ptr, size_t bytes) {
    return guarded([&] {
        hipError_t e = hipMalloc(ptr, bytes ? bytes : 16);
        if (e != hipSuccess) throw Error{ABY3G_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e)};
    });
}
int aby3g_malloc_uncached(void** ptr, size_t bytes) {
    return guarded([&] {
        hipError_t e = hipExtMallocWithFlags(ptr, bytes ? bytes : 16, hipDeviceMallocUncached);
        if (e != hipSuccess) throw Error{ABY3G_ENOMEM, std::string("hipExtMallocWithFlags: ") + hipGetErrorString(e)};
    });
}
int aby3g_free(void* ptr) {
    return guarded([&] { ABY3G_CHECK_HIP(hipFree(ptr)); });
}
int aby3g_host_malloc(void** ptr, size_t bytes) {
    return guarded([&] { ABY3G_CHECK_HIP(hipHostMalloc(ptr, bytes ? bytes : 16, hipHostMallocDefault)); });
}
int aby3g_host_free(void* ptr) {
    return guarded([&] { ABY3G_CHECK_HIP(hipHostFree(ptr)); });
}
int aby3g_memcpy(void* dst, const void* src, size_t bytes, int kind, aby3g_stream stream) {
    return guarded([&] {
        if (!bytes) return;
        hipMemcpyKind k = kind == 0   ? hipMemcpyHostToDevice
                          : kind == 1 ? hipMemcpyDeviceToHost
                          : kind == 2 ? hipMemcpyDeviceToDevice
                                      : hipMemcpyDefault;
        if (k == hipMemcpyDeviceToDevice) {
            // device-to-device on the current device: one copy kernel, cheaper to
            // issue than the runtime's blit path
            launch_copy(dst, src, bytes, S(stream));
            return;
        }
        ABY3G_CHECK_HIP(hipMemcpyAsync(dst, src, bytes, k, S(stream)));
    });
}
int aby3g_memset(void* dst, int value, size_t bytes, aby3g_stream stream) {
    return guarded([&] {
        if (bytes) ABY3G_CHECK_HIP(hipMemsetAsync(dst, value, bytes, S(stream)));
    });
}
static std::mutex g_stream_mu;
static std::map<hipStream_t, int> g_streams;  // live streams -> device
int aby3g_stream_create(aby3g_stream* stream) {
    return guarded([&] {
        hipStream_t s;
        ABY3G_CHECK_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        *stream = s;
        std::lock_guard<std::mutex> lk(g_stream_mu);
        g_streams[s] = current_device();
    });
}
int aby3g_stream_destroy(aby3g_stream stream) {
    return guarded([&] {
        ABY3G_CHECK_HIP(hipStreamDestroy(S(stream)));
        std::lock_guard<std::mutex> lk(g_stream_mu);
        g_streams.erase(S(stream));
    });
}
int aby3g_null_queue_init(void) {
    return guarded([&] {
        static std::mutex mu;
        static std::map<int, void*> done;  // per device: the word the null stream zeroed
        const int dev = current_device();
        std::lock_guard<std::mutex> lk(mu);
        if (done.count(dev)) return;
        void* q = nullptr;
        ABY3G_CHECK_HIP(hipMalloc(&q, 256));
        ABY3G_CHECK_HIP(hipMemset(q, 0, 256));  // the null stream: its hardware queue is created here
        done[dev] = q;
    });
}
int aby3g_stream_count(int device, int* n) {
    return guarded([&] {
        ABY3G_REQUIRE(n != nullptr, "null argument");
        std::lock_guard<std::mutex> lk(g_stream_mu);
        int c = 0;
        for (const auto& e : g_streams) c += e.second == device;
        *n = c;
    });
}
int aby3g_stream_sync(aby3g_stream stream) {
    return guarded([&] { ABY3G_CHECK_HIP(hipStreamSynchronize(S(stream))); });
}
int aby3g_device_sync(void) {
    return guarded([&] { ABY3G_CHECK_HIP(hipDeviceSynchronize()); });
}
int aby3g_event_create(aby3g_event* ev) {
    return guarded([&] {
        hipEvent_t e;
        ABY3G_CHECK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        *ev = e;
    });
}
int aby3g_event_create_timed(aby3g_event* ev) {
    return guarded([&] {
        hipEvent_t e;
        ABY3G_CHECK_HIP(hipEventCreate(&e));
        *ev = e;
    });
}
int aby3g_event_destroy(aby3g_event ev) {
    return guarded([&] { ABY3G_CHECK_HIP(hipEventDestroy((hipEvent_t)ev)); });
}
int aby3g_event_record(aby3g_event ev, aby3g_stream stream) {
    return guarded([&] { ABY3G_CHECK_HIP(hipEventRecord((hipEvent_t)ev, S(stream))); });
}
int aby3g_event_sync(aby3g_event ev) {
    return guarded([&] { ABY3G_CHECK_HIP(hipEventSynchronize((hipEvent_t)ev)); });
}
int aby3g_event_query(aby3g_event ev, int* done) {
    return guarded([&] {
        ABY3G_REQUIRE(done != nullptr, "null argument");
        const hipError_t e = hipEventQuery((hipEvent_t)ev);
        if (e == hipErrorNotReady) {
            *done = 0;
            return;
        }
        ABY3G_CHECK_HIP(e);
        *done = 1;
    });
}
int aby3g_stream_wait_event(aby3g_stream stream, aby3g_event ev) {
    return guarded([&] { ABY3G_CHECK_HIP(hipStreamWaitEvent(S(stream), (hipEvent_t)ev, 0)); });
}
int aby3g_event_elapsed_ms(aby3g_event start, aby3g_event end, float* ms) {
    return guarded([&] { ABY3G_CHECK_HIP(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)end)); });
}
int aby3g_signal_alloc(uint64_t** word) {
    return guarded([&] {
        ABY3G_REQUIRE(word != nullptr, "null word");
        ABY3G_CHECK_HIP(hipMalloc(word, sizeof(uint64_t)));
        // zeroed on a stream of its own and waited for, not on the null
        // stream (whose hardware queue would be created here and shared with
        // a party's stream)
        hipStream_t s;
        ABY3G_CHECK_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        const hipError_t e1 = hipMemsetAsync(*word, 0, sizeof(uint64_t), s);
        const hipError_t e2 = e1 == hipSuccess ? hipStreamSynchronize(s) : e1;
        (void)hipStreamDestroy(s);
        ABY3G_CHECK_HIP(e2);
    });
}
int aby3g_stream_write_value(aby3g_stream stream, uint64_t* word, uint64_t value) {
    return guarded([&] { ABY3G_CHECK_HIP(hipStreamWriteValue64(S(stream), word, value, 0)); });
}
int aby3g_stream_wait_value(aby3g_stream stream, uint64_t* word, uint64_t value) {
    return guarded(
        [&] { ABY3G_CHECK_HIP(hipStreamWaitValue64(S(stream), word, value, hipStreamWaitValueGte, ~0ull)); });
}

int aby3g_handoff_status(uint32_t* timeouts) {
    return guarded([&] {
        ABY3G_REQUIRE(timeouts != nullptr, "null argument");
        *timeouts = *(volatile u32*)handoff_status_word();
    });
}
int aby3g_set_handoff_timeout_us(uint64_t us) {
    return guarded([&] {
        ABY3G_REQUIRE(us >= 1 && us <= 60000000ull, "timeout must be 1 us .. 60 s");
        g_handoff_timeout_ticks.store(us * 100, std::memory_order_relaxed);  // 100 MHz wall clock
    });
}

static_assert(sizeof(aby3g_ipc_handle) == sizeof(hipIpcMemHandle_t), "IPC handle size");
int aby3g_ipc_get_handle(void* ptr, aby3g_ipc_handle* handle) {
    return guarded([&] {
        ABY3G_REQUIRE(ptr != nullptr && handle != nullptr, "null argument");
        // whole 2 MiB-granular allocations only (include/aby3gpu.h)
        void* base = nullptr;
        size_t size = 0;
        ABY3G_CHECK_HIP(hipMemGetAddressRange(&base, &size, ptr));
        ABY3G_REQUIRE(base == ptr, "IPC export of a pointer inside an allocation");
        ABY3G_REQUIRE(size % ABY3G_IPC_GRANULE == 0, "IPC export of an allocation that is not a multiple of 2 MiB");
        hipIpcMemHandle_t h;
        ABY3G_CHECK_HIP(hipIpcGetMemHandle(&h, ptr));
        std::memcpy(handle->bytes, &h, sizeof(h));
    });
}
int aby3g_ipc_open(const aby3g_ipc_handle* handle, void** ptr) {
    return guarded([&] {
        ABY3G_REQUIRE(ptr != nullptr && handle != nullptr, "null argument");
        hipIpcMemHandle_t h;
        std::memcpy(&h, handle->bytes, sizeof(h));
        ABY3G_CHECK_HIP(hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess));
    });
}
int aby3g_ipc_close(void* ptr) {
    return guarded([&] { ABY3G_CHECK_HIP(hipIpcCloseMemHandle(ptr)); });
}
int aby3g_host_register(void* host, size_t bytes, void** dev) {
    return guarded([&] {
        ABY3G_REQUIRE(host != nullptr && dev != nullptr && ((uintptr_t)host & 4095) == 0, "host memory must be page aligned");
        ABY3G_CHECK_HIP(hipHostRegister(host, bytes, hipHostRegisterMapped));
        ABY3G_CHECK_HIP(hipHostGetDevicePointer(dev, host, 0));
    });
}
int aby3g_host_unregister(void* host) {
    return guarded([&] { ABY3G_CHECK_HIP(hipHostUnregister(host)); });
}
int aby3g_device_uuid(int device, uint8_t uuid[16]) {
    return guarded([&] {
        ABY3G_REQUIRE(uuid != nullptr, "null argument");
        hipUUID u;
        ABY3G_CHECK_HIP(hipDeviceGetUuid(&u, device));
        std::memcpy(uuid, u.bytes, 16);
    });
}
int aby3g_enable_peer_access(int device, int peer) {
    return guarded([&] {
        if (device == peer) return;
        int can = 0;
        ABY3G_CHECK_HIP(hipDeviceCanAccessPeer(&can, device, peer));
        ABY3G_REQUIRE(can, "devices cannot access each other's memory (no peer path)");
        int cur = 0;
        ABY3G_CHECK_HIP(hipGetDevice(&cur));
        ABY3G_CHECK_HIP(hipSetDevice(device));
        hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
        (void)hipSetDevice(cur);
        if (e == hipErrorPeerAccessAlreadyEnabled) {
            (void)hipGetLastError();
            return;
        }
        ABY3G_CHECK_HIP(e);
    });
}

// the T-table image the AES round function reads, built once on the host
static const std::vector<u32>& host_aes_tables() {
    static const std::vector<u32> rep = [] {
        std::vector<u32> r(kAesLdsWords);
        for (int i = 0; i < kAesLdsWords; ++i) {
            const u32 v = tables().T0[i >> 6];
            r[i] = (i & 32) ? rotl(v, 8) : v;
        }
        return r;
    }();
    return rep;
}

int aby3g_aes_block_host(const uint8_t key[16], uint64_t ctr, uint8_t out[16]) {
    return guarded([&] {
        const std::vector<u32>& rep = host_aes_tables();
        AesKey k = expand_key(key);
        u64 lo, hi;
        aes_ctr_block(rep.data(), 0, k, ctr, lo, hi);
        std::memcpy(out, &lo, 8);
        std::memcpy(out + 8, &hi, 8);
    });
}

int aby3g_aes_ctr_host(const uint8_t key[16], uint64_t ctr_base, uint64_t nblocks, uint8_t* out) {
    return guarded([&] {
        ABY3G_REQUIRE(key && (out || !nblocks), "null key or output");
        const std::vector<u32>& rep = host_aes_tables();
        AesKey k = expand_key(key);
        for (u64 i = 0; i < nblocks; ++i) {
            u64 lo, hi;
            aes_ctr_block(rep.data(), 0, k, ctr_base + i, lo, hi);
            std::memcpy(out + 16 * i, &lo, 8);
            std::memcpy(out + 16 * i + 8, &hi, 8);
        }
    });
}

int aby3g_probe_enable(int on) {
    return guarded([&] {
        if (!on) t_probe.drain();
        t_probe.on = on != 0;
        t_probe.mask = on ? 0xffu : 0u;
    });
}
int aby3g_probe_enable_mask(uint32_t mask) {
    return guarded([&] {
        if (!mask) t_probe.drain();
        t_probe.on = mask != 0;
        t_probe.mask = mask;
    });
}
int aby3g_probe_read(int family, double* ms, uint64_t* launches) {
    return guarded([&] {
        ABY3G_REQUIRE(family >= 0 && family < 8, "family out of range");
        t_probe.drain();
        *ms = t_probe.ms[family];
        *launches = t_probe.launches[family];
    });
}
int aby3g_probe_reset(void) {
    return guarded([&] {
        t_probe.drain();
        for (int i = 0; i < 8; ++i) {
            t_probe.ms[i] = 0;
            t_probe.launches[i] = 0;
        }
    });
}

}  // extern "C"
