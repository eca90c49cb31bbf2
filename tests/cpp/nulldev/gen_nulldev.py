"""Generates nulldev.cpp: a host-memory stand-in for libaby3gpu.so used ONLY
to run the C++ host runtime (scheduler, channels, pools, fences, sessions)
under AddressSanitizer on a machine without a GPU. Every compute entry point
is a no-op returning success; memory, copies, streams and events are plain
host operations. Results computed through it are meaningless -- it checks
memory safety of the host code, nothing else."""
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
HDR = os.path.join(HERE, "..", "..", "..", "include", "aby3gpu.h")

OVERRIDES = {
    "aby3g_last_error": 'return "";',
    "aby3g_version": "return 1;",
    "aby3g_recent_calls": "if (cap) out[0] = 0; return 0;",
    "aby3g_device_count": "*n = ND_DEVICES; return 0;",
    "aby3g_set_device": "if (device < 0 || device >= ND_DEVICES) return 1; t_device = device; return 0;",
    "aby3g_get_device": "*device = t_device; return 0;",
    "aby3g_enable_peer_access": "return nd_peer(device, peer);",
    "aby3g_api_time": "*us = 0; *calls = 0; return 0;",
    "aby3g_malloc": "*ptr = nd_alloc(bytes); return *ptr ? 0 : 1;",
    "aby3g_malloc_uncached": "*ptr = nd_alloc(bytes); return *ptr ? 0 : 1;",
    "aby3g_device_uuid": "memset(uuid, 0, 16); uuid[0] = (uint8_t)device; return 0;",
    "aby3g_free": "g_blocking.fetch_add(1); nd_sync_all(); nd_free(ptr); return 0;",
    "aby3g_device_sync": "g_blocking.fetch_add(1); nd_sync_all(); return 0;",
    "aby3g_host_malloc": "*ptr = calloc(1, bytes ? bytes : 1); return *ptr ? 0 : 1;",
    "aby3g_host_free": "free(ptr); return 0;",
    "aby3g_memcpy": "return nd_memcpy(dst, src, bytes, kind, stream);",
    "aby3g_memset": "if (bytes) nd_enqueue(stream, [=] { memset(dst, value, bytes); }); return 0;",
    "aby3g_stream_create": "*stream = nd_stream_new(); return 0;",
    "aby3g_stream_destroy": "nd_stream_delete(stream); return 0;",
    "aby3g_event_create": "*ev = new NdEventHandle{std::make_shared<NdEvent>()}; return 0;",
    "aby3g_event_create_timed": "*ev = new NdEventHandle{std::make_shared<NdEvent>()}; return 0;",
    "aby3g_event_destroy": "delete (NdEventHandle*)ev; return 0;",
    "aby3g_event_record": "nd_event_record(ev, stream); return 0;",
    "aby3g_event_elapsed_ms": "*ms = 0; return 0;",
    "aby3g_event_query": "*done = nd_event_done(ev) ? 1 : 0; return 0;",
    "aby3g_signal_alloc": "g_blocking.fetch_add(1); *word = (uint64_t*)nd_alloc(8); return *word ? 0 : 1;",
    "aby3g_stream_write_value": "nd_enqueue(stream, [=] { __atomic_store_n(word, value, __ATOMIC_RELEASE); }); return 0;",
    "aby3g_stream_wait_value": "if (!nd_async()) return nd_wait(word, value); nd_enqueue(stream, [=] { if (nd_wait(word, value)) nd_fatal(\"a stream wait on a signal word timed out\"); }); return 0;",
    "aby3g_ipc_get_handle": "if (!nd_ipc_exportable(ptr)) return 1; memset(handle, 0, sizeof *handle); memcpy(handle->bytes, &ptr, sizeof ptr); return 0;",
    "aby3g_ipc_open": "memcpy(ptr, handle->bytes, sizeof *ptr); nd_map_open(*ptr); return 0;",
    "aby3g_host_register": "*dev = host; return 0;",
    "aby3g_ipc_close": "nd_map_close(ptr); return 0;",
    "aby3g_stream_sync": "nd_stream_sync(stream); return 0;",
    "aby3g_event_sync": "nd_event_sync(ev); return 0;",
    "aby3g_stream_wait_event": "nd_stream_wait_event(stream, ev); return 0;",
    "aby3g_probe_read": "*ms = 0; *launches = 0; return 0;",
    "aby3g_handoff_status": "*timeouts = 0; return 0;",
    "aby3g_stream_count": "*n = 0; return 0;",
    "aby3g_null_queue_init": "return 0;",
    "aby3g_bin_level_residency": "*cus = 256; *per_cu_small = 1; *per_cu_large = 5; *small_max_wgs = 128; return 0;",
    "aby3g_aes_block_host": "for (int i = 0; i < 16; ++i) out[i] = key[i] ^ (uint8_t)(ctr >> (8 * (i & 7))); return 0;",
    "aby3g_lr_mailbox_bytes": "return 4096;",
    "aby3g_lr_scratch_bytes": "return 4096;",
    "aby3g_mul_workspace_bytes": "return mode == 1 ? (size_t)(M + 64) * (K + 64) * 16 + (N + 64) * (K + 64) * 16 + 4 * M * N * 8 : 0;",
}


# "Device" memory comes from calloc, or -- after nulldev_shared_arena(), called
# before fork() by the one-party-per-process driver -- from one MAP_SHARED
# arena that every forked party sees at the same address: an IPC handle is
# then just the pointer. Stream-ordered waits spin on the word (all "device"
# work is synchronous here, so a wait ends as soon as the peer's host code
# has run the matching write).
PREAMBLE = r"""
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <set>
#include <vector>
#include <chrono>
#include <fcntl.h>
#include <sys/mman.h>
#include <thread>
#include <unistd.h>
// three "devices" with distinct ordinals, so the host runtime's cross-device
// branches (peer access between parties' devices, peer copies of staged
// messages) run here too; the current device is per thread, as in HIP
constexpr int ND_DEVICES = 3;
static thread_local int t_device = 0;
static std::atomic<unsigned> g_peer{0};       // bit 3 * device + peer: access enabled
static std::atomic<unsigned long> g_kind3{0}; // copies between devices (kind 3)
// calls that wait for the whole device on real hardware (hipDeviceSynchronize,
// hipFree, the synchronous zeroing of a signal word): none may happen while a
// party's protocol runs -- a host blocked in one cannot enqueue the producer
// that another party's spinning consumer waits for
static std::atomic<unsigned long> g_blocking{0};
extern "C" unsigned long nulldev_blocking_calls() { return g_blocking.load(); }
static int nd_peer(int device, int peer) {
    if (device < 0 || peer < 0 || device >= ND_DEVICES || peer >= ND_DEVICES || device == peer) return 1;
    g_peer.fetch_or(1u << (3 * device + peer));
    return 0;
}
extern "C" void nulldev_stats(unsigned* peer_bits, unsigned long* kind3_copies) {
    *peer_bits = g_peer.load();
    *kind3_copies = g_kind3.load();
}
// failure injection (tests/cpp/nulldev/party_fail.cpp): the n-th copy from
// now on fails, as a faulted device's next call does
static std::atomic<long> g_fail_in{0};
extern "C" void nulldev_fail_nth_memcpy(long n) { g_fail_in.store(n); }
static bool nd_inject() {
    long v = g_fail_in.load();
    while (v > 0 && !g_fail_in.compare_exchange_weak(v, v - 1)) {}
    return v == 1;
}
static char* g_arena = nullptr;
extern "C" size_t nulldev_arena_used();
static std::atomic<size_t>* g_off = nullptr;
static size_t g_cap = 0;
extern "C" int nulldev_shared_arena(size_t bytes) {
    void* p;
    if (const char* name = getenv("ND_ARENA")) {
        // unrelated processes: a named segment mapped at one fixed address in
        // all of them, so that a pointer means the same memory everywhere
        int fd = shm_open(name, O_CREAT | O_RDWR, 0600);
        if (fd < 0 || ftruncate(fd, (off_t)(bytes + 4096)) != 0) return 1;
        p = mmap((void*)0x7e0000000000ull, bytes + 4096, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_FIXED_NOREPLACE, fd, 0);
        close(fd);
        if (p != (void*)0x7e0000000000ull) return 1;
        g_off = reinterpret_cast<std::atomic<size_t>*>(p);  // zero-filled by ftruncate
    } else {
        p = mmap(nullptr, bytes + 4096, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) return 1;
        g_off = new (p) std::atomic<size_t>(0);
    }
    g_arena = (char*)p + 4096;
    g_cap = bytes;
    return 0;
}
// every block carries a 256-byte header (magic, size): the IPC export rule
// of aby3g_ipc_get_handle -- base pointers of whole 2 MiB-granular
// allocations only -- is checked here as on the device
constexpr uint64_t ND_MAGIC = 0x6e646d656d626c6bull;
// arena blocks this process freed, by size: reused by its later allocations
// of the same size (the arena itself only grows)
static std::mutex g_free_mu;
static std::multimap<size_t, char*> g_free_blocks;
extern "C" size_t nulldev_arena_used() { return g_off ? g_off->load() : 0; }
static void* nd_alloc(size_t b) {
    if (!b) b = 1;
    char* h = nullptr;
    if (!g_arena) {
        h = (char*)calloc(1, b + 256);
        if (!h) return nullptr;
    } else {
        {
            std::lock_guard<std::mutex> lk(g_free_mu);
            auto it = g_free_blocks.find(b);
            if (it != g_free_blocks.end()) {
                h = it->second;
                g_free_blocks.erase(it);
            }
        }
        if (!h) {
            const size_t o = g_off->fetch_add((b + 256 + 255) & ~(size_t)255);
            if (o + b + 256 > g_cap) return nullptr;
            h = g_arena + o;
        }
        memset(h, 0, b + 256);
    }
    ((uint64_t*)h)[0] = ND_MAGIC;
    ((uint64_t*)h)[1] = b;
    return h + 256;
}
static void nd_free(void* p) {
    if (!p) return;
    char* h = (char*)p - 256;
    if (g_arena && (char*)p >= g_arena && (char*)p < g_arena + g_cap) {
        std::lock_guard<std::mutex> lk(g_free_mu);
        g_free_blocks.emplace(((uint64_t*)h)[1], h);
        return;
    }
    free(h);
}
static bool nd_ipc_exportable(void* p) {
    const uint64_t* h = (const uint64_t*)((char*)p - 256);
    if (h[0] != ND_MAGIC) {
        fprintf(stderr, "nulldev: IPC export of a pointer that is not an allocation's base\n");
        return false;
    }
    if (h[1] % ((size_t)2 << 20)) {
        fprintf(stderr, "nulldev: IPC export of a %llu-byte allocation (not whole 2 MiB blocks)\n", (unsigned long long)h[1]);
        return false;
    }
    return true;
}
// ---- asynchronous streams (ND_ASYNC=1) ----
// Each stream is a thread that runs its operations in order, some after a
// random delay, so the host runs ahead of its streams as on a GPU: copies,
// memsets, signal-word writes and waits, event records and event waits are
// stream-ordered; host copies (kinds 0 / 1) drain the stream first, as a
// pageable-memory hipMemcpyAsync does. Checks on top of ASan / TSan: a copy
// through an IPC mapping this process has closed aborts, and so does a
// stream wait that never ends (60 s). Compute entry points stay no-ops.
static bool nd_async() {
    static const bool a = [] {
        const char* e = getenv("ND_ASYNC");
        return e && e[0] == '1';
    }();
    return a;
}
[[noreturn]] static void nd_fatal(const char* what) {
    fprintf(stderr, "nulldev: %s\n", what);
    fflush(stderr);
    abort();
}
struct NdStream {
    std::mutex mu;
    std::condition_variable cv, idle;
    std::deque<std::function<void()>> q;
    bool stop = false, busy = false;
    std::thread th;
    explicit NdStream(unsigned seed) {
        if (nd_async()) th = std::thread([this, seed] { run(seed); });
    }
    ~NdStream() {
        if (!th.joinable()) return;
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        th.join();
    }
    void run(unsigned seed) {
        std::minstd_rand rng(seed);
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || !q.empty(); });
                if (q.empty()) return;
                f = std::move(q.front());
                q.pop_front();
                busy = true;
            }
            if (rng() % 4 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 200));
            f();
            {
                std::lock_guard<std::mutex> lk(mu);
                busy = false;
                if (q.empty()) idle.notify_all();
            }
        }
    }
    void enqueue(std::function<void()> f) {
        if (!th.joinable()) {
            f();
            return;
        }
        {
            std::lock_guard<std::mutex> lk(mu);
            q.push_back(std::move(f));
        }
        cv.notify_one();
    }
    void sync() {
        if (!th.joinable()) return;
        std::unique_lock<std::mutex> lk(mu);
        idle.wait(lk, [&] { return q.empty() && !busy; });
    }
};
// live streams; a device-wide sync holds references, so a stream destroyed
// meanwhile by another thread is drained and freed by whoever drops it last
static std::mutex g_streams_mu;
static std::map<NdStream*, std::shared_ptr<NdStream>> g_streams;
static std::atomic<unsigned> g_stream_seed{1};
static void* nd_stream_new() {
    auto s = std::make_shared<NdStream>(g_stream_seed.fetch_add(7919) ^ (unsigned)getpid());
    std::lock_guard<std::mutex> lk(g_streams_mu);
    g_streams.emplace(s.get(), s);
    return s.get();
}
static void nd_stream_delete(void* p) {
    std::shared_ptr<NdStream> s;
    {
        std::lock_guard<std::mutex> lk(g_streams_mu);
        auto it = g_streams.find((NdStream*)p);
        if (it == g_streams.end()) return;
        s = std::move(it->second);
        g_streams.erase(it);
    }
    s->sync();  // (the destructor of the last reference drains and joins)
}
static void nd_stream_sync(void* p) {
    if (p) ((NdStream*)p)->sync();
}
static void nd_sync_all() {
    std::vector<std::shared_ptr<NdStream>> all;
    {
        std::lock_guard<std::mutex> lk(g_streams_mu);
        for (auto& kv : g_streams) all.push_back(kv.second);
    }
    for (auto& s : all) s->sync();
}
template <class F>
static void nd_enqueue(void* stream, F&& f) {
    if (stream)
        ((NdStream*)stream)->enqueue(std::forward<F>(f));
    else
        f();  // the null stream: at once (the library never queues work on it)
}
struct NdEvent {
    std::atomic<uint64_t> rec{0}, done{0};
};
struct NdEventHandle {
    std::shared_ptr<NdEvent> e;  // records still queued keep the event alive
};
static void nd_event_record(void* h, void* stream) {
    std::shared_ptr<NdEvent> e = ((NdEventHandle*)h)->e;
    const uint64_t g = ++e->rec;
    nd_enqueue(stream, [e, g] {
        uint64_t d = e->done.load();
        while (d < g && !e->done.compare_exchange_weak(d, g)) {
        }
    });
}
static bool nd_event_done(void* h) {
    const auto& e = ((NdEventHandle*)h)->e;
    return e->done.load() >= e->rec.load();
}
static void nd_event_sync(void* h) {
    std::shared_ptr<NdEvent> e = ((NdEventHandle*)h)->e;
    const uint64_t g = e->rec.load();
    const auto t0 = std::chrono::steady_clock::now();
    while (e->done.load() < g) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) nd_fatal("an event sync timed out");
        std::this_thread::sleep_for(std::chrono::microseconds(5));
    }
}
static void nd_stream_wait_event(void* stream, void* h) {
    std::shared_ptr<NdEvent> e = ((NdEventHandle*)h)->e;
    const uint64_t g = e->rec.load();  // the event's latest record at the time of the call
    if (!g) return;
    nd_enqueue(stream, [e, g] {
        const auto t0 = std::chrono::steady_clock::now();
        while (e->done.load() < g) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) nd_fatal("a stream wait on an event timed out");
            std::this_thread::sleep_for(std::chrono::microseconds(5));
        }
    });
}
// IPC mappings of this process: a copy through one that was closed is the
// fault a GPU would take
static std::mutex g_maps_mu;
static std::map<const void*, int> g_maps;
static std::set<const void*> g_closed;
static void nd_map_open(const void* p) {
    std::lock_guard<std::mutex> lk(g_maps_mu);
    ++g_maps[p];
    g_closed.erase(p);
}
static void nd_map_close(const void* p) {
    std::lock_guard<std::mutex> lk(g_maps_mu);
    if (--g_maps[p] <= 0) {
        g_maps.erase(p);
        g_closed.insert(p);
    }
}
static bool nd_map_closed(const void* p) {
    std::lock_guard<std::mutex> lk(g_maps_mu);
    return g_closed.count(p) != 0;
}
static int nd_memcpy(void* dst, const void* src, size_t bytes, int kind, void* stream) {
    if (nd_inject()) return 1;
    if (!bytes) return 0;
    if (kind == 3) g_kind3.fetch_add(1);
    if (kind == 0 || kind == 1) {
        // host memory: a pageable hipMemcpyAsync completes before it returns
        nd_stream_sync(stream);
        memmove(dst, src, bytes);
        return 0;
    }
    nd_enqueue(stream, [=] {
        // a copy takes a while, as on the device: the host may act on the
        // mapping (close it, reuse the slot) while it is in flight
        thread_local std::minstd_rand r((unsigned)getpid() * 31u + (unsigned)(uintptr_t)&r);
        std::this_thread::sleep_for(std::chrono::microseconds(r() % 300));
        if (nd_map_closed(src) || nd_map_closed(dst)) nd_fatal("a copy through a closed IPC mapping");
        memmove(dst, src, bytes);
    });
    return 0;
}
static int nd_wait(uint64_t* w, uint64_t v) {
    const auto t0 = std::chrono::steady_clock::now();
    while (__atomic_load_n(w, __ATOMIC_ACQUIRE) < v) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) return 1;
        std::this_thread::sleep_for(std::chrono::microseconds(5));
    }
    return 0;
}
"""


def main():
    text = open(HDR).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    out = ['// generated by gen_nulldev.py -- host-memory stand-in for ASan runs of the host runtime',
           "#include <aby3gpu.h>", "#include <cstdlib>", "#include <cstring>", PREAMBLE, 'extern "C" {']
    for m in re.finditer(r"(const char\*|int|size_t|uint64_t)\s+(aby3g_\w+)\s*\(([^;]*?)\)\s*;", text, flags=re.S):
        ret, name, args = m.group(1), m.group(2), " ".join(m.group(3).split())
        body = OVERRIDES.get(name, "return 0;")
        out.append(f"{ret} {name}({args}) {{ {body} }}")
    out.append("}")
    dst = sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "nulldev.cpp")
    open(dst, "w").write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
