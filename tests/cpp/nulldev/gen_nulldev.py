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
    "aby3g_free": "g_blocking.fetch_add(1); nd_free(ptr); return 0;",
    "aby3g_device_sync": "g_blocking.fetch_add(1); return 0;",
    "aby3g_host_malloc": "*ptr = calloc(1, bytes ? bytes : 1); return *ptr ? 0 : 1;",
    "aby3g_host_free": "free(ptr); return 0;",
    "aby3g_memcpy": "if (nd_inject()) return 1; if (kind == 3) g_kind3.fetch_add(1); if (bytes) memmove(dst, src, bytes); return 0;",
    "aby3g_memset": "if (bytes) memset(dst, value, bytes); return 0;",
    "aby3g_stream_create": "*stream = new int(0); return 0;",
    "aby3g_stream_destroy": "delete (int*)stream; return 0;",
    "aby3g_event_create": "*ev = new int(0); return 0;",
    "aby3g_event_create_timed": "*ev = new int(0); return 0;",
    "aby3g_event_destroy": "delete (int*)ev; return 0;",
    "aby3g_event_record": "*(int*)ev = 1; return 0;",
    "aby3g_event_elapsed_ms": "*ms = 0; return 0;",
    "aby3g_event_query": "*done = 1; return 0;",
    "aby3g_signal_alloc": "g_blocking.fetch_add(1); *word = (uint64_t*)nd_alloc(8); return *word ? 0 : 1;",
    "aby3g_stream_write_value": "__atomic_store_n(word, value, __ATOMIC_RELEASE); return 0;",
    "aby3g_stream_wait_value": "return nd_wait(word, value);",
    "aby3g_ipc_get_handle": "if (!nd_ipc_exportable(ptr)) return 1; memset(handle, 0, sizeof *handle); memcpy(handle->bytes, &ptr, sizeof ptr); return 0;",
    "aby3g_ipc_open": "memcpy(ptr, handle->bytes, sizeof *ptr); return 0;",
    "aby3g_host_register": "*dev = host; return 0;",
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
#include <cstdio>
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
static void* nd_alloc(size_t b) {
    if (!b) b = 1;
    char* h;
    if (!g_arena) {
        h = (char*)calloc(1, b + 256);
        if (!h) return nullptr;
    } else {
        const size_t o = g_off->fetch_add((b + 256 + 255) & ~(size_t)255);
        if (o + b + 256 > g_cap) return nullptr;
        h = g_arena + o;
        memset(h, 0, b + 256);
    }
    ((uint64_t*)h)[0] = ND_MAGIC;
    ((uint64_t*)h)[1] = b;
    return h + 256;
}
static void nd_free(void* p) {
    if (!p) return;
    if (g_arena && (char*)p >= g_arena && (char*)p < g_arena + g_cap) return;
    free((char*)p - 256);
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
