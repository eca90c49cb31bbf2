#include "Channel.h"
#include "Link.h"
#include <cstdio>
#include <cstring>
#include <chrono>
#include <cstdlib>
#include <atomic>
#include <deque>
#include <map>
#include <thread>

namespace aby3 {

namespace {
struct Slot {
    void* ptr = nullptr;
    size_t cap = 0;
    int device = -1;
    std::unique_ptr<Event> ready;     // recorded on the sender's stream
    std::unique_ptr<Event> consumed;  // recorded on the receiver's stream
    bool busy = false;
    bool consumedRecorded = false;
};
struct Msg {
    bool device = false;
    std::vector<u8> host;
    Slot* slot = nullptr;
    size_t bytes = 0;
    std::shared_ptr<DeviceBuffer> shared;  // zero-copy payload
    std::shared_ptr<Event> ready;          // recorded on the sender's stream
    // or, between parties on one device: the sender's stream writes sigValue
    // to *sigWord when the payload is ready (cheaper than an event hand-off)
    u64* sigWord = nullptr;
    u64 sigValue = 0;
    // or published chunk by chunk by the producing kernel (in-kernel hand-off)
    u64* hsFlags = nullptr;
    u64 hsSeq = 0;
    // from another process (LinkEnd): the payload sits in the sender's
    // staging slot `lslot` (generation lgen, IPC handle lh) once the link's
    // ready word reaches lseq
    bool link = false;
    u32 lslot = 0;
    u64 lgen = 0, lseq = 0;
    int ldevice = -1;
    aby3g_ipc_handle lh{};
    // or, from another process on this GPU, in the sender's arena at larena
    // offset, published in-kernel with sequence number lseq
    bool linkInKernel = false;
    u64 larena = 0;
    // or, from another process on this GPU, in the sender's arena at larena,
    // ready once the link's ready word reaches lseq (stream hand-off, no copy)
    bool linkArena = false;
};

// a message descriptor on a link's ring (host payloads follow it)
struct WireMsg {
    u64 bytes;
    u32 kind;  // 0 host payload, 1 device payload (staged), 2 in-kernel (arena), 3 arena announce,
               // 4 device identity (the sender's device UUID in handle.bytes[0..15]),
               // 5 arena payload behind the ready word (stream hand-off, read in place)
    u32 slot;
    u64 gen, seq;  // kind 2: gen = offset in the arena's slots; kind 3: gen = slot bytes
    i64 device;    // the sender's device
    aby3g_ipc_handle handle;
};

// In-kernel hand-offs between processes sharing one GPU: the sender's arena
// per direction, [kHandoffChunks flags][2 slots], exported once through IPC
// at setup (zeroed before its handle leaves). Each evaluation takes the next
// slot for all its levels' messages (evalSendBuffer), the level kernels write
// their AND shares there write-through and publish per-chunk flags, and the
// receiver's level kernels poll the flags and read the shares in place from
// their mapping. A slot is rewritten two evaluations later: by then the
// receiver has finished reading it (the ring of three: a party completes
// evaluation e+1 only with its previous party's e+1 messages, which need the
// receiver's e+1 messages, which its kernels produce after its kernels that
// read evaluation e completed).
constexpr u64 kArenaFlagBytes = 4096;  // kHandoffChunks flags
constexpr u32 kNoSlot = ~0u;

// a sender's staging slot of a link (device memory exported through IPC)
struct LinkSlot {
    void* ptr = nullptr;
    size_t cap = 0;
    u64 gen = 0, lastSeq = 0;
    aby3g_ipc_handle h{};
    bool reserved = false;  // handed to a producer (linkReserve), its message not sent yet
};
}  // namespace

// in-kernel hand-offs: messages of at most kHandoffMaxChunks chunks (128 Ki
// rows), or of at most kHandoffChunks chunks (1 Mi rows) from a light
// producer -- and only within the device's residency rule
// (handoffResidencyOk: with the hand-off level kernel at 74 VGPRs, 6
// workgroups of the large form per CU, two 512-chunk consumers hold 172 of
// 256 CUs on MI355X).
constexpr u64 kHandoffMaxChunks = 64;
constexpr u64 kHandoffChunks = 512;  // flags per direction
// A producing launch of at most this many HBM bytes is light: its consumer's
// workgroups spin only briefly. On C3 / C5 (2^20 / 2^19 rows, 512 / 256
// chunks) in one A/B (scripts/gpu_ab_env.sh): stream hand-offs for every
// large message 0.386-0.399 ms / 80.3-80.8 ms; in-kernel from producers of
// <= 2 MiB the same; <= 8 MiB 0.376-0.382 / 75.6-76.6; <= 32 MiB
// 0.363-0.368 / 72.1-73.6; every level in-kernel 0.376-0.384 / 75.7-75.9.
// The bound is also a safety margin: with the 16-byte level kernels (round
// 5) every level in-kernel ended a 300-step C3 run with 55 hand-off
// timeouts, the three parties' heavy first levels and their consumers
// holding the device; <= 64 MiB measured 2-3 % faster in one sample and is
// not taken without a safety argument that covers heavy producers.
constexpr u64 kHandoffLightBytes = (u64)32 << 20;

// how long a receive polls before it sleeps on the condition variable
constexpr int kSpinUs = 500;
thread_local double t_recvWaitUs = 0;

struct Pipe {
    std::mutex mu;
    std::condition_variable cv;
    std::map<u64, Msg> msgs;
    u64 sendSeq = 0, recvTicket = 0;
    std::vector<std::unique_ptr<Slot>> slots;
    u64 sent = 0, received = 0;
    // sender and receiver on this device (-1: unknown / different): device
    // payloads are then signalled through a stream-ordered word
    int signalDevice = -1;
    // allocated and zeroed when the ring is built (makeLocalRing), never
    // mid-run: zeroing needs a device-wide wait, and a party host blocked in
    // one cannot enqueue the producer another party's waiting kernel needs
    // (the round-4 hand-off timeouts)
    u64* word = nullptr;
    u64 devSeq = 0;       // device payloads signalled so far (sender thread only)
    // in-kernel hand-offs (Channel::handoffPost): one flag per chunk of
    // ABY3G_HANDOFF_ROWS rows, reused by every message with increasing seq
    bool kernelHandoff = false;
    u64* hsFlags = nullptr;  // kHandoffChunks flags, zeroed on the sender's stream at its first message
    u64 hsCap = 0, hsSeq = 0;

    // cross-process direction: this process holds one end of it
    std::unique_ptr<LinkEnd> link;
    int linkDevice = -1;                      // this end's device
    std::vector<LinkSlot> lslots;             // sender: staging slots
    struct Retired {
        void* ptr;
        u32 slot;
        u64 lastSeq;
    };
    // sender: outgrown slot buffers, freed at teardown once their last
    // copy-out finished (not before: aby3g_free may synchronize the device,
    // and a party's stream can hold a wait on a peer whose next message this
    // host has yet to send -- a free mid-protocol could deadlock; slots are
    // outgrown rarely, so few pile up)
    std::vector<Retired> retired;
    std::map<std::pair<u32, u64>, void*> mapped;  // receiver: opened slots by (slot, gen)
    struct Closing {
        void* ptr;
        std::unique_ptr<Event> done;
    };
    std::vector<Closing> closing;  // receiver: openings of replaced slot buffers, closed once `done`
    u64 linkRead = 0;                         // receiver: messages taken off the ring
    // the arena (sender: own allocation; receiver: its IPC mapping)
    void* arena = nullptr;
    u64 arenaSlot = 0;   // bytes per evaluation slot
    u64 arenaNext = 0;   // sender: slots handed out
    int arenaOpen = 0;   // sender: an evaluation holds a slot (evalSendBuffer's lease alive)
    bool arenaMapped = false;
    u64* arenaFlags() const { return (u64*)arena; }
    u8* arenaSlots() const { return (u8*)arena + kArenaFlagBytes; }
    // sender: the ring is written by a thread of its own, in the order the
    // messages were sent, so a send never blocks on the peer's reads: a host
    // payload larger than the ring (4 MiB) then streams through it while the
    // sending party goes on, as with in-process pipes -- a cyclic exchange
    // where every party sends more than the ring holds before it receives
    // would otherwise wait on itself until the link timeout
    std::thread writer;
    std::mutex wmu;
    std::condition_variable wcv;
    std::deque<std::vector<u8>> wq;
    bool wstop = false;
    std::string werr;

    void ringWrite(std::vector<u8>&& bytes) {
        std::lock_guard<std::mutex> lk(wmu);
        if (!werr.empty()) throw std::runtime_error("link writer: " + werr);
        wq.push_back(std::move(bytes));
        if (!writer.joinable()) writer = std::thread([this] { writerLoop(); });
        wcv.notify_one();
    }
    void writerLoop() {
        for (;;) {
            std::vector<u8> b;
            {
                std::unique_lock<std::mutex> lk(wmu);
                wcv.wait(lk, [&] { return wstop || !wq.empty(); });
                if (wq.empty()) return;  // stopped and drained
                b = std::move(wq.front());
                wq.pop_front();
            }
            try {
                if (!b.empty()) link->write(b.data(), b.size());
            } catch (const std::exception& e) {
                std::lock_guard<std::mutex> lk(wmu);
                werr = e.what();
                wq.clear();
                return;
            }
        }
    }
    // drains the queue (each write bounded by the link timeout) and joins
    void stopWriter() {
        {
            std::lock_guard<std::mutex> lk(wmu);
            wstop = true;
        }
        wcv.notify_one();
        if (writer.joinable()) writer.join();
    }

    // readiness of a device payload enqueued so far on `gpu`'s stream
    void signalReady(Msg& m, Gpu& gpu, Event* fallback, bool useWord = true) {
        if (useWord && signalDevice >= 0 && signalDevice == gpu.device()) {
            if (!word) throw std::runtime_error("channel: signal word not allocated at ring construction");
            m.sigWord = word;
            m.sigValue = ++devSeq;
            GPU_CALL(aby3g_stream_write_value(gpu.stream(), word, m.sigValue));
        } else {
            fallback->record(gpu.stream());
        }
    }

    ~Pipe() {
        stopWriter();
        if (link && getenv("ABY3_LINK_STATS")) {
            u64 gens = 0;
            for (const LinkSlot& ls : lslots) gens += ls.gen;
            std::fprintf(stderr, "link %s: %zu slots (%llu buffers made), %zu retired, %zu openings, %llu msgs sent\n",
                         link->sender() ? "out" : "in", lslots.size(), (unsigned long long)gens, retired.size(),
                         mapped.size(), (unsigned long long)devSeq);
        }
        if (link) {
            aby3g_set_device(linkDevice);
            aby3g_device_sync();
            for (auto& m : mapped) aby3g_ipc_close(m.second);
            for (auto& c : closing) aby3g_ipc_close(c.ptr);
            closing.clear();
            if (arena) {
                if (arenaMapped)
                    aby3g_ipc_close(arena);
                else
                    aby3g_free(arena);  // the receiver's mapping keeps it alive until it closes
                arena = nullptr;
            }
            // the peer process may still be copying out of a staging slot:
            // free each buffer once its last message is consumed -- within 10 s
            // in all (a live peer takes milliseconds; one that died, or a
            // session torn down after an error, leaves nothing to wait for)
            const auto t0 = std::chrono::steady_clock::now();
            auto left = [&] {
                return std::max(0.0, 10.0 - std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
            };
            for (size_t i = 0; i < lslots.size(); ++i)
                if (lslots[i].ptr) {
                    if (lslots[i].lastSeq) link->waitConsumed((u32)i, lslots[i].lastSeq, left());
                    aby3g_free(lslots[i].ptr);
                }
            for (auto& r : retired) {
                link->waitConsumed(r.slot, r.lastSeq, left());
                aby3g_free(r.ptr);
            }
        }
        for (auto& s : slots)
            if (s->ptr) {
                aby3g_set_device(s->device);
                aby3g_device_sync();
                aby3g_free(s->ptr);
            }
        if (word || hsFlags) {
            aby3g_set_device(signalDevice);
            aby3g_device_sync();
            if (word) aby3g_free(word);
            if (hsFlags) aby3g_free(hsFlags);
        }
    }

    std::atomic<u64> published{0};  // messages pushed so far (sendSeq, readable without the lock)

    void push(Msg&& m) {
        if (link) {
            linkPush(std::move(m));
            return;
        }
        std::lock_guard<std::mutex> lk(mu);
        sent += m.bytes;
        msgs.emplace(sendSeq++, std::move(m));
        published.store(sendSeq, std::memory_order_release);
        cv.notify_all();
    }
    Msg pop(u64 ticket) {
        // The parties' threads hand messages to each other every protocol
        // round; a condition-variable sleep costs a futex wake-up (tens of us)
        // per round, so poll for a while first.
        const auto t0 = std::chrono::steady_clock::now();
        struct WaitClock {
            std::chrono::steady_clock::time_point t0;
            ~WaitClock() { t_recvWaitUs += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count(); }
        } clock{t0};
        if (link) {
            std::lock_guard<std::mutex> lk(mu);
            while (!msgs.count(ticket)) linkTake();
            Msg m = std::move(msgs[ticket]);
            msgs.erase(ticket);
            received += m.bytes;
            return m;
        }
        while (published.load(std::memory_order_acquire) <= ticket &&
               std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(kSpinUs)) {
            for (int i = 0; i < 64; ++i) __builtin_ia32_pause();
        }
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return msgs.count(ticket) != 0; });
        Msg m = std::move(msgs[ticket]);
        msgs.erase(ticket);
        received += m.bytes;
        return m;
    }
    Slot* acquire(size_t bytes, int device) {
        std::lock_guard<std::mutex> lk(mu);
        for (auto& s : slots)
            if (!s->busy && s->cap >= bytes && s->device == device) {
                s->busy = true;
                return s.get();
            }
        auto s = std::make_unique<Slot>();
        s->cap = bytes < 4096 ? 4096 : bytes;
        s->device = device;
        GPU_CALL(aby3g_malloc(&s->ptr, s->cap));
        s->ready = std::make_unique<Event>();
        s->busy = true;
        slots.push_back(std::move(s));
        return slots.back().get();
    }
    void releaseSlot(Slot* s) {
        std::lock_guard<std::mutex> lk(mu);
        s->busy = false;
    }

    // ---- cross-process ends ----
    // sender: host payloads go onto the ring; device payloads are copied into
    // a staging slot whose previous message the receiver has already taken
    // (its copy-out enqueued), the stream waiting for that copy-out to finish.
    void linkPush(Msg&& m) {
        std::lock_guard<std::mutex> lk(mu);
        WireMsg w{};
        w.bytes = m.bytes;
        w.kind = 0;
        w.slot = kNoSlot;
        w.device = linkDevice;
        sent += m.bytes;
        ringWrite(std::vector<u8>((const u8*)&w, (const u8*)&w + sizeof w));
        if (m.bytes) {
            m.host.resize(m.bytes);
            ringWrite(std::move(m.host));
        }
    }
    // sender (mu held): a staging slot of at least `bytes` that the receiver
    // has released -- its previous message's copy-out enqueued (host mark),
    // and this stream made to wait for that copy-out to finish
    u32 pickSlot(size_t bytes, Gpu& gpu) {
        int k = -1;
        auto free = [&](size_t i) {
            return !lslots[i].reserved && link->posted((u32)i).load(std::memory_order_acquire) >= lslots[i].lastSeq;
        };
        u64 staged = 0;
        for (const LinkSlot& ls : lslots) staged += ls.cap;
        for (size_t i = 0; i < lslots.size() && k < 0; ++i)
            if (lslots[i].cap >= bytes && free(i)) k = (int)i;
        if (k < 0 && (lslots.size() >= LinkEnd::kMaxSlots || staged + bytes > LinkEnd::kMaxStagedBytes) &&
            !lslots.empty()) {
            // every slot holds a message the receiver has not taken yet and
            // no more may be added: wait (up to the link timeout) until it
            // takes the oldest one -- messages are taken in order, so a
            // sender that runs ahead (party 2 of a truncating asyncMul only
            // sends) is throttled instead of failing
            size_t oldest = lslots.size();
            for (size_t i = 0; i < lslots.size(); ++i)
                if (!lslots[i].reserved && (oldest == lslots.size() || lslots[i].lastSeq < lslots[oldest].lastSeq))
                    oldest = i;
            if (oldest == lslots.size()) throw std::runtime_error("link: every staging slot is reserved");
            link->waitPosted((u32)oldest, lslots[oldest].lastSeq);
        }
        for (size_t i = 0; i < lslots.size() && k < 0; ++i)
            if (lslots[i].cap >= bytes && free(i)) k = (int)i;
        for (size_t i = 0; i < lslots.size() && k < 0; ++i)
            if (free(i)) {
                // free but too small: replace it (the receiver may still be
                // reading the old buffer on its stream: retire, don't free)
                k = (int)i;
                retired.push_back(Retired{lslots[i].ptr, (u32)i, lslots[i].lastSeq});
                lslots[i].ptr = nullptr;
            }
        if (k < 0) {
            lslots.emplace_back();
            k = (int)lslots.size() - 1;
        }
        LinkSlot& sl = lslots[(size_t)k];
        if (!sl.ptr) {
            // capacities are powers of two from 2 MiB (whole blocks: the
            // IPC export rule, aby3g_ipc_get_handle): a slot is outgrown at
            // most log2(largest message / 2 MiB) times, so the retired
            // buffers behind it (kept until teardown) add up to less than
            // its current capacity, whatever the sequence of message sizes
            size_t cap = ipcBytes(1);
            while (cap < bytes) cap <<= 1;
            sl.cap = cap;
            GPU_CALL(aby3g_malloc(&sl.ptr, sl.cap));
            GPU_CALL(aby3g_ipc_get_handle(sl.ptr, &sl.h));
            ++sl.gen;
        } else if (sl.lastSeq) {
            // the receiver's copy-out of the slot's previous message
            GPU_CALL(aby3g_stream_wait_value(gpu.stream(), link->consumedDev((u32)k), sl.lastSeq));
        }
        return (u32)k;
    }
    // sender: a staging slot for a producer to write its message into
    // directly (Channel::linkSendBuffer); the send then skips the copy
    void* linkReserve(size_t bytes, Gpu& gpu) {
        std::lock_guard<std::mutex> lk(mu);
        const u32 k = pickSlot(std::max<size_t>(bytes, 8), gpu);
        lslots[k].reserved = true;
        return lslots[k].ptr;
    }
    void linkSendDevice(const void* src, size_t bytes, Gpu& gpu) {
        std::lock_guard<std::mutex> lk(mu);
        WireMsg w{};
        w.bytes = bytes;
        w.kind = 1;
        w.slot = kNoSlot;
        w.device = gpu.device();
        int k = -1;
        for (size_t i = 0; i < lslots.size() && k < 0; ++i)
            if (lslots[i].reserved && lslots[i].ptr == src) k = (int)i;
        if (k >= 0) {
            // produced in place (linkReserve): no copy
            if (bytes > lslots[(size_t)k].cap) throw std::runtime_error("link: message larger than its reserved slot");
            lslots[(size_t)k].reserved = false;
            if (!bytes) k = -1;
        } else if (bytes) {
            k = (int)pickSlot(bytes, gpu);
            GPU_CALL(aby3g_memcpy(lslots[(size_t)k].ptr, src, bytes, 2, gpu.stream()));
        }
        if (k >= 0) {
            LinkSlot& sl = lslots[(size_t)k];
            sl.lastSeq = ++devSeq;
            GPU_CALL(aby3g_stream_write_value(gpu.stream(), link->readyDev(), sl.lastSeq));
            w.slot = (u32)k;
            w.gen = sl.gen;
            w.seq = sl.lastSeq;
            w.handle = sl.h;
        }
        sent += bytes;
        ringWrite(std::vector<u8>((const u8*)&w, (const u8*)&w + sizeof w));
    }
    // sender: a payload already in this direction's arena (the binary
    // engine's evaluation slot, evalSendBuffer) goes by reference: the stream
    // writes the ready word behind the producing kernel and the receiver's
    // stream waits for it, then its kernels read the arena in place -- no
    // staging copies. The slot is rewritten two evaluations later, after the
    // receiver has read it (the rule of evalSendBuffer).
    bool linkSendArena(const void* src, size_t bytes, Gpu& gpu) {
        const u8* q = (const u8*)src;
        if (!arena || arenaMapped || !q || q < arenaSlots() || q + bytes > arenaSlots() + 2 * arenaSlot) return false;
        std::lock_guard<std::mutex> lk(mu);
        WireMsg w{};
        w.bytes = bytes;
        w.kind = 5;
        w.slot = kNoSlot;
        w.gen = (u64)(q - arenaSlots());
        w.seq = ++devSeq;
        w.device = gpu.device();
        GPU_CALL(aby3g_stream_write_value(gpu.stream(), link->readyDev(), w.seq));
        sent += bytes;
        ringWrite(std::vector<u8>((const u8*)&w, (const u8*)&w + sizeof w));
        return true;
    }
    // receiver: the next message off the ring, filed under its ticket
    void linkTake() {
        WireMsg w;
        link->read(&w, sizeof w);
        Msg m;
        m.bytes = w.bytes;
        if (w.kind == 0) {
            m.host.resize(w.bytes);
            if (w.bytes) link->read(m.host.data(), w.bytes);
        } else if (w.kind == 2) {
            m.device = true;
            m.link = true;
            m.linkInKernel = true;
            m.larena = w.gen;
            m.lseq = w.seq;
            m.ldevice = (int)w.device;
        } else if (w.kind == 5) {
            m.device = true;
            m.link = true;
            m.linkArena = true;
            m.larena = w.gen;
            m.lseq = w.seq;
            m.ldevice = (int)w.device;
        } else if (w.kind == 3) {
            throw std::runtime_error("link: an arena announce after setup");
        } else {
            m.device = true;
            m.link = true;
            m.lslot = w.slot;
            m.lgen = w.gen;
            m.lseq = w.seq;
            m.ldevice = (int)w.device;
            m.lh = w.handle;
        }
        msgs.emplace(linkRead++, std::move(m));
    }
    // receiver: enqueue the copy of a linked device payload into dst
    void linkCopyOut(const Msg& m, void* dst, Gpu& g) {
        if (!m.bytes) return;
        void* src;
        {
            std::lock_guard<std::mutex> lk(mu);
            auto key = std::make_pair(m.lslot, m.lgen);
            auto it = mapped.find(key);
            if (it == mapped.end()) {
                // a new buffer behind this slot: close the openings of its
                // older ones once this stream's copy-outs from them finished
                // (slots are outgrown rarely; the sync is off the common path)
                for (auto o = mapped.begin(); o != mapped.end();)
                    if (o->first.first == m.lslot && o->first.second < m.lgen) {
                        // every copy-out from it is already on this stream:
                        // close it once an event recorded now has completed
                        // (never a blocking sync here: the stream can hold a
                        // wait on a peer that needs this host's next send)
                        auto ev = std::make_unique<Event>();
                        ev->record(g.stream());
                        closing.push_back(Closing{o->second, std::move(ev)});
                        o = mapped.erase(o);
                    } else {
                        ++o;
                    }
                void* p = nullptr;
                GPU_CALL(aby3g_ipc_open(&m.lh, &p));
                it = mapped.emplace(key, p).first;
            }
            src = it->second;
            for (size_t i = 0; i < closing.size();)
                if (closing[i].done->done()) {
                    GPU_CALL(aby3g_ipc_close(closing[i].ptr));
                    closing[i] = std::move(closing.back());
                    closing.pop_back();
                } else {
                    ++i;
                }
        }
        GPU_CALL(aby3g_stream_wait_value(g.stream(), link->readyDev(), m.lseq));
        GPU_CALL(aby3g_memcpy(dst, src, m.bytes, m.ldevice == g.device() ? 2 : 3, g.stream()));
        GPU_CALL(aby3g_stream_write_value(g.stream(), link->consumedDev(m.lslot), m.lseq));
        link->posted(m.lslot).store(m.lseq, std::memory_order_release);
    }
};

struct RecvFuture::State {
    std::shared_ptr<Pipe> pipe;
    u64 ticket = 0;
    void* dst = nullptr;
    size_t bytes = 0;
    Gpu* gpu = nullptr;  // null: host payload
    bool shared = false;
    std::shared_ptr<DeviceBuffer> out;
    bool done = false;
    std::mutex mu;
    // set by getSharedHandoff for the duration of its getShared
    std::mutex hsMu;
    aby3g_handoff* handoff = nullptr;
};

void RecvFuture::get() const {
    if (!mState) throw std::runtime_error("RecvFuture::get on an empty future");
    if (mState->shared) {
        getShared();
        return;
    }
    State& st = *mState;
    std::lock_guard<std::mutex> lk(st.mu);
    if (st.done) return;
    Msg m = st.pipe->pop(st.ticket);
    if (m.shared || m.linkArena || m.linkInKernel)
        throw std::runtime_error("channel: zero-copy payload received by a copying receive");
    if (m.bytes != st.bytes)
        throw std::runtime_error("channel: message size mismatch (expected " + std::to_string(st.bytes) + ", got " +
                                 std::to_string(m.bytes) + ")");
    if (!st.gpu) {
        if (m.device) throw std::runtime_error("channel: device payload received into a host buffer");
        if (st.bytes) std::memcpy(st.dst, m.host.data(), st.bytes);
    } else {
        if (!m.device) throw std::runtime_error("channel: host payload received into a device buffer");
        Gpu& g = *st.gpu;
        GPU_CALL(aby3g_set_device(g.device()));
        if (m.link) {
            st.pipe->linkCopyOut(m, st.dst, g);
            st.done = true;
            return;
        }
        Slot* s = m.slot;
        if (st.bytes) {
            if (m.sigWord)
                GPU_CALL(aby3g_stream_wait_value(g.stream(), m.sigWord, m.sigValue));
            else
                GPU_CALL(aby3g_stream_wait_event(g.stream(), s->ready->get()));
            // same device: copy kernel; across devices: the runtime's peer copy
            GPU_CALL(aby3g_memcpy(st.dst, s->ptr, st.bytes, s->device == g.device() ? 2 : 3, g.stream()));
        }
        if (!s->consumed) s->consumed = std::make_unique<Event>();
        s->consumed->record(g.stream());
        s->consumedRecorded = true;
        st.pipe->releaseSlot(s);
    }
    st.done = true;
}

std::shared_ptr<DeviceBuffer> RecvFuture::getSharedHandoff(aby3g_handoff& wait) const {
    if (!mState || !mState->shared) throw std::runtime_error("RecvFuture::getSharedHandoff on a non-shared receive");
    wait = aby3g_handoff{nullptr, 0, nullptr};
    std::lock_guard<std::mutex> lk(mState->hsMu);
    mState->handoff = &wait;
    auto out = getShared();
    mState->handoff = nullptr;
    return out;
}

std::shared_ptr<DeviceBuffer> RecvFuture::getShared() const {
    if (!mState || !mState->shared) throw std::runtime_error("RecvFuture::getShared on a non-shared receive");
    State& st = *mState;
    std::lock_guard<std::mutex> lk(st.mu);
    if (st.done) return st.out;
    Msg m = st.pipe->pop(st.ticket);
    if (m.link && m.linkInKernel) {
        // from another process on this GPU, handed over in-kernel: read in
        // place from the sender's arena (this process's mapping)
        if (m.bytes != st.bytes)
            throw std::runtime_error("channel: message size mismatch (expected " + std::to_string(st.bytes) +
                                     ", got " + std::to_string(m.bytes) + ")");
        if (!st.handoff)
            throw std::runtime_error("channel: a message published in-kernel must be received by a waiting kernel "
                                     "(RecvFuture::getSharedHandoff)");
        Pipe& p = *st.pipe;
        if (!p.arena || m.larena + m.bytes > 2 * p.arenaSlot)
            throw std::runtime_error("channel: in-kernel message outside the sender's arena");
        st.out = DeviceBuffer::borrow(p.arenaSlots() + m.larena, std::max<size_t>(m.bytes, 8), st.gpu);
        st.handoff->flags = p.arenaFlags();
        st.handoff->seq = m.lseq;
        st.handoff->wait_ticks = st.gpu->waitTicks();
        st.done = true;
        return st.out;
    }
    if (m.link && m.linkArena) {
        // from another process on this GPU, by reference into the sender's
        // arena: wait for the ready word, read in place (this mapping)
        if (m.bytes != st.bytes)
            throw std::runtime_error("channel: message size mismatch (expected " + std::to_string(st.bytes) +
                                     ", got " + std::to_string(m.bytes) + ")");
        Pipe& p = *st.pipe;
        if (!p.arena || m.larena + m.bytes > 2 * p.arenaSlot)
            throw std::runtime_error("channel: arena message outside the sender's arena");
        GPU_CALL(aby3g_set_device(st.gpu->device()));
        GPU_CALL(aby3g_stream_wait_value(st.gpu->stream(), p.link->readyDev(), m.lseq));
        st.out = DeviceBuffer::borrow(p.arenaSlots() + m.larena, std::max<size_t>(m.bytes, 8), st.gpu);
        st.done = true;
        return st.out;
    }
    if (m.link) {
        // from another process: the payload is copied out of the sender's
        // staging slot into a buffer of this party
        if (m.bytes != st.bytes)
            throw std::runtime_error("channel: message size mismatch (expected " + std::to_string(st.bytes) +
                                     ", got " + std::to_string(m.bytes) + ")");
        GPU_CALL(aby3g_set_device(st.gpu->device()));
        st.out = std::make_shared<DeviceBuffer>(*st.gpu, std::max<size_t>(m.bytes, 8));
        st.pipe->linkCopyOut(m, st.out->data(), *st.gpu);
        st.done = true;
        return st.out;
    }
    if (!m.shared) throw std::runtime_error("channel: expected a zero-copy device payload");
    if (m.bytes != st.bytes)
        throw std::runtime_error("channel: message size mismatch (expected " + std::to_string(st.bytes) + ", got " +
                                 std::to_string(m.bytes) + ")");
    GPU_CALL(aby3g_set_device(st.gpu->device()));
    if (m.hsFlags) {
        if (!st.handoff)
            throw std::runtime_error("channel: a message published in-kernel must be received by a waiting kernel "
                                     "(RecvFuture::getSharedHandoff)");
        st.handoff->flags = m.hsFlags;
        st.handoff->seq = m.hsSeq;
        st.handoff->wait_ticks = st.gpu->waitTicks();
    } else if (m.sigWord)
        GPU_CALL(aby3g_stream_wait_value(st.gpu->stream(), m.sigWord, m.sigValue));
    else
        GPU_CALL(aby3g_stream_wait_event(st.gpu->stream(), m.ready->get()));
    st.out = std::move(m.shared);
    st.done = true;
    return st.out;
}

void Channel::sendShared(std::shared_ptr<DeviceBuffer> buf, size_t bytes, Gpu& gpu, bool word) {
    if (!mOut) throw std::runtime_error("channel not connected");
    if (!buf || buf->bytes() < bytes) throw std::runtime_error("asyncSendShared: buffer smaller than the message");
    GPU_CALL(aby3g_set_device(gpu.device()));
    if (mOut->link) {
        // another process reads an arena payload in place; anything else is
        // staged (a copy into an IPC-exported slot)
        if (!mOut->linkSendArena(buf->data(), bytes, gpu)) mOut->linkSendDevice(buf->data(), bytes, gpu);
        return;
    }
    Msg m;
    m.device = true;
    m.bytes = bytes;
    m.shared = std::move(buf);
    if (!word || mOut->signalDevice != gpu.device()) m.ready = std::make_shared<Event>();
    mOut->signalReady(m, gpu, m.ready.get(), word);
    mOut->push(std::move(m));
}

void Channel::asyncSendShared(std::shared_ptr<DeviceBuffer> buf, size_t bytes, Gpu& gpu) {
    sendShared(std::move(buf), bytes, gpu, true);
}

void Channel::asyncSendSharedEvent(std::shared_ptr<DeviceBuffer> buf, size_t bytes, Gpu& gpu) {
    sendShared(std::move(buf), bytes, gpu, false);
}

aby3g_handoff Channel::handoffPost(Gpu& gpu, u64 rows, u64 producerBytes, const void* payload) {
    if (!mOut) throw std::runtime_error("channel not connected");
    Pipe& p = *mOut;
    if (p.link) {
        // between processes on one GPU: only a payload in this direction's arena
        const u8* q = (const u8*)payload;
        if (!p.arena || kernelsSerialized() || !q || q < p.arenaSlots() || q >= p.arenaSlots() + 2 * p.arenaSlot)
            return aby3g_handoff{nullptr, 0, nullptr};
        const u64 chunks = std::max<u64>(1, (rows + ABY3G_HANDOFF_ROWS - 1) / ABY3G_HANDOFF_ROWS);
        // three processes on the device: each brings its own queues' stream-op waits
        if (!handoffResidencyOk(handoffResidency(gpu.device()), chunks, 3) || chunks > kHandoffChunks ||
            (chunks > kHandoffMaxChunks && producerBytes > kHandoffLightBytes))
            return aby3g_handoff{nullptr, 0, nullptr};
        return aby3g_handoff{p.arenaFlags(), ++p.hsSeq, nullptr};
    }
    if (!p.kernelHandoff || p.signalDevice != gpu.device() || kernelsSerialized())
        return aby3g_handoff{nullptr, 0, nullptr};
    if (!p.hsFlags) {
        // First message of this direction: the flags are zeroed on the
        // sender's stream and this message still goes by a stream hand-off,
        // whose wait orders every later in-kernel poll of the receiver after
        // the zeroing (no null-stream memset or device sync, which would take
        // a hardware queue of the process or wait on a polling kernel).
        void* f = nullptr;
        GPU_CALL(aby3g_set_device(gpu.device()));
        GPU_CALL(aby3g_malloc(&f, kHandoffChunks * 8));
        GPU_CALL(aby3g_memset(f, 0, kHandoffChunks * 8, gpu.stream()));
        p.hsFlags = (u64*)f;
        p.hsCap = kHandoffChunks;
        return aby3g_handoff{nullptr, 0, nullptr};
    }
    const u64 chunks = std::max<u64>(1, (rows + ABY3G_HANDOFF_ROWS - 1) / ABY3G_HANDOFF_ROWS);
    // the residency rule first: a consumer launch that could starve its
    // producer of slots keeps the stream hand-off
    if (!handoffResidencyOk(handoffResidency(gpu.device()), chunks)) return aby3g_handoff{nullptr, 0, nullptr};
    // Large messages from a heavy producer keep the stream hand-off: a
    // consumer launch of many workgroups would hold its CUs spinning while the
    // producer still runs (measured slower on C3 / C5 at 512 chunks with every
    // level handed over in-kernel); small ones are latency-bound
    if (chunks > kHandoffChunks || (chunks > kHandoffMaxChunks && producerBytes > kHandoffLightBytes))
        return aby3g_handoff{nullptr, 0, nullptr};
    return aby3g_handoff{p.hsFlags, ++p.hsSeq, nullptr};
}

bool Channel::handoffCapable(const Gpu& gpu) const {
    if (!mOut || !mIn || kernelsSerialized()) return false;
    for (const Pipe* p : {mOut.get(), mIn.get()})
        if (!p->kernelHandoff || p->link || p->signalDevice != gpu.device()) return false;
    return true;
}

bool handoffResidencyOk(const HandoffResidency& r, u64 chunks, int processes) {
    const int per = chunks < (u64)std::max(0, r.smallMaxWgs) ? r.perCuSmall : r.perCuLarge;
    if (per <= 0 || r.cus <= 0 || !chunks || processes < 1) return false;
    const u64 cusHeld = (chunks + (u64)per - 1) / (u64)per;
    return 2 * cusHeld + (u64)processes * (u64)std::max(0, r.otherSpinners) + 1 <= (u64)r.cus;
}

const HandoffResidency& handoffResidency(int device) {
    static std::mutex mu;
    static std::map<int, HandoffResidency> byDevice;
    std::lock_guard<std::mutex> lk(mu);
    auto it = byDevice.find(device);
    if (it != byDevice.end()) return it->second;
    HandoffResidency r;
    GPU_CALL(aby3g_set_device(device));
    GPU_CALL(aby3g_bin_level_residency(&r.cus, &r.perCuSmall, &r.perCuLarge, &r.smallMaxWgs));
    // stream-operation waits can spin on every stream of the device: at most
    // one per hardware queue of the process
    r.otherSpinners = hwQueuesPerDevice();
    return byDevice.emplace(device, r).first->second;
}

std::shared_ptr<DeviceBuffer> Channel::evalSendBuffer(Gpu& gpu, size_t bytes, u64 andLevels,
                                                     std::shared_ptr<void>* lease) {
    if (!lease) throw std::runtime_error("evalSendBuffer: null lease");
    if (!mOut || !mOut->link || !mOut->arena || kernelsSerialized() || bytes > mOut->arenaSlot) return nullptr;
    Pipe& p = *mOut;
    if (andLevels < 2 || p.arenaOpen) return nullptr;
    p.arenaOpen = 1;
    std::weak_ptr<Pipe> pipe = mOut;  // the lease does not keep the channel alive
    static int tag;  // a non-null token: the lease tests true while held
    *lease = std::shared_ptr<void>(&tag, [pipe](void*) {
        if (auto q = pipe.lock()) q->arenaOpen = 0;
    });
    const u64 slot = p.arenaNext++ & 1;
    return DeviceBuffer::borrow(p.arenaSlots() + slot * p.arenaSlot, bytes, &gpu);
}

bool Channel::linkedConcurrent() const {
    return mOut && mIn && mOut->link && mIn->link && !kernelsSerialized();
}

void Channel::asyncSendShared(std::shared_ptr<DeviceBuffer> buf, size_t bytes, Gpu& gpu, const aby3g_handoff& posted) {
    if (!posted.flags) {
        asyncSendShared(std::move(buf), bytes, gpu);
        return;
    }
    if (!mOut) throw std::runtime_error("channel not connected");
    if (!buf || buf->bytes() < bytes) throw std::runtime_error("asyncSendShared: buffer smaller than the message");
    if (mOut->link) {
        Pipe& p = *mOut;
        if (posted.flags != p.arenaFlags() || posted.seq != p.hsSeq)
            throw std::runtime_error("asyncSendShared: the hand-off is not this channel's latest (handoffPost)");
        std::lock_guard<std::mutex> lk(p.mu);
        WireMsg w{};
        w.bytes = bytes;
        w.kind = 2;
        w.slot = kNoSlot;
        w.gen = (u64)((const u8*)buf->data() - p.arenaSlots());
        w.seq = posted.seq;
        w.device = gpu.device();
        p.sent += bytes;
        p.ringWrite(std::vector<u8>((const u8*)&w, (const u8*)&w + sizeof w));
        return;
    }
    if (posted.flags != mOut->hsFlags || posted.seq != mOut->hsSeq)
        throw std::runtime_error("asyncSendShared: the hand-off is not this channel's latest (handoffPost)");
    Msg m;
    m.device = true;
    m.bytes = bytes;
    m.shared = std::move(buf);
    m.hsFlags = posted.flags;
    m.hsSeq = posted.seq;
    mOut->push(std::move(m));
}

bool Channel::linked() const { return mOut && mOut->link; }

std::shared_ptr<DeviceBuffer> Channel::linkSendBuffer(Gpu& gpu, size_t bytes) {
    if (!mOut) throw std::runtime_error("channel not connected");
    if (!mOut->link) return std::make_shared<DeviceBuffer>(gpu, std::max<size_t>(bytes, 8));
    GPU_CALL(aby3g_set_device(gpu.device()));
    return DeviceBuffer::borrow(mOut->linkReserve(bytes, gpu), std::max<size_t>(bytes, 8), &gpu);
}

RecvFuture Channel::asyncRecvShared(size_t bytes, Gpu& gpu) {
    RecvFuture f = asyncRecv(nullptr, bytes);
    f.mState->gpu = &gpu;
    f.mState->shared = true;
    return f;
}

void Channel::asyncSendCopy(const void* data, size_t bytes) {
    if (!mOut) throw std::runtime_error("channel not connected");
    Msg m;
    m.bytes = bytes;
    m.host.assign((const u8*)data, (const u8*)data + bytes);
    mOut->push(std::move(m));
}

RecvFuture Channel::asyncRecv(void* dst, size_t bytes) {
    if (!mIn) throw std::runtime_error("channel not connected");
    RecvFuture f;
    f.mState = std::make_shared<RecvFuture::State>();
    f.mState->pipe = mIn;
    f.mState->dst = dst;
    f.mState->bytes = bytes;
    {
        std::lock_guard<std::mutex> lk(mIn->mu);
        f.mState->ticket = mIn->recvTicket++;
    }
    return f;
}

void Channel::asyncSendDevice(const void* src, size_t bytes, Gpu& gpu) {
    if (!mOut) throw std::runtime_error("channel not connected");
    GPU_CALL(aby3g_set_device(gpu.device()));
    if (mOut->link) {
        mOut->linkSendDevice(src, bytes, gpu);
        return;
    }
    Slot* s = mOut->acquire(bytes, gpu.device());
    if (s->consumedRecorded) GPU_CALL(aby3g_stream_wait_event(gpu.stream(), s->consumed->get()));
    if (bytes) GPU_CALL(aby3g_memcpy(s->ptr, src, bytes, 2, gpu.stream()));  // staging slot on the sender's device
    Msg m;
    m.device = true;
    m.slot = s;
    m.bytes = bytes;
    mOut->signalReady(m, gpu, s->ready.get());
    mOut->push(std::move(m));
}

RecvFuture Channel::asyncRecvDevice(void* dst, size_t bytes, Gpu& gpu) {
    RecvFuture f = asyncRecv(dst, bytes);
    f.mState->gpu = &gpu;
    return f;
}

u64 Channel::bytesSent() const { return mOut ? mOut->sent : 0; }
u64 Channel::bytesRecv() const { return mIn ? mIn->received : 0; }
void Channel::resetStats() {
    if (mOut) mOut->sent = 0;
    if (mIn) mIn->received = 0;
}

double recvWaitUs() { return t_recvWaitUs; }

// Stream-ordered signal words are waited for by a spinning blit kernel: a
// tool that serialises kernels (rocprofv3 --pmc, which sets
// ROCPROF_COUNTER_COLLECTION in the profiled process; AMD_SERIALIZE_KERNEL)
// would run the waiting kernel alone and never the writer -- there the
// channels use events.
bool kernelsSerialized() {
    static const bool ser = [] {
        for (const char* v : {"AMD_SERIALIZE_KERNEL", "ROCPROF_COUNTER_COLLECTION"}) {
            const char* e = getenv(v);
            if (e && e[0] && e[0] != '0') return true;
        }
        return false;
    }();
    return ser;
}
static bool signalWordsAllowed() { return !kernelsSerialized(); }

int hwQueuesPerDevice() {
    static const int n = [] {
        const char* e = getenv("GPU_MAX_HW_QUEUES");
        const int v = e ? atoi(e) : 0;
        return v > 0 ? v : 4;
    }();
    return n;
}

std::vector<CommPkg> makeLocalRing(const int* devices, bool kernelHandoff) {
    // parties on different devices read each other's buffers in place
    // (zero-copy messages): that needs peer access both ways
    if (devices)
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                if (devices[i] != devices[j]) GPU_CALL(aby3g_enable_peer_access(devices[i], devices[j]));
    if (!signalWordsAllowed()) devices = nullptr;
    // pipe[i][j]: messages from party i to party j
    std::shared_ptr<Pipe> p[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            if (i != j) {
                p[i][j] = std::make_shared<Pipe>();
                if (devices && devices[i] == devices[j]) {
                    p[i][j]->signalDevice = devices[i];
                    p[i][j]->kernelHandoff = kernelHandoff;
                }
            }
    // every same-device direction's signal word, zeroed now, before any
    // party's work is enqueued (aby3g_signal_alloc zeroes it on a stream of
    // its own: a null-stream memset here created the null stream's hardware
    // queue ahead of the parties' streams and shifted which streams share a
    // queue -- C3 0.41 against 0.334 ms in a same-box A/B)
    if (devices) {
        int cur = 0;
        GPU_CALL(aby3g_get_device(&cur));
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                if (i != j && p[i][j]->signalDevice >= 0) {
                    GPU_CALL(aby3g_set_device(p[i][j]->signalDevice));
                    GPU_CALL(aby3g_signal_alloc(&p[i][j]->word));
                }
        GPU_CALL(aby3g_set_device(cur));
    }
    std::vector<CommPkg> c(3);
    for (int i = 0; i < 3; ++i) {
        int nx = (i + 1) % 3, pv = (i + 2) % 3;
        c[i].mNext = Channel(p[i][nx], p[nx][i]);
        c[i].mPrev = Channel(p[i][pv], p[pv][i]);
    }
    return c;
}

CommPkg makeProcessRing(int party, const std::string& link, int device, bool sameDevice, bool forceRemote) {
    if (forceRemote) sameDevice = false;  // no arenas: staged copies, as between GPUs
    if (party < 0 || party > 2) throw std::runtime_error("makeProcessRing: party must be 0, 1 or 2");
    if (link.empty() || link.find('/') != std::string::npos)
        throw std::runtime_error("makeProcessRing: link name must be non-empty without '/'");
    auto seg = [&](int from, int to) { return "/aby3." + link + "." + std::to_string(from) + std::to_string(to); };
    auto end = [&](int from, int to) {
        auto p = std::make_shared<Pipe>();
        p->link = std::make_unique<LinkEnd>(seg(from, to), from == party, device);
        p->linkDevice = device;
        return p;
    };
    const int nx = (party + 1) % 3, pv = (party + 2) % 3;
    // attach order is the same in every process (lower party pair first),
    // so the handshakes never wait on each other in a cycle
    std::shared_ptr<Pipe> pipes[3][3];
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b)
            if (a != b && (a == party || b == party)) pipes[a][b] = end(a, b);
    {
        // `sameDevice` is the caller's claim; the arenas need all three
        // parties on ONE GPU (their level kernels poll agent-scope flags and
        // read coarse-grained payloads). Each process sends its claim and its
        // device UUID to both neighbours and checks both: every process then
        // reaches the same answer (all three claim it and their UUIDs are
        // equal, or not), so they all take the arenas or none do -- a mixed
        // layout (two parties on one GPU, one on another) or a disagreeing
        // claim falls back to the staged copies.
        u8 own[16];
        GPU_CALL(aby3g_device_uuid(device, own));
        for (int to : {nx, pv}) {
            WireMsg w{};
            w.kind = 4;
            w.slot = kNoSlot;
            w.seq = sameDevice ? 1 : 0;
            w.device = device;
            std::memcpy(w.handle.bytes, own, 16);
            pipes[party][to]->ringWrite(std::vector<u8>((const u8*)&w, (const u8*)&w + sizeof w));
        }
        for (int from : {pv, nx}) {
            WireMsg w;
            pipes[from][party]->link->read(&w, sizeof w);
            if (w.kind != 4) throw std::runtime_error("makeProcessRing: expected the peer's device identity");
            if (w.seq != 1 || std::memcmp(w.handle.bytes, own, 16) != 0) sameDevice = false;
        }
    }
    if (sameDevice && !kernelsSerialized()) {
        // the arenas of in-kernel hand-offs: each process announces its two
        // outgoing ones (zeroed, then exported), then maps the two incoming
        const char* e = getenv("ABY3_ARENA_MB");
        const u64 slot = (u64)(e && atoi(e) > 0 ? atoi(e) : 32) << 20;
        GPU_CALL(aby3g_set_device(device));
        aby3g_stream tmp = nullptr;  // not the null stream (it would hold a hardware queue)
        GPU_CALL(aby3g_stream_create(&tmp));
        for (int to : {nx, pv}) {
            Pipe& p = *pipes[party][to];
            GPU_CALL(aby3g_malloc(&p.arena, ipcBytes(kArenaFlagBytes + 2 * slot)));
            GPU_CALL(aby3g_memset(p.arena, 0, kArenaFlagBytes, tmp));
            GPU_CALL(aby3g_stream_sync(tmp));
            p.arenaSlot = slot;
            WireMsg w{};
            w.kind = 3;
            w.slot = kNoSlot;
            w.gen = slot;
            w.device = device;
            GPU_CALL(aby3g_ipc_get_handle(p.arena, &w.handle));
            p.ringWrite(std::vector<u8>((const u8*)&w, (const u8*)&w + sizeof w));
        }
        GPU_CALL(aby3g_stream_destroy(tmp));
        for (int from : {pv, nx}) {
            Pipe& p = *pipes[from][party];
            WireMsg w;
            p.link->read(&w, sizeof w);
            if (w.kind != 3) throw std::runtime_error("makeProcessRing: expected the peer's arena announce");
            GPU_CALL(aby3g_ipc_open(&w.handle, &p.arena));
            p.arenaSlot = w.gen;
            p.arenaMapped = true;
        }
    }
    CommPkg c;
    c.mNext = Channel(pipes[party][nx], pipes[nx][party]);
    c.mPrev = Channel(pipes[party][pv], pipes[pv][party]);
    c.forceRemote = forceRemote;
    return c;
}

}  // namespace aby3
