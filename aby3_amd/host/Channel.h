// Ordered point-to-point message channels between parties (the role of
// cryptoTools' oc::Channel in the reference; CommPkg = {mPrev, mNext},
// aby3/sh3/Sh3Types.h:32-34).
//
// Semantics kept from the reference:
//   * FIFO per direction, untyped on the wire: the receiver must post its
//     receives in the order the sender sent (sizes are checked);
//   * asyncSendCopy copies the payload at send time;
//   * asyncRecv returns a future; the payload is usable after get().
// Device payloads never touch the host: the sender copies into a staging slot
// on its own stream and records an event; the receiver's get() makes its
// stream wait for that event and copies the slot into the destination (peer
// copy over xGMI when the parties sit on different GPUs). Every enqueue on a
// party's stream is issued by that party's thread, so stream order equals the
// protocol order.
#pragma once
#include "Device.h"
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace aby3 {

struct Pipe;  // one direction

class RecvFuture {
public:
    RecvFuture() = default;
    // Waits for the message and makes its payload available at the
    // destination (device payload: ordered on the receiver's stream).
    void get() const;
    // for asyncRecvShared: waits (on the receiver's stream) for the message
    // and returns the sender's buffer itself. After enqueueing its last read
    // of it, the receiver calls buffer->fence(its stream).
    std::shared_ptr<DeviceBuffer> getShared() const;
    // getShared for a consumer kernel that can wait on the device itself
    // (aby3g_handoff): when the sender's kernel published the message chunk by
    // chunk (Channel::handoffPost), fills `wait` and enqueues nothing; else
    // enqueues the stream wait as getShared does and leaves wait.flags null.
    // wait.wait_ticks is the receiver's Gpu::waitTicks().
    std::shared_ptr<DeviceBuffer> getSharedHandoff(aby3g_handoff& wait) const;
    bool valid() const { return (bool)mState; }

    struct State;
    std::shared_ptr<State> mState;
};

class Channel {
public:
    Channel() = default;
    Channel(std::shared_ptr<Pipe> out, std::shared_ptr<Pipe> in) : mOut(std::move(out)), mIn(std::move(in)) {}

    // host payloads
    void asyncSendCopy(const void* data, size_t bytes);
    template <class T>
    void asyncSendCopy(const T& v) {
        asyncSendCopy(&v, sizeof(T));
    }
    void send(const void* data, size_t bytes) { asyncSendCopy(data, bytes); }
    RecvFuture asyncRecv(void* dst, size_t bytes);
    void recv(void* dst, size_t bytes) { asyncRecv(dst, bytes).get(); }
    template <class T>
    void recv(T& v) {
        recv(&v, sizeof(T));
    }

    // device payloads, enqueued on / delivered to `gpu`'s stream
    void asyncSendDevice(const void* src, size_t bytes, Gpu& gpu);
    RecvFuture asyncRecvDevice(void* dst, size_t bytes, Gpu& gpu);
    // zero-copy device payloads: the message is the sender's buffer (the same
    // buffer may go to several receivers); readiness is an event recorded on
    // the sender's stream at send time. The receiver reads it in place (over
    // xGMI when on another GPU) and fences it when done.
    void asyncSendShared(std::shared_ptr<DeviceBuffer> buf, size_t bytes, Gpu& gpu);
    // the same, readiness signalled by an event record even on one device (no
    // stream-write / stream-wait blit kernels on the queues): for messages
    // whose receiver waits long anyway (asyncMul's truncation z, behind the
    // peers' share GEMMs), where it measured as fast as the signal word
    // (C2 0.2548-0.2566 vs 0.2568-0.2575 ms); the binary engine's level
    // messages keep the signal word (C3 0.313-0.315 vs 0.323 ms with events)
    void asyncSendSharedEvent(std::shared_ptr<DeviceBuffer> buf, size_t bytes, Gpu& gpu);
    RecvFuture asyncRecvShared(size_t bytes, Gpu& gpu);
    // A buffer for a message this party is about to produce and then send
    // with asyncSendShared / asyncSendSharedEvent on this channel. Between
    // processes it is one of the direction's IPC-exported staging slots, so
    // the send skips the staging copy (the producer writes the slot itself,
    // ordered behind the receiver's copy-out of the slot's previous message);
    // otherwise a buffer of this party's pool. It must be sent on this
    // channel before the next linkSendBuffer; it may also go to other
    // channels (they stage a copy) and be read by this party.
    std::shared_ptr<DeviceBuffer> linkSendBuffer(Gpu& gpu, size_t bytes);
    bool linked() const;  // the outgoing direction leads to another process
    // In-kernel hand-off of the next zero-copy message (co-located parties on
    // one device whose ring was made with kernel hand-offs): the flags and
    // sequence number for the producing kernel to publish a message of `rows`
    // rows (aby3g_handoff); flags null when this channel cannot do it. The
    // producer is enqueued with it, then the message is sent with
    // asyncSendShared(buf, bytes, gpu, posted): no stream operation.
    // producerBytes: HBM bytes of the producing launch (large messages go
    // in-kernel only from light producers)
    // payload: the message's buffer; between processes it must lie in this
    // direction's arena (evalSendBuffer) for an in-kernel hand-off
    aby3g_handoff handoffPost(Gpu& gpu, u64 rows, u64 producerBytes = 0, const void* payload = nullptr);
    // One party per process on one GPU: a buffer for an evaluation's messages
    // inside this direction's IPC-mapped arena (two slots, alternating per
    // call), which the receiver reads in place -- null when the direction has
    // no arena, `bytes` exceeds a slot, the circuit has fewer than two AND
    // levels, or another evaluation's lease on the arena is still open (the
    // caller then allocates its own). A slot is rewritten two evaluations
    // later; that is safe only when the evaluations run one after another on
    // the party's stream and each has two or more AND levels (the receiver's
    // reads of evaluation e precede, in its stream, its first message of e+1,
    // which the sender's e+1 needs before it starts e+2). The lease is held by
    // *lease and ends when the caller drops it -- once the evaluation's last
    // message is sent, or whenever the evaluation is reset or abandoned.
    std::shared_ptr<DeviceBuffer> evalSendBuffer(Gpu& gpu, size_t bytes, u64 andLevels, std::shared_ptr<void>* lease);
    // Both directions join parties on `gpu`'s device in this process whose
    // ring allows kernel hand-offs (a fused launch may then address the
    // peer's device memory and poll it).
    bool handoffCapable(const Gpu& gpu) const;
    // Both directions are links to parties in other processes
    // (makeProcessRing): each party's streams own their hardware queues, so a
    // kernel may poll a peer's IPC-mapped memory while kernels run
    // concurrently (not under a kernel-serialising profiler).
    bool linkedConcurrent() const;
    void asyncSendShared(std::shared_ptr<DeviceBuffer> buf, size_t bytes, Gpu& gpu, const aby3g_handoff& posted);

    u64 bytesSent() const;
    u64 bytesRecv() const;
    void resetStats();

    bool connected() const { return mOut && mIn; }

private:
    void sendShared(std::shared_ptr<DeviceBuffer> buf, size_t bytes, Gpu& gpu, bool word);
    std::shared_ptr<Pipe> mOut, mIn;
};

struct CommPkg {
    Channel mPrev, mNext;
    // one party per process, all three on one GPU, but every branch taken as
    // if each party had a GPU of its own (makeProcessRing's forceRemote): the
    // staged IPC copies for every device message and the fused LR
    // iteration's system-scope mailboxes -- the north-star layout's code
    // paths, run on a one-GPU box
    bool forceRemote = false;
};

// Host time this thread has spent inside receives waiting for messages (us).
double recvWaitUs();

// True when a profiler or the runtime serialises kernels (rocprofv3 --pmc,
// AMD_SERIALIZE_KERNEL): no kernel or blit may then wait on another stream's
// progress on the device, so channels hand off through events.
bool kernelsSerialized();

// Hardware queues HIP gives a process per device (GPU_MAX_HW_QUEUES, default
// 4): streams beyond it share queues, and a kernel waiting in a shared queue
// would block the work queued behind it.
int hwQueuesPerDevice();

// The in-kernel hand-off residency rule. A consumer launch's workgroups spin
// until their chunks arrive, so the producer of a message must always find a
// slot: at most two parties' consumer launches spin at once (a party's next
// level waits behind its own current one on its stream, so one of the three
// is always the producer), besides at most `otherSpinners` stream-operation
// wait kernels (one per hardware queue of each process on the device: three
// processes sharing one GPU bring three sets). Counted in whole CUs, since
// the dispatcher may spread a launch over every CU: a consumer of c chunks
// (c workgroups of the small form when c < smallMaxWgs, else of the large
// one) holds at most ceil(c / perCu) CUs' worth of its kernel's slots, and
//     2 ceil(c / perCu) + processes * otherSpinners + 1 <= cus
// leaves the producer a CU. The rule holds for consumers of ONE chunk per
// workgroup (the level kernel's hand-off instantiations): a workgroup that
// looped over several chunks would hold its slot across waits on different
// producers' chunks, and would need every party's whole grid co-resident.
struct HandoffResidency {
    int cus = 0;
    int perCuSmall = 0, perCuLarge = 0;  // level-kernel workgroups resident per CU
    int smallMaxWgs = 0;
    int otherSpinners = 0;
};
bool handoffResidencyOk(const HandoffResidency& r, u64 chunks, int processes = 1);
// the current device's figures (aby3g_bin_level_residency, computed once per
// device; otherSpinners = GPU_MAX_HW_QUEUES)
const HandoffResidency& handoffResidency(int device);

// Three in-process parties connected in a ring: result[i].mNext talks to
// party i+1, result[i].mPrev to party i-1. With `devices` (party i runs on
// devices[i]), device payloads between parties on one device are signalled
// through stream-ordered words instead of events.
// kernelHandoff: messages between parties on one device may be handed over
// inside the kernels (Channel::handoffPost); only for parties whose streams
// each own a hardware queue (one stream per party, at most GPU_MAX_HW_QUEUES
// streams on the device), which the caller vouches for.
std::vector<CommPkg> makeLocalRing(const int* devices = nullptr, bool kernelHandoff = false);

// One party per process (the reference's deployment): the CommPkg of `party`
// in this process, its four directions carried by shared-memory links named
// after `link` (the same string in the three processes, unique per session;
// Link.h). Blocks until the two other parties have attached. Device payloads
// are staged in IPC-exported slots and copied out by the receiver; a
// zero-copy send (asyncSendShared) becomes such a staged copy.
// sameDevice: the three processes share this GPU; the binary engine's level
// messages then go in-kernel through IPC-mapped arenas (one per direction).
CommPkg makeProcessRing(int party, const std::string& link, int device, bool sameDevice = false,
                        bool forceRemote = false);

}  // namespace aby3
