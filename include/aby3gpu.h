/*
 * aby3gpu.h -- C-ABI of the MI355X (gfx950) local-compute engine for ABY3's
 * replicated-secret-sharing hot path.
 *
 * Every entry point replaces one local-compute step of the reference
 * (Fannxy/aby3 @ 2024-10-24, paths relative to /root/reference). The host
 * runtime (aby3_amd/host: Sh3Runtime / Sh3Evaluator / Sh3Encryptor /
 * Sh3BinaryEvaluator / Sh3Piecewise) is the only intended caller; it owns the
 * protocol, the message schedule and every stream offset, and calls these
 * functions with plain device pointers.
 *
 * Conventions
 *   - All data pointers are DEVICE pointers owned by the caller unless a
 *     parameter says "host". Calls are asynchronous on `stream` (a hipStream_t
 *     passed as void*; NULL = the default stream) and thread-compatible.
 *   - A shared matrix of one party is ONE contiguous allocation [2][rows][cols]
 *     of int64: share 0 (x_i) followed by share 1 (x_{i-1}) -- the two
 *     Eigen buffers of si64Matrix (aby3/sh3/Sh3Types.h:198-271) made adjacent.
 *   - Arithmetic is mod 2^64 (two's complement wrap), shifts are arithmetic.
 *   - Randomness follows cryptoTools: AES(k, c) encrypts LE64(c) || 0^8;
 *     PRNG(seed) is the byte stream of AES(seed, 0), AES(seed, 1), ...
 *     (SURVEY.md Appendix A). Stream positions are explicit arguments.
 *   - Return value: 0 on success, nonzero ABY3G_E* on error; the message is
 *     available from aby3g_last_error() (thread-local). No exceptions cross.
 */
#ifndef ABY3GPU_H
#define ABY3GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* aby3g_stream;
typedef void* aby3g_event;

enum { ABY3G_OK = 0, ABY3G_EINVAL = 1, ABY3G_EHIP = 2, ABY3G_ENOMEM = 3 };

/* ------------------------------------------------------------------ misc -- */
const char* aby3g_last_error(void);
/* Diagnostics: the names of this process's last 32 C-ABI calls, newest
 * first, joined by " < " into out (cap bytes, NUL-terminated). A device fault
 * is reported by a later call than the one that enqueued the faulting work;
 * that work is among these. (No reference counterpart.) */
int aby3g_recent_calls(char* out, size_t cap);
int aby3g_version(void);
int aby3g_device_count(int* n);
/* The calling thread's current device. The library remembers the device
 * each thread last set here (hipSetDevice / hipGetDevice serialise with other
 * threads' launches), so a thread that drives the library switches devices
 * only through aby3g_set_device. */
int aby3g_set_device(int device);
int aby3g_get_device(int* device);
/* Host time the calling thread has spent inside aby3g_* calls, and their number. */
int aby3g_api_time(double* us, uint64_t* calls);

/* Memory, streams and events. The host runtime reaches the GPU only through
 * this header. kind: 0 host->device, 1 device->host, 2 device->device with
 * both buffers readable / writable from the current device (a copy kernel),
 * 3 let the runtime infer (also peer copies between devices). */
int aby3g_malloc(void** ptr, size_t bytes);
int aby3g_free(void* ptr);
/* device memory that no cache holds (hipDeviceMallocUncached): flags and
 * mailboxes polled from other GPUs; free with aby3g_free */
int aby3g_malloc_uncached(void** ptr, size_t bytes);
int aby3g_host_malloc(void** ptr, size_t bytes); /* pinned host memory */
int aby3g_host_free(void* ptr);
int aby3g_memcpy(void* dst, const void* src, size_t bytes, int kind, aby3g_stream stream);
int aby3g_memset(void* dst, int value, size_t bytes, aby3g_stream stream);
int aby3g_stream_create(aby3g_stream* stream);
int aby3g_stream_destroy(aby3g_stream stream);
/* streams created through aby3g_stream_create and not yet destroyed on
 * `device` in this process (HIP gives a process GPU_MAX_HW_QUEUES hardware
 * queues per device; more live streams share them) */
int aby3g_stream_count(int device, int* n);
int aby3g_stream_sync(aby3g_stream stream);
int aby3g_device_sync(void);
int aby3g_event_create(aby3g_event* ev);       /* ordering only (no timestamp: cheaper to record) */
int aby3g_event_create_timed(aby3g_event* ev); /* for aby3g_event_elapsed_ms */
int aby3g_event_destroy(aby3g_event ev);
int aby3g_event_record(aby3g_event ev, aby3g_stream stream);
int aby3g_event_sync(aby3g_event ev);
/* *done = 1 once the work captured by the event's last record has completed
 * (never blocks; hipEventQuery) */
int aby3g_event_query(aby3g_event ev, int* done);
int aby3g_stream_wait_event(aby3g_stream stream, aby3g_event ev);
int aby3g_event_elapsed_ms(aby3g_event start, aby3g_event end, float* ms);
/* Stream-ordered signal words (device memory, 8 bytes): `stream` writes
 * `value` to *word once its earlier work is done / waits until *word >=
 * value before its later work starts. A cross-stream hand-off on one device
 * costs ~8 us this way against ~13.5 us for an event record + wait
 * (scripts/pingpong.hip); the channels of co-located parties use it. */
/* Creates HIP's null stream (and so its hardware queue) on the current
 * device, once per process and device; a no-op afterwards. The host calls it
 * after all its parties' streams exist and before they enqueue work: HIP
 * hands out hardware queues in stream-creation order, and where the null
 * stream's queue comes in that order changed the jobs' speed. */
int aby3g_null_queue_init(void);
int aby3g_signal_alloc(uint64_t** word); /* zeroed (on a temporary stream, never the null stream,
                                            and waited for), on the current device */
int aby3g_stream_write_value(aby3g_stream stream, uint64_t* word, uint64_t value);
int aby3g_stream_wait_value(aby3g_stream stream, uint64_t* word, uint64_t value);

/* In-kernel hand-off between co-located parties (one device, one process;
 * replaces the stream write + stream wait of a channel message). A message
 * of `rows` rows is split into chunks of ABY3G_HANDOFF_ROWS rows; the kernel
 * that produces it stores the payload write-through and, per chunk it wrote,
 * publishes flags[chunk] = seq once its stores have drained; a kernel that
 * consumes it waits, per workgroup and only for the chunks that workgroup
 * reads, until flags[chunk] >= seq, and reads the payload with L1-bypassing
 * loads. `flags` is a zeroed device array (one u64 per chunk) that a channel
 * direction reuses with increasing seq. wait_ticks (optional, consumer side):
 * the first workgroup's wait in 100 MHz wall-clock ticks is added there (the
 * device-side time a party spends blocked on its peers). Entry points taking
 * an aby3g_handoff accept NULL or flags == NULL for "no hand-off".
 * A waiting kernel can only progress while the producer's stream has a
 * hardware queue of its own; a wait gives up after 5 s, counts a timeout and
 * makes every wait enqueued before that count was seen give up too (wrong
 * results, no hang). */
#define ABY3G_HANDOFF_ROWS 2048
typedef struct {
    uint64_t* flags;
    uint64_t seq;
    uint64_t* wait_ticks;
} aby3g_handoff;
/* The count of in-kernel hand-off waits on the current device that timed
 * out since the process started (never reset: a caller compares the count
 * before and after its run; a change means its results are invalid, also
 * when another caller on the device caused it). No GPU call (the counter is
 * pinned host memory). */
int aby3g_handoff_status(uint32_t* timeouts);
/* Debug: the wait limit of in-kernel hand-offs enqueued from now on
 * (default 5 s), so tests can force a timeout quickly. */
int aby3g_set_handoff_timeout_us(uint64_t us);

/* Cross-process transport: one party per process (the
 * reference's parties are processes joined by cryptoTools Channels over TCP,
 * Sh3Types.h:32-34, Eval/dis_exec.sh:10-12). A channel's staging slots are
 * device buffers exported through IPC handles (hipIpcGetMemHandle); its
 * stream-ordered signal words live in host memory shared by the processes
 * (POSIX shm) and registered with each party's device; parties on different
 * devices of one process reach each other's buffers through peer access. */
typedef struct {
    unsigned char bytes[64];
} aby3g_ipc_handle;
/* ptr: the base pointer of an aby3g_malloc / aby3g_malloc_uncached allocation
 * whose size is a multiple of ABY3G_IPC_GRANULE (2 MiB) -- anything else is
 * refused (ABY3G_EINVAL). Smaller allocations may be fragments that the
 * runtime carves out of a shared 2 MiB block; only whole blocks are exported. */
#define ABY3G_IPC_GRANULE ((size_t)2 << 20)
int aby3g_ipc_get_handle(void* ptr, aby3g_ipc_handle* handle);
int aby3g_ipc_open(const aby3g_ipc_handle* handle, void** ptr); /* mapped for the current device */
int aby3g_ipc_close(void* ptr);
/* page-aligned host memory -> an address the current device's streams can
 * write / wait on (aby3g_stream_write_value / aby3g_stream_wait_value) */
int aby3g_host_register(void* host, size_t bytes, void** dev);
int aby3g_host_unregister(void* host);
/* lets `device` read and write `peer`'s memory (0 also when already enabled;
 * an error when the two devices cannot reach each other) */
int aby3g_enable_peer_access(int device, int peer);
/* the device's 16-byte UUID (hipDeviceGetUuid): which physical GPU an
 * ordinal is, comparable between processes whatever their visible devices */
int aby3g_device_uuid(int device, uint8_t uuid[16]);

/* Kernel timing probe: when enabled, every kernel launched by this library on
 * the calling thread is bracketed by events; aby3g_probe_read() returns the
 * accumulated device time (ms) and launch count per kernel family:
 * 0 share GEMM (MFMA), 1 mul epilogue / hadamard,
 * 2 binary gate layers, 3 AES streams, 4 other, 5 GEMM digit planes.
 * Used by bench.py. */
int aby3g_probe_enable(int on);             /* all families (on != 0) or none */
int aby3g_probe_enable_mask(uint32_t mask); /* only the families in mask (bit = 1 << family) */
int aby3g_probe_read(int family, double* ms, uint64_t* launches);
int aby3g_probe_reset(void);

/* --------------------------------------------------- AES / PRNG streams -- */
/* oc::AES::ecbEncCounterMode: out[i] = AES(key, ctr_base + i), 16 B each.
 * Replaces the host AES-NI refills of Sh3ShareGen.h:50-56 and SharedOT.cpp:15. */
int aby3g_aes_ctr(const uint8_t key[16], uint64_t ctr_base, uint64_t nblocks, void* out, aby3g_stream stream);

/* Host-side AES-128 of one counter block, out = AES(key, LE64(ctr) || 0^8).
 * Runs on the CPU (no GPU work, no synchronization); the host runtime uses
 * it only to derive keys from the first blocks of a PRNG stream
 * (Sh3ShareGen.h:19-20, Sh3Evaluator.cpp:13-14, Sh3BinaryEvaluator.h:96-102). */
int aby3g_aes_block_host(const uint8_t key[16], uint64_t ctr, uint8_t out[16]);
/* Host-side AES-CTR of n counter blocks (one key schedule): the host PRNG
 * of the aby3-ML driver's setup -- the data model's PRNG(toBlock(1)) and
 * SGD_Logistic's mini-batch PRNG(toBlock(234543234)) (main-logistic.cpp:
 * 82-92, Regression.h:24-40, 255). CPU only. */
int aby3g_aes_ctr_host(const uint8_t key[16], uint64_t ctr_base, uint64_t nblocks, uint8_t* out);

/* oc::PRNG(seed) bytes [byte_off, byte_off + nbytes) (both multiples of 8).
 * Replaces mPrevCommon/mNextCommon.get(...) (Sh3Evaluator.cpp:526-527,
 * Sh3BinaryEvaluator.h:96-102, Sh3Evaluator.cpp:151-153,188,234-235). */
int aby3g_prng_fill(const uint8_t seed[16], uint64_t byte_off, uint64_t nbytes, void* out, aby3g_stream stream);

/* The calling thread's cap on the workgroups of aby3g_share_draws (default
 * 256, one per CU: the draws run beside co-located parties' work). A party
 * alone on its stream (one party per process) raises it: its draws stand in
 * front of its own first level. (No reference counterpart.) */
int aby3g_set_draw_workgroups(int cap);
/* Sh3ShareGen draws j = draw_base .. draw_base+n-1 with the two zero-share
 * keys (k_prev = mShareGen[0], k_next = mShareGen[1]; Sh3ShareGen.h:19-20).
 *   ABY3G_DRAW_ARITH:    out0[i] = getShare()       (+ addend[i])   Sh3ShareGen.h:60-75
 *   ABY3G_DRAW_BIN:      out0[i] = getBinaryShare() (^ addend[i])   Sh3ShareGen.h:77-92
 *   ABY3G_DRAW_RANDPAIR: (out0[i], out1[i]) = getRandIntShare()     Sh3ShareGen.h:95-109
 * addend may be NULL. Used by Sh3Encryptor::local/remote*Matrix
 * (Sh3Encryptor.cpp:229-340) and the binary engine's AND-gate masks
 * (Sh3BinaryEvaluator.cpp:1406-1434, where z[k][w] is draw k*words + w). */
enum { ABY3G_DRAW_ARITH = 0, ABY3G_DRAW_BIN = 1, ABY3G_DRAW_RANDPAIR = 2 };
int aby3g_share_draws(int kind, const uint8_t k_prev[16], const uint8_t k_next[16], uint64_t draw_base, uint64_t n,
                      const int64_t* addend, int64_t* out0, int64_t* out1, aby3g_stream stream);
/* Rows of draws (kind ARITH or BIN): out0[r * row_len + i] = draw
 * (draw_base + r * row_stride + i) for r < nrows, i < row_len; draw_base,
 * row_len and row_stride even. A row slice of the binary engine's masks: z[k]
 * of words [w0, w0 + row_len) of a circuit over row_stride words is
 * draw_base = w0, row stride row_stride (Sh3BinaryEvaluator::setCirRows).
 * (No reference counterpart: the reference never splits a party's rows.) */
int aby3g_share_draws_rows(int kind, const uint8_t k_prev[16], const uint8_t k_next[16], uint64_t draw_base,
                           uint64_t row_len, uint64_t row_stride, uint64_t nrows, int64_t* out0, aby3g_stream stream);

/* -------------------------------------------------- arithmetic evaluator -- */
/* Local share product of Sh3Evaluator::asyncMul:
 *   ABY3G_MUL_HADAMARD  C0(i) = A0(i)B0(i) + A0(i)B1(i) + A1(i)B0(i)
 *                       (the fork: Sh3Evaluator.cpp:101-103, 667-668);
 *                       A, B, C are M x N (K is ignored).
 *   ABY3G_MUL_GEMM      C0 = A0 B0 + A0 B1 + A1 B0 = [A0|A1] [[B0+B1];[B0]]
 *                       (upstream: Sh3Evaluator.cpp:96-99, 662-665);
 *                       A is [2][M][K], B is [2][K][N], C is M x N.
 * GEMM runs on int8 MFMA over an exact balanced base-256 digit split
 * (36 digit-pair planes, i32 accumulation, i64 recombination). */
enum { ABY3G_MUL_HADAMARD = 0, ABY3G_MUL_GEMM = 1 };

/* Zero-share added to C0 (Sh3Evaluator.cpp:104: C0(i) += getShare(), draw
 * draw_base + i in row-major order). */
typedef struct {
    uint8_t k_prev[16];
    uint8_t k_next[16];
    uint64_t draw_base;
} aby3g_zero_share;

/* Truncation-pair streams (Sh3Evaluator.cpp:526-527): t0 <- next stream at
 * next_off, t1 <- prev stream at prev_off, 8 bytes per element, row-major. */
typedef struct {
    uint8_t next_seed[16];
    uint64_t next_off;
    uint8_t prev_seed[16];
    uint64_t prev_off;
} aby3g_trunc_streams;

/* Share-GEMM launches on one device take turns (1) or may overlap (0, the
 * default): co-located parties'
 * overlapping GEMMs finish sooner together, but a launch's span then includes
 * the CUs spent on the others' -- bench.py's roofline pass takes turns. */
int aby3g_mfma_turn(int on);
/* The calling thread's share GEMMs run beside those of `parties` parties in
 * all (co-located parties, one stream each): split-K then fills 1/parties of
 * the CUs per GEMM (the others' GEMMs take the rest) instead of the whole
 * device. Default 1. Plans (and aby3g_mul_workspace_bytes) depend on it. */
int aby3g_set_gemm_sharing(int parties);

/* 1 when the whole round-1 local part runs best as one fused launch
 * (aby3g_mul_trunc_local / aby3g_mul_local with zs): Hadamard, and GEMMs of
 * up to 2^23 product terms, which run on the VALU instead of the int8-MFMA
 * digit GEMM. 0 when the truncation pair should be overlapped on a second
 * stream (aby3g_trunc_tuple + aby3g_mul_sub_local). */
int aby3g_mul_prefers_fused(int mode, uint64_t M, uint64_t K, uint64_t N);

/* Scratch needed by aby3g_mul_local / aby3g_mul_trunc_local (0 for Hadamard
 * and small GEMMs). */
size_t aby3g_mul_workspace_bytes(int mode, uint64_t M, uint64_t K, uint64_t N);

/* asyncMul without truncation, local part (Sh3Evaluator.cpp:92-116):
 * C0 = share product (+ zero-share if zs != NULL). The caller sends C0 to
 * next and receives C1 from prev. zs is a HOST pointer. */
int aby3g_mul_local(int mode, const int64_t* A, const int64_t* B, int64_t* C0, uint64_t M, uint64_t K, uint64_t N,
                    const aby3g_zero_share* zs, void* workspace, size_t workspace_bytes, aby3g_stream stream);

/* getTruncationTuple (Sh3Evaluator.cpp:503-566): R = t0 >> 2,
 * RT = (t0 >> (d+2), t1 >> (d+2)); RT is [2][n]. ts is a HOST pointer. */
int aby3g_trunc_tuple(const aby3g_trunc_streams* ts, uint64_t n, unsigned d, int64_t* R, int64_t* RT,
                      aby3g_stream stream);

/* asyncMul with truncation, round-1 local part (Sh3Evaluator.cpp:658-673):
 * z = share product - R (the value sent to P0/P1), C = RT ([2][M][N]). */
int aby3g_mul_trunc_local(int mode, const int64_t* A, const int64_t* B, uint64_t M, uint64_t K, uint64_t N, unsigned d,
                          const aby3g_trunc_streams* ts, int64_t* z, int64_t* C, void* workspace,
                          size_t workspace_bytes, aby3g_stream stream);

/* The same round-1 z split for overlap (Sh3Evaluator.cpp:667-673):
 * out = share product - sub, where sub = R of aby3g_trunc_tuple, which the
 * caller may produce concurrently on another stream. The product kernels
 * are enqueued at once; the stream waits for `sub_ready` (NULL: no wait)
 * only before the final pass that reads `sub`. */
int aby3g_mul_sub_local(int mode, const int64_t* A, const int64_t* B, const int64_t* sub, aby3g_event sub_ready,
                        int64_t* out, uint64_t M, uint64_t K, uint64_t N, void* workspace, size_t workspace_bytes,
                        aby3g_stream stream);

/* Round-2 continuation (Sh3Evaluator.cpp:703-719), parties 0 and 1:
 * C[party] += (z_a + z_b + z_own) >> d  over n elements ([2][n] layout). */
int aby3g_trunc_finalize(int party, const int64_t* z_a, const int64_t* z_b, const int64_t* z_own, unsigned d,
                         int64_t* C, uint64_t n, aby3g_stream stream);

/* --------------------------------------------- 3-party OT multiplications -- */
/* A stream position: PRNG(seed) at byte offset off. */
typedef struct {
    uint8_t seed[16];
    uint64_t off;
} aby3g_stream_pos;

/* asyncMul(si64Matrix A, sbMatrix B (1 bit), C), party 0 (Sh3Evaluator.cpp:132-163):
 * per element: z <- prev, c0 <- next, c1 <- prev (prev advances 16n, next 8n);
 * C = (c0, c1); s0[bb0] = -(c0+c1)-z, s0[bb0^1] = A0+A1 + that;
 * send_msgs = SharedOT::send pads (ot_key, ctr ot_ctr) ^ s0  ([n][2]);
 * help_msgs = SharedOT::help pads (ot_key, ctr ot_ctr + n) chosen by B0 ([n]). */
int aby3g_bitmul_p0(const int64_t* A, const int64_t* B, uint64_t n, const aby3g_stream_pos* prev,
                    const aby3g_stream_pos* next, const uint8_t ot_key[16], uint64_t ot_ctr, int64_t* C,
                    int64_t* send_msgs, int64_t* help_msgs, aby3g_stream stream);
/* party 2 (:202-240): z <- next, c0 <- next per element (next advances 16n);
 * C share 0 = c0; help_msgs = pads(ot_key, ot_ctr) chosen by B1;
 * send_msgs = pads(ot_key, ot_ctr + n) ^ s1 with s1[bb1] = z, s1[bb1^1] = A1 + z. */
int aby3g_bitmul_p2(const int64_t* A, const int64_t* B, uint64_t n, const aby3g_stream_pos* next,
                    const uint8_t ot_key[16], uint64_t ot_ctr, int64_t* C, int64_t* help_msgs, int64_t* send_msgs,
                    aby3g_stream stream);
/* SharedOT::recv (SharedOT.cpp:102-126): out[i] (+)= msgs[i][c_i] ^ mc[i] where
 * c_i = choice_src[i] & 1; accumulate != 0 adds into out (mod 2^64). */
int aby3g_ot_recv(const int64_t* msgs, const int64_t* mc, const int64_t* choice_src, uint64_t n, int accumulate,
                  int64_t* out, aby3g_stream stream);

/* ---- share conversions (aby3/sh3/Sh3Converter.cpp) ----------------------
 * Choice bits come from packed binary rows: bit k of a [rows][cols64] share
 * matrix with `bits` bits per row is bit k % bits of row k / bits
 * (BitVector::append per row, Sh3Converter.cpp:240-247, 268-274).
 *
 * toBinaryMatrix's resharing (Sh3Converter.cpp:61-207), one party's part,
 * one launch over n = rows * cols64 words: with r = the draws' stream words
 * (mPrevCommon / mNextCommon.get<i64>() per element; `draws` may be NULL
 * when neither out_r nor xor_draws is used),
 *   out_r[e] = r[e] & m(e),  out_x[e] = ((a[e] + b[e]) ^ (xor_draws ? r[e] : 0)) & m(e),
 * b optional, m(e) = last_mask on the last word of each row (the
 * bitCount % 64 trim, :96-106), all ones elsewhere. Either output may be NULL. */
int aby3g_a2b_reshare(const aby3g_stream_pos* draws, uint64_t n, uint64_t cols64, uint64_t last_mask,
                      const int64_t* a, const int64_t* b, int xor_draws, int64_t* out_x, int64_t* out_r,
                      aby3g_stream stream);
/* bitInjection, party 2 = OT sender (Sh3Converter.cpp:319-361): `in` is P2's
 * [2][rows][cols64] binary shares; per bit k: dest[0][k] = next stream word,
 * dest[1][k] = prev stream word, b = bit k of in[0] ^ in[1],
 * m[k][c] = -dest0 - dest1 + (c ^ b); msgs_a = SharedOT::send pads
 * (key_a, ctr_a) ^ m, and msgs_b likewise with (key_b, ctr_b) when non-NULL
 * (the one-round variant's second OT). dest is [2][rows * bits]. */
int aby3g_bitinj_send(const int64_t* in, uint64_t rows, uint64_t cols64, uint64_t bits,
                      const aby3g_stream_pos* next, const aby3g_stream_pos* prev, const uint8_t key_a[16],
                      uint64_t ctr_a, const uint8_t key_b[16], uint64_t ctr_b, int64_t* dest, int64_t* msgs_a,
                      int64_t* msgs_b, aby3g_stream stream);
/* SharedOT::help with packed choice bits (SharedOT.cpp:30-94):
 * mc[k] = half (bit k) of AES(ot_key, ctr + k). */
int aby3g_ot_help_bits(const int64_t* choice_rows, uint64_t rows, uint64_t cols64, uint64_t bits,
                       const uint8_t ot_key[16], uint64_t ctr, int64_t* mc, aby3g_stream stream);
/* SharedOT::recv with packed choice bits: out[k] = msgs[k][bit k] ^ mc[k]. */
int aby3g_ot_recv_bits(const int64_t* msgs, const int64_t* mc, const int64_t* choice_rows, uint64_t rows,
                       uint64_t cols64, uint64_t bits, int64_t* out, aby3g_stream stream);

/* bool2arith (aby3-Basic/BoolBasic.cpp:517-593): out[i] = scale * (i64) the
 * i-th int32 of the PRNG stream from byte s->off (PRNG(seed).get<int32_t>(),
 * sign-extended; :533-545 with scale 1, :562-569 with scale -1). */
int aby3g_prng_i32(const aby3g_stream_pos* s, uint64_t n, int64_t scale, int64_t* out, aby3g_stream stream);
/* bool2arith, party 2 (:573-587): out = (c0 ^ c1 ^ recv) - t. */
int aby3g_b2a_open(const int64_t* c0, const int64_t* c1, const int64_t* recv, const int64_t* t, uint64_t n,
                   int64_t* out, aby3g_stream stream);

/* asyncMul(i64 a, sbMatrix B, C) party 0 (Sh3Evaluator.cpp:430-447):
 * s0[bb] = getShare(), s0[bb^1] = a + that, bb = B0^B1;
 * msgs_next = pads(ot_next_key, ctr_next) ^ s0; msgs_prev = pads(ot_prev_key, ctr_prev) ^ s0. */
int aby3g_pubmul_p0(int64_t a, const int64_t* B, uint64_t n, const aby3g_zero_share* zs,
                    const uint8_t ot_next_key[16], uint64_t ctr_next, const uint8_t ot_prev_key[16],
                    uint64_t ctr_prev, int64_t* msgs_next, int64_t* msgs_prev, aby3g_stream stream);
/* parties 1 and 2 (:452-487): share_out[i] = getShare(); help_msgs = pads(ot_key, ctr)
 * chosen by choice_src (P1: B share 0, P2: B share 1). */
int aby3g_pubmul_helper(const int64_t* choice_src, uint64_t n, const aby3g_zero_share* zs, const uint8_t ot_key[16],
                        uint64_t ctr, int64_t* share_out, int64_t* help_msgs, aby3g_stream stream);

/* ------------------------------------------------------- binary engine -- */
/* Gate types of the bit-sliced engine (Sh3BinaryEvaluator.cpp:700-1065) plus
 * INV (local NOT of both shares). AND, OR, NOR, NA_AND are "AND-type": their
 * share 0 is masked by z and sent to next; share 1 arrives next level. */
enum {
    ABY3G_GATE_XOR = 0,
    ABY3G_GATE_NXOR = 1,
    ABY3G_GATE_AND = 2,
    ABY3G_GATE_OR = 3,
    ABY3G_GATE_NOR = 4,
    ABY3G_GATE_NA_AND = 5,
    ABY3G_GATE_COPY = 6,
    ABY3G_GATE_INV = 7
};
/* One gate of a batch. z_row: row of the z matrix (AND-type gates);
 * send_row: row of the level's send buffer (AND-type gates). */
typedef struct {
    uint32_t in0, in1, out, type;
    uint32_t z_row, send_row;
} aby3g_gate;

/* Evaluate a batch of mutually independent gates over `words` 64-row words.
 * mem = [2][wires][words] u64 (wire-major, Sh3Types.h:537-599 sPackedBin),
 * z = [nAnd][words] masks (aby3g_share_draws ABY3G_DRAW_BIN with the setCir
 * keys), sendbuf = [levelAnds][words]. gates is a DEVICE array. */
int aby3g_bin_gates(const aby3g_gate* gates, uint32_t ngates, uint64_t* mem, uint64_t wires, uint64_t words,
                    const uint64_t* z, uint64_t* sendbuf, aby3g_stream stream);
/* Level entry (:555-573): share-1 row of out_wires[j] <- recvbuf row j. */
/* One whole communication level in one launch (roundCallback,
 * Sh3BinaryEvaluator.cpp:539-1196): first the previous level's received AND
 * shares are unpacked (share 1 of wire unpack_wires[j] = recvbuf row j),
 * then the level's gates run in batch order -- batch b is gates
 * [batch_ends[b-1], batch_ends[b]) (device array), the gates of one batch
 * independent -- with AND-type outputs also written to sendbuf row
 * send_row. Either part may be empty. Equivalent to aby3g_bin_unpack then
 * one aby3g_bin_gates per batch. */
int aby3g_bin_level(const aby3g_gate* gates, const uint32_t* batch_ends, uint32_t nbatches, const uint64_t* recvbuf,
                    const uint32_t* unpack_wires, uint32_t nunpack, uint64_t* mem, uint64_t wires, uint64_t words,
                    const uint64_t* z, uint64_t* sendbuf, aby3g_stream stream);
/* aby3g_bin_level where the gates take share 1 of the previous level's AND
 * outputs straight from recvbuf: recv_rows (device, 2 per gate, in gate
 * order) holds the recvbuf row of in0 and in1 when that wire is unpacked by
 * this launch, else 0xffffffff. The unpack still fills the engine memory
 * for later levels, but the first batch no longer waits for it. */
int aby3g_bin_level_rr(const aby3g_gate* gates, const uint32_t* recv_rows, const uint32_t* batch_ends,
                       uint32_t nbatches, const uint64_t* recvbuf, const uint32_t* unpack_wires, uint32_t nunpack,
                       uint64_t* mem, uint64_t wires, uint64_t words, const uint64_t* z, uint64_t* sendbuf,
                       aby3g_stream stream);
/* aby3g_bin_level_rr with in-kernel hand-offs between co-located parties:
 * `wait` for the received AND shares in recvbuf (the previous party's level
 * launch published them), `post` for this level's send rows (the next
 * party's level launch waits for them). A workgroup is one
 * ABY3G_HANDOFF_ROWS chunk of rows. Either may be NULL. */
int aby3g_bin_level_hs(const aby3g_gate* gates, const uint32_t* recv_rows, const uint32_t* batch_ends,
                       uint32_t nbatches, const uint64_t* recvbuf, const uint32_t* unpack_wires, uint32_t nunpack,
                       uint64_t* mem, uint64_t wires, uint64_t words, const uint64_t* z, uint64_t* sendbuf,
                       const aby3g_handoff* wait, const aby3g_handoff* post, aby3g_stream stream);
/* Residency of the hand-off level kernels on the current device, for the
 * host's in-kernel hand-off budget (a consumer's workgroups spin, so two
 * consumer launches must leave a producer workgroup a slot): CUs, and
 * workgroups of each hand-off instantiation resident per CU
 * (hipOccupancyMaxActiveBlocksPerMultiprocessor) -- the small-grid form
 * (launches of fewer than *small_max_wgs workgroups) and the large one. */
int aby3g_bin_level_residency(int* cus, int* per_cu_small, int* per_cu_large, int* small_max_wgs);
int aby3g_bin_unpack(const uint64_t* recvbuf, const uint32_t* out_wires, uint32_t n, uint64_t* mem, uint64_t wires,
                     uint64_t words, aby3g_stream stream);
/* setInput (:200-276): bit-transpose a [rows][cols64] i64 share matrix into
 * nbits consecutive wire rows starting at wire_rows (stride `words`),
 * zero padding rows >= rows. */
int aby3g_bits_to_wires(const int64_t* in, uint64_t rows, uint64_t cols64, uint32_t nbits, uint64_t* wire_rows,
                        uint64_t words, aby3g_stream stream);
/* getOutput (:1285-1404): transpose wire rows (wire ids in the DEVICE array
 * wires, row base = mem_share) back to [rows][ceil(nbits/64)] i64. */
int aby3g_wires_to_bits(const uint64_t* mem_share, const uint32_t* wires, uint32_t nbits, uint64_t words,
                        int64_t* out, uint64_t rows, aby3g_stream stream);
/* Both shares in one launch: `in` / `out` are [2][rows][cols] share pairs
 * (SharedMat layout); share s's wire rows start share_stride u64 after
 * share 0's (= wires * words for the engine memory). */
int aby3g_bits_to_wires2(const int64_t* in, uint64_t rows, uint64_t cols64, uint32_t nbits, uint64_t* wire_rows,
                         uint64_t share_stride, uint64_t words, aby3g_stream stream);
int aby3g_wires_to_bits2(const uint64_t* mem, uint64_t share_stride, const uint32_t* wires, uint32_t nbits,
                         uint64_t words, int64_t* out, uint64_t rows, aby3g_stream stream);

/* Row maps of the merge network's compare-exchange rounds (aby3-Basic
 * Sort.cpp:361-398 x_mask / y_mask and the gathers around
 * bool_cipher_max_min_split, :375-392; batched over merges as
 * high_dimensional_odd_even_merge, :506-570). Element p of a circuit input or
 * output is row map(p) of a row-major sbMatrix:
 *   idx != NULL : idx[first + p]                       (explicit, DEVICE array)
 *   otherwise   : q = first + p, rep = q / per_rep, k = q % per_rep,
 *                 start + rep * rep_stride + k * step  (affine)
 * The struct is passed by host pointer and copied into the launch. */
typedef struct {
    uint64_t first, start, step, per_rep, rep_stride;
    const uint32_t* idx;
} aby3g_rowmap;
/* setInput from mapped rows: circuit row p (p < rows) of both shares takes
 * row map(p) of `in` ([2][in_rows][cols64]); rows >= rows are zero. */
int aby3g_bits_to_wires_map(const int64_t* in, uint64_t in_rows, uint64_t cols64, uint32_t nbits,
                            const aby3g_rowmap* map, uint64_t rows, uint64_t* wire_rows, uint64_t share_stride,
                            uint64_t words, aby3g_stream stream);
/* getOutput into mapped rows: row map(p) of `out` ([2][out_rows][ceil(nbits/64)])
 * of both shares takes circuit row p, for p < rows; other rows of `out` are
 * untouched (the compare-exchange's scatter back into the merge array). */
int aby3g_wires_to_bits_map(const uint64_t* mem, uint64_t share_stride, const uint32_t* wires, uint32_t nbits,
                            uint64_t words, int64_t* out, uint64_t out_rows, const aby3g_rowmap* map, uint64_t rows,
                            aby3g_stream stream);
/* One or two mapped transposes in one launch (n <= 2): the two gathers of a
 * compare-exchange round's inputs (same source, maps[k] -> wire_rows[k]), or
 * its two scatters (wire lists wires[k] -> maps[k] rows of the same out, the
 * maps' target rows disjoint). Same semantics as n separate calls. */
int aby3g_bits_to_wires_map_n(const int64_t* in, uint64_t in_rows, uint64_t cols64, uint32_t nbits,
                              const aby3g_rowmap* maps, uint64_t* const* wire_rows, uint32_t n, uint64_t rows,
                              uint64_t share_stride, uint64_t words, aby3g_stream stream);
int aby3g_wires_to_bits_map_n(const uint64_t* mem, uint64_t share_stride, const uint32_t* const* wires,
                              uint32_t nbits, uint64_t words, int64_t* out, uint64_t out_rows,
                              const aby3g_rowmap* maps, uint32_t n, uint64_t rows, aby3g_stream stream);

/* setInput of shares that are linear combinations of arithmetic shares,
 * several inputs / shares in one launch (the two-input binary resharing of
 * fetch_msb and Sh3Piecewise::getInputRegions, BuildingBlocks.cpp:475-502,
 * Sh3Piecewise.cpp:392-470): source k writes nbits wire rows of the value
 * v[r] = sum_t coef[t] * term[t][r * cols64 + c] + constant (mod 2^64);
 * all terms NULL writes zero wires. copy_out (optional) receives
 * sum_t coef[t] * term[t][...] (without the constant), e.g. P0's share to
 * send. At most ABY3G_WIRE_SRC_MAX sources per call. */
#define ABY3G_WIRE_SRC_MAX 8
typedef struct {
    const int64_t* term[4];
    int64_t coef[4];
    int64_t constant;
    uint64_t cols64;
    uint32_t nbits;
    uint64_t* wire_rows;
    int64_t* copy_out;
} aby3g_wire_src;
int aby3g_bits_to_wires_lin(const aby3g_wire_src* srcs, uint32_t nsrc, uint64_t rows, uint64_t words,
                            aby3g_stream stream);
/* copy_out of each source only (sum_t coef[t] * term[t], rows x cols64):
 * the part of aby3g_bits_to_wires_lin a message needs before its level */
int aby3g_lin_copy_out(const aby3g_wire_src* srcs, uint32_t nsrc, uint64_t rows, aby3g_stream stream);
/* The first level of a circuit together with its inputs: setInput of
 * linear combinations (Sh3BinaryEvaluator.cpp:200-276) fused into the level
 * launch (:539-1196). Per 2048-row chunk, every source (one 64-bit input of
 * at most 64 wires and one share, cols64 == 1, no copy_out: call
 * aby3g_lin_copy_out first) is transposed into LDS, then the level's gate
 * batches read the input wires [in_lo, in_hi) (at most
 * ABY3G_LEVEL_IN_MAX_WIRES) from LDS and every other wire from mem. The
 * input wires reach mem only when write_inputs != 0 (a later level reads
 * them). Sources' wire_rows name their wires in mem as for
 * aby3g_bits_to_wires_lin; a source without terms is all zero and must have
 * constant 0 (rejected otherwise). post: the level's AND shares handed over
 * in-kernel (aby3g_handoff), or NULL. */
#define ABY3G_LEVEL_IN_MAX_WIRES 128
int aby3g_bin_level_in(const aby3g_wire_src* srcs, uint32_t nsrc, uint64_t rows, uint32_t in_lo, uint32_t in_hi,
                       int write_inputs, const aby3g_gate* gates, const uint32_t* batch_ends, uint32_t nbatches,
                       uint64_t* mem, uint64_t wires, uint64_t words, const uint64_t* z, uint64_t* sendbuf,
                       const aby3g_handoff* post, aby3g_stream stream);

/* ----------------------------------------- fused SGD_Logistic iteration -- */
/* One whole SGD_Logistic iteration (aby3-ML/Regression.h:249-293) of one
 * party in ONE launch, for three parties co-located on one device in one
 * process: extractBatch, mul(XX, w) with truncation (Sh3Evaluator.cpp:
 * 651-730), the piecewise sigmoid (Sh3Piecewise.cpp:184-567: the two-input
 * resharing, the int_Sh3Piecewise_helper circuit level by level, the OT
 * product and the public-constant product, Sh3Evaluator.cpp:119-263,
 * 418-501), err = f - YY, mulTruncate(XX^T, err, aB) and w -= update.
 * Every message goes through the parties' mailboxes as in-kernel hand-offs:
 * each 64-bit word as two write-through {epoch, 32-bit half} words that the
 * reader polls until both carry its epoch (no flags); the randomness is the
 * op-by-op path's, at the stream positions, draw indices and OT counters the
 * host passes, so the shares are bit-identical to that path's.
 *
 * The levelized circuit, as device arrays (host-built from the levelized
 * gate list; gates in batch order as for aby3g_bin_level). */
typedef struct {
    uint32_t first_gate;   /* index into gates of the level's first gate */
    uint32_t nbatch;       /* batches of mutually independent gates */
    uint32_t batch_off;    /* into batch_ends (relative to first_gate) */
    uint32_t nand;         /* AND-type gates = send rows of the level */
    uint32_t and_wire_off; /* into and_wires: the level's AND outputs in send-row order */
    uint32_t fused_first;  /* gates of the level from this index on have an ext entry (ext != NULL) */
    uint32_t ext_off;      /* into ext: the entry of gate fused_first */
    uint32_t pad;
} aby3g_lr_level;
/* Operands of a gate folded into its level's first batch: operand x is the
 * XOR of in0 and the wires x[0..2] (0xFFFF: none), inverted (both shares)
 * when flags bit 0 is set; y likewise with in1, y[] and bit 1 -- the local
 * XOR / NXOR / INV gates of the level's earlier batches substituted. */
typedef struct {
    uint16_t x[3], y[3];
    uint16_t flags, pad;
} aby3g_lr_gate_ext;
typedef struct {
    uint32_t nlevels, wires, nand, ngates;
    uint32_t in_wire[3];  /* first wires of the 64-bit inputs aa_0, aa_1, b */
    uint32_t out_wire[3]; /* the region outputs c_0, c_1, c_2 (1 bit each) */
    const aby3g_gate* gates;
    const uint32_t* batch_ends;
    const aby3g_lr_level* levels;
    const uint32_t* and_wires;
    const aby3g_lr_gate_ext* ext; /* optional (NULL: no folded gates) */
    uint32_t next;                /* entries of ext */
    uint32_t pad;
} aby3g_lr_circuit;

/* The positions of one iteration's randomness (the same-named fields of
 * aby3g_lr_iter): the next iteration's, for drawing it ahead. */
typedef struct {
    uint64_t t1_next_off, t1_prev_off, t2_next_off, t2_prev_off;
    uint8_t mask_prev[16], mask_next[16];
    uint64_t ot_prev_off, ot_next_off, ot_ctr, pm_ctr_next, pm_ctr_prev, pm_draw;
} aby3g_lr_rand;

/* Arguments of one iteration of one party. Mailboxes: aby3g_lr_mailbox_bytes
 * each, zeroed before the first iteration; a party writes only its own and
 * reads its neighbours' (next = party + 1, prev = party + 2 mod 3) -- in
 * this process, or mapped from another process (aby3g_ipc_open). epoch:
 * 1 for the first iteration, +1 per iteration, the same for the three.
 * sys_scope: 0 when the three mailboxes are on this device (agent-scope
 * messages), 1 when a neighbour's is on another GPU (system scope; every
 * mailbox then from aby3g_malloc_uncached). */
/* phase_ticks slots: 0-15 phases, 16 + lv end of circuit level lv (lv < 16),
 * 32 + 4 lv + b / 64 + 4 lv + b batch b of level lv (lv < 8, b < 4),
 * 96 + lv level lv - 1's AND shares received (1 <= lv < 16) */
#define ABY3G_LR_PHASE_SLOTS 112
typedef struct {
    int32_t party;
    uint32_t B, d, D, aB;
    uint64_t n;              /* dataset rows */
    const int64_t* X;        /* [2][n][d] */
    const int64_t* Y;        /* [2][n][1] */
    int64_t* w;              /* [2][d][1], updated in place */
    const uint32_t* batch;   /* B row ids (getSubset) */
    aby3g_lr_circuit cir;    /* int_Sh3Piecewise_helper(64, 2) */
    void* scratch;           /* aby3g_lr_scratch_bytes */
    void* mailbox;
    const void* next_mailbox;
    const void* prev_mailbox;
    uint64_t epoch;
    uint32_t sys_scope;
    uint64_t* wait_ticks;    /* optional: in-kernel wait (100 MHz ticks) added here */
    uint64_t* phase_ticks;   /* optional: [ABY3G_LR_PHASE_SLOTS] wall-clock stamps of the phases (profiling) */
    /* the evaluator's ShareGen streams (seeds) and zero-share keys */
    uint8_t prev_seed[16], next_seed[16];
    uint8_t zs_prev[16], zs_next[16];
    uint64_t t1_next_off, t1_prev_off;  /* mul(XX, w): truncation pair stream positions (bytes) */
    uint64_t t2_next_off, t2_prev_off;  /* mulTruncate(XX^T, err): ditto */
    uint8_t mask_prev[16], mask_next[16];  /* setCir keys of the circuit (getPrevBlock / getNextBlock) */
    uint64_t ot_prev_off, ot_next_off;  /* the OT product's stream positions (bytes; per party) */
    uint8_t ot_next_key[16], ot_prev_key[16];
    uint64_t ot_ctr;                    /* the OT product's SharedOT counter (P0: next, P2: prev) */
    uint64_t pm_ctr_next, pm_ctr_prev;  /* the public product's counters (P0 both; P1 next; P2 prev) */
    uint64_t pm_draw;                   /* the public product's first zero-share draw */
    int64_t thr_off[2];                 /* circuit input offsets -t_0, -t_1 (fixed point) */
    int64_t half;                       /* region 1: half + slope * x */
    int64_t slope;
    int64_t one;                        /* region 2: the public constant */
    /* Randomness drawn ahead (none of it depends on data): pre_have != 0 --
     * the previous launch with this scratch drew this iteration's (the
     * positions above) into scratch slot epoch & 1, so the protocol
     * workgroup only reads it; pre_next != 0 -- the helper workgroups draw
     * the next iteration's (next_rand) into slot (epoch + 1) & 1 while this
     * one runs. */
    uint32_t pre_have, pre_next;
    aby3g_lr_rand next_rand;
    /* optional: the next iteration's batch (B row ids). The helpers touch its
     * dataset rows after their last product, so that the next launch's
     * helpers (the same workgroup ids, so the same XCDs) find them in L2. */
    const uint32_t* next_batch;
} aby3g_lr_iter;
uint64_t aby3g_lr_mailbox_bytes(uint32_t B, uint32_t d, const aby3g_lr_circuit* cir);
uint64_t aby3g_lr_scratch_bytes(uint32_t B, uint32_t d, const aby3g_lr_circuit* cir);
/* ABY3G_EINVAL for shapes the fused form does not take (B > 2048, d > 4096). */
int aby3g_lr_iteration(const aby3g_lr_iter* it, aby3g_stream stream);

/* ------------------------------------------------ element-wise helpers -- */
/* out[i] = ca*a[i] + cb*b[i] + c (mod 2^64); b may be NULL. Covers share
 * sums/differences (BuildingBlocks.cpp:475-480, Sh3Piecewise.cpp:403-470,
 * :543-563), fixed-point constants and output accumulation. */
int aby3g_i64_lincomb(uint64_t n, int64_t ca, const int64_t* a, int64_t cb, const int64_t* b, int64_t c, int64_t* out,
                      aby3g_stream stream);
/* Bitwise ops on u64 vectors: 0 xor, 1 and, 2 not(a), 3 lsb-to-mask (-(a&1)),
 * 4 copy. b may be NULL for unary ops. */
int aby3g_u64_bitop(int op, uint64_t n, const uint64_t* a, const uint64_t* b, uint64_t* out, aby3g_stream stream);
/* Row gather of a [2][rows][cols] share matrix: dst[s][i][:] = src[s][idx[i]][:]
 * (extractBatch, aby3-ML/Regression.h:42-58); dst is [2][n][cols]. */
int aby3g_i64_gather_rows(const int64_t* src, uint64_t rows, uint64_t cols, const uint32_t* idx, uint64_t n,
                          int64_t* dst, aby3g_stream stream);
/* Transpose of both shares: dst[s] = src[s]^T, src [2][rows][cols] -> dst [2][cols][rows]
 * (sMatrix::transpose / transposeInPlace, Sh3Types.h:198-271). */
int aby3g_i64_transpose(const int64_t* src, uint64_t rows, uint64_t cols, int64_t* dst, aby3g_stream stream);
/* dst[i] = src[idx[i]] (gather) and dst[idx[i]] = src[i] (scatter), u64. */
int aby3g_u64_gather(uint64_t n, const uint32_t* idx, const uint64_t* src, uint64_t* dst, aby3g_stream stream);
int aby3g_u64_scatter(uint64_t n, const uint32_t* idx, const uint64_t* src, uint64_t* dst, aby3g_stream stream);
/* One step of the 3-party shuffle (aby3-Basic/Shuffle.cpp): `units` units of
 * `unit` u64 words, out[i] = a[g] ^ b[g] ^ c[g] ^ mask with g = idx[i] (idx
 * NULL: g = i; any of a, b, c, mask NULL: omitted; mask is one unit, the
 * same for every unit, as get_random_mask draws it for a vector of units).
 * A permutation that scatters (tmp[p[i]] = data[i], Basics.h:324-332) is
 * applied as the gather of its inverse. */
int aby3g_u64_xor_gather_units(uint64_t units, uint64_t unit, const uint32_t* idx, const uint64_t* a,
                               const uint64_t* b, const uint64_t* c, const uint64_t* mask, uint64_t* out,
                               aby3g_stream stream);

#ifdef __cplusplus
}
#endif
#endif /* ABY3GPU_H */
