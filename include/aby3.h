/*
 * aby3.h -- C entry points of the host runtime (aby3_amd/lib/libaby3.so),
 * for drivers that are not C++ (bench.py, the Python tests, a cgo/ctypes
 * binding). The C++ API itself is the headers under aby3_amd/host/ (namespace aby3),
 * mirroring the reference's Sh3Runtime / Sh3Encryptor / Sh3Evaluator /
 * Sh3BinaryEvaluator / Sh3Piecewise classes.
 *
 * A session runs the three ABY3 parties as three persistent host threads of
 * this process, each with its own Sh3Runtime, HIP stream and device (party i
 * on devices[i]; all three may share one GPU), connected by in-process
 * device channels. aby3h_session_run(s, k) executes k protocol steps of the
 * session's job on all parties and returns when every party's stream has
 * drained, so the caller can bracket exactly k steps with its own clock.
 */
#ifndef ABY3_H
#define ABY3_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct aby3h_session aby3h_session;

enum {
    /* params: M, K, N, D, mode (1 GEMM, 0 Hadamard)[, inflight]. One step = one
     * Sh3Evaluator::asyncMul(A, B, C, D) with truncation (Sh3Evaluator.cpp:651-730).
     * inflight 2: step s issues product s (into one of two output matrices)
     * and then waits for product s - 1, so the runtime holds two independent
     * products; the run's last one completes when the run ends.
     * [, shard, shards] (GEMM only): this session runs rows [shard * M / shards,
     * (shard + 1) * M / shards) of the product -- A's slice shared by
     * localIntMatrixRows, the product by Sh3Evaluator::asyncMulRows -- so the
     * result holds those rows of the unsplit job's shares (one party's rows
     * split over `shards` GPUs, each GPU with its own three-party session). */
    ABY3H_JOB_MUL_TRUNC = 0,
    /* params: M, K, N, mode. One step = asyncMul without truncation (:92-116). */
    ABY3H_JOB_MUL = 1,
    /* params: rows[, shard, shards]. One step = cipher_gt / fetch_msb over
     * `rows` 64-bit values: reshare + MSB(a+b) circuit (BuildingBlocks.cpp:
     * 464-532). shard k of `shards`: rows [e(k), e(k+1)) with e(k) = rows * k /
     * shards rounded down to a multiple of 2048 (e(shards) = rows), by
     * cipher_gt_rows: those rows of the unsplit job's shares. */
    ABY3H_JOB_MSB = 2,
    /* params: rows (dataset), dim, batch, D, lr_log2[, sample]. One step = one
     * SGD_Logistic iteration (aby3-ML/Regression.h:249-293): xw = X_B w,
     * sigmoid (Sh3Piecewise), err = f - Y_B, w -= X_B^T err >> (D + aB).
     * sample 0 (default): the first 8192 mini-batches are drawn at setup and
     * kept in HBM; 1: each step draws its batch with getSubset
     * (DeviceBatchSampler, the pool resident in HBM) inside the step. */
    ABY3H_JOB_LR = 3,
    /* params: keys, order. One step = odd_even_merge_sort of `keys` 64-bit
     * keys (distinct, (U[0, 2^43) << 20) | i): the multi-merge of singleton
     * lists (Sort.cpp:413-628). order 0 (default): batched, every round of
     * every level one cmp_swap evaluation; 1: sequential, the reference's
     * loop of one odd_even_merge after another (Sort.cpp:423-429), so the
     * reference's order of randomness draws and shares (MergeOrder). */
    ABY3H_JOB_SORT = 4,
    /* params: rows. One step = Sh3Converter::toBinaryMatrix of rows x 1
     * 64-bit values (resharing + 64-bit adder, Sh3Converter.cpp:61-207). */
    ABY3H_JOB_A2B = 5,
    /* params: rows, bits (<= 64). One step = Sh3Converter::bitInjection of
     * a rows x bits binary matrix (3-party OT per bit, :209-370). */
    ABY3H_JOB_BITINJ = 6
};

/* info slots returned by aby3h_session_info */
enum {
    ABY3H_INFO_MULTS_PER_STEP = 0,    /* secret-shared 64-bit mults per step (metric unit) */
    ABY3H_INFO_GEMM_INT8_OPS = 1,     /* int8 MFMA ops per GEMM launch (144 M N K) */
    ABY3H_INFO_AND_WORDS = 2,         /* AND-type gates x 64-row words per step */
    ABY3H_INFO_GATE_WORDS = 3,        /* all gates x words per step */
    ABY3H_INFO_GATE_BYTES = 4,        /* algorithmic HBM bytes of the gate kernels per step */
    ABY3H_INFO_BYTES_SENT = 5,        /* bytes sent by party 0 per step */
    ABY3H_INFO_HOST_ENQUEUE_US = 6,   /* last run: host time per step issuing work, max over parties */
    ABY3H_INFO_HOST_DRAIN_US = 7,     /* last run: host wait for the streams to drain after the last step */
    ABY3H_INFO_HOST_RECV_WAIT_US = 8, /* last run: host time per step waiting for peers' messages (party 0) */
    ABY3H_INFO_HOST_API_US = 9,       /* last run: host time per step inside aby3g_* calls (party 0) */
    ABY3H_INFO_HOST_API_CALLS = 10,   /* last run: aby3g_* calls per step (party 0) */
    ABY3H_INFO_DEVICE_WAIT_US = 11,   /* last run: in-kernel wait for peers per step and party (us, mean of the local parties) */
    ABY3H_INFO_LR_FUSED = 12,         /* JOB_LR: 1 when the iterations ran as the fused launch (aby3g_lr_iteration) */
    ABY3H_INFO_LR_SYS_SCOPE = 13,     /* JOB_LR: 1 when that launch's messages were system-scope (uncached mailboxes) */
    ABY3H_INFO_COUNT = 14
};

const char* aby3h_last_error(void);

/* probe: 0 off, else a bitmask of aby3gpu.h probe families (1 << family) whose
 * launches are bracketed by timing events */
aby3h_session* aby3h_session_create(int job, const uint64_t* params, int nparams, const int* devices, int probe);
/* One party of a session in this process: the reference's deployment of
 * three processes, one per party (Eval/dis_exec.sh:10-12), here one GPU per
 * party. The three processes call this with the same job,
 * params and `link` (a session name unique on the machine, no '/'), each with
 * its own party 0..2 and device; the call returns once the session is set up
 * in all three. The parties' messages travel over shared-memory links (host
 * control words) and IPC-exported device staging slots (payloads; peer reads
 * over xGMI between GPUs). colocated: 0 = the parties run on different GPUs;
 * 1 = other parties share this party's GPU (one stream per party, in-kernel
 * hand-offs through IPC-mapped arenas); 2 = they share it, but every
 * cross-GPU branch is taken as if they did not (staged copies for every
 * device message, the fused LR iteration's uncached mailboxes and
 * system-scope messages) -- the north-star layout's code on one GPU. Every aby3h_session_* call below must then be
 * made by all three processes in the same order; info and probe report this
 * process's party, check reports party 0's verdict in party 0's process (the
 * others return 0 when their part succeeded). */
aby3h_session* aby3h_party_create(int job, const uint64_t* params, int nparams, int party, int device,
                                  const char* link, int colocated, int probe);
int aby3h_session_run(aby3h_session* s, uint64_t steps);
/* kernel time (ms) and launches of a probe family (aby3gpu.h), summed over parties */
int aby3h_session_probe(aby3h_session* s, int family, double* ms, uint64_t* launches);
int aby3h_session_probe_reset(aby3h_session* s);
int aby3h_session_info(aby3h_session* s, double* out, int n);
/* FNV-1a digest of party `party`'s two shares of the last step's result (a
 * party this session runs): share-level comparisons between layouts, e.g. one
 * party per process against three in one process on the same seeds. */
int aby3h_session_digest(aby3h_session* s, int party, uint64_t* out);
/* Party `party`'s share `share` (0 or 1) of the last step's result: copies
 * min(count, elements) int64 values (row-major) into out and stores the
 * result's element count in *elements. Between runs only. */
int aby3h_session_result(aby3h_session* s, int party, int share, int64_t* out, uint64_t count, uint64_t* elements);
/* reveals the last step's result and checks it against plaintext; 0 = ok */
int aby3h_session_check(aby3h_session* s);
void aby3h_session_destroy(aby3h_session* s);

/* A library circuit, levelized, as flat arrays (for CPU tests and external
 * evaluators). name: "int_comp_helper", "int_int_lt", "int_eq", "int_int_add",
 * "int_int_sub", "int_int_bitwiseAnd", "int_int_bitwiseOr", "bits_nor_helper",
 * "cmp_swap", "int_Sh3Piecewise_helper" (param = thresholds).
 * Call with NULL buffers to get the sizes (counts[0..5] = wires, gates,
 * levels, input bundles, output bundles, total bundle wires); gates are
 * 4 x u32 {in0, in1, out, type} in evaluation order. */
int aby3h_circuit(const char* name, uint64_t size, uint64_t param, uint64_t counts[6], uint32_t* gates,
                  uint32_t* level_counts, uint32_t* in_sizes, uint32_t* in_wires, uint32_t* out_sizes,
                  uint32_t* out_wires);

/* Writes a library circuit to `path` in the BetaCircuit binary format
 * (BetaCircuit::writeBin, aby3_amd/host/Circuit.h). Any circuit name above
 * also accepts "bin:<path>": the circuit stored in that file (readBin,
 * levelized on load), so externally built circuits run on the engine. */
int aby3h_circuit_write(const char* name, uint64_t size, uint64_t param, const char* path);

/* ---- one protocol call by three in-process parties ---------------------
 * The topology and seeds of the reference's unit tests
 * (Sh3EvaluatorTests.cpp:23-131): encryptor seeds toBlock(0, i) /
 * toBlock(0, i+1), evaluator seeds toBlock(1, i) / toBlock(1, i+1), all on
 * `device`; party 0 shares the inputs (Sh3Encryptor::localIntMatrix /
 * localBinMatrix, inputs shared in argument order). out_shares receives
 * every party's two shares as [party][share][n] i64 (n = result elements),
 * out_plain the result revealed by revealAll. Any output pointer may be
 * NULL. Returns 0, or 1 with aby3h_sim_last_error() set. */
const char* aby3h_sim_last_error(void);
/* asyncMul(A, B, C [, d]) (Sh3Evaluator.cpp:92-116, :651-730); mode 1 GEMM
 * (a M x K, b K x N), 0 Hadamard (a, b M x K) */
int aby3h_sim_mul(int device, int mode, int trunc, uint64_t d, const int64_t* a, const int64_t* b, uint64_t M,
                  uint64_t K, uint64_t N, int64_t* out_shares, int64_t* out_plain);
/* kind 0: asyncMul(si64 a, sb bits) (:119-263); 1: asyncMul(i64 apub, sb bits) (:418-501); bits shared first */
int aby3h_sim_mul_bit(int device, int kind, const int64_t* a, int64_t apub, const int64_t* bits, uint64_t n,
                      int64_t* out_shares, int64_t* out_plain);
/* a library circuit (aby3h_circuit names) on binary-shared inputs: ins is
 * [input bundle][rows][ceil(bits/64)] i64; outs / out_shares the same per output bundle */
int aby3h_sim_circuit(int device, const char* name, uint64_t size, uint64_t param, uint64_t rows, const int64_t* ins,
                      int64_t* outs, int64_t* out_shares);
/* Sh3Piecewise::eval on an n x 1 shared input (Sh3Piecewise.cpp:184-378):
 * kind 0 the logistic sigmoid of aby3ML.h:121-139, kind 1 ReLU */
int aby3h_sim_piecewise(int device, int kind, const int64_t* x, uint64_t n, uint64_t D, int64_t* out_shares,
                        int64_t* out_plain);
/* cipher_gt(A, B) = MSB(B - A) (BuildingBlocks.cpp:525-532), 1-bit result */
int aby3h_sim_cipher_gt(int device, const int64_t* a, const int64_t* b, uint64_t n, int64_t* out_plain,
                        int64_t* out_shares);
/* The merge network (Sort.cpp:327-628, batched as aby3_amd/host/Sort.h) on
 * nlists sorted lists of 64-bit keys (concatenated in `keys`):
 * mode 0 odd_even_multi_merge(vector<sbMatrix>), each list shared on its own;
 * mode 1 the flat odd_even_multi_merge, all keys shared as one matrix
 *        (all lists of length 1: odd_even_merge_sort);
 * mode 2 high_dimensional_odd_even_multi_merge, lists [dim][nlists / dim];
 * mode 3 high_dimensional_odd_even_merge (nlists = 2 * dim);
 * mode 4 / 5 mode 0 / 2 in the reference's sequential merge order (MergeOrder).
 * out_sorted: the revealed merged list(s) back to back; out_shares
 * [party][share][total] of the same (either may be NULL). */
int aby3h_sim_merge(int device, int mode, const uint64_t* lens, uint64_t nlists, uint64_t dim, const int64_t* keys,
                    int64_t* out_sorted, int64_t* out_shares);
/* The 3-party shuffle (aby3-Basic/Shuffle.cpp, aby3_amd/host/Shuffle.h) of
 * x [len][unit] (binary-shared by party 0 as one matrix): mode 0
 * efficient_shuffle(vector<sbMatrix>, one unit per matrix), 1
 * efficient_shuffle(sbMatrix) (unit 1), 2 efficient_shuffle_with_random_
 * permutation (out_pi_shares [party][share][len]: the applied permutation),
 * 3 the packed form efficient_shuffle_units (same result as mode 0).
 * out_shares [party][share][len*unit], out_plain the revealed units. */
int aby3h_sim_shuffle(int device, int mode, const int64_t* x, uint64_t len, uint64_t unit, int64_t* out_shares,
                      int64_t* out_pi_shares, int64_t* out_plain);
/* `iters` SGD_Logistic iterations (aby3-ML/Regression.h:249-293) by three
 * parties seeded as aby3ML::init (aby3ML.cpp:4-17): party 0 shares X [n][d],
 * Y [n] (fixed point D) and w = 0 [d], iteration t uses the B row indices
 * batches[t * B ...]. out_w_shares [party][share][d], out_w_plain [d]. */
int aby3h_sim_lr(int device, uint64_t n, uint64_t d, uint64_t B, uint64_t D, uint64_t aB, uint64_t iters,
                 const int64_t* X, const int64_t* Y, const uint64_t* batches, int64_t* out_w_shares,
                 int64_t* out_w_plain);

/* The C4 driver's host side (CPU only, no GPU): the LogisticModelGen dataset
 * of main-logistic.cpp:82-100 in fixed point D (X [n][dim], Y [n], the model
 * [dim]; NULL outputs skipped) and getSubset's first `iters` mini-batches of
 * B rows over n (Regression.h:24-40), out [iters][B]. */
int aby3h_lr_dataset(uint64_t n, uint64_t dim, uint64_t D, int64_t* X, int64_t* Y, double* model);
int aby3h_lr_batches(uint64_t n, uint64_t B, uint64_t iters, uint64_t* out);

#ifdef __cplusplus
}
#endif
#endif /* ABY3_H */
