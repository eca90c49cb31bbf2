// aby3-Basic merge network (aby3-Basic/Sort.cpp:327-628) on the GPU engine.
//
// Every compare-exchange of one network round -- over every merge that runs
// in that round -- is ONE cmp_swap circuit evaluation (Circuit.cpp cmp_swap:
// outputs (min, max)), chunked at MAX_SENDING_SIZE rows as
// high_dimensional_odd_even_merge (:506-570). The gather of the round's
// pairs is fused into the circuit's input transposes and the scatter back
// into its output transposes (aby3g_bits_to_wires_map /
// aby3g_wires_to_bits_map), so a round is: z-mask draw, two gather
// transposes, the circuit's levels, two scatter transposes.
//
// Round schedule per merge of lists of lengths (L1, L2), length = max(L1, L2)
// (Sort.cpp:361-398): the lists are interleaved into 2 * length slots (list 1
// at even, list 2 at odd slots, missing slots padded with max(last1, last2));
// round 0 compares slots (i, i + 1) for even i; with t = ceil(log2(length) + 1)
// and q = 2^(t-1), the following rounds use d = q - 1, q >>= 1, r = 1,
// comparing (i, i + d) for i = r, r + 2, ... < 2 * length - d, until d = 0. The
// first L1 + L2 slots are the merged list.
//
// Batched semantics (the restatement tests/ and oracle/ follow): a batch of
// merges runs its rounds together; round j evaluates the pairs of every merge
// that has a round j, merge-major then pair order (the reference's
// x_mask_mat row order i * unit_mask_len + j, Sort.cpp:514-519). The padding
// maxima are one cmp_swap evaluation over the batch's merges (rows = merges),
// taken only when some merge has L1 != L2 (with equal lengths no slot is
// padding). Where the reference runs bool_cipher_max_min_split as three
// circuits (lt, then two ANDs, BoolBasic.cpp:275-312), this engine evaluates
// the single fused cmp_swap circuit: same revealed result, its own
// randomness consumption (16 bytes of each stream per evaluation).
#pragma once
#include "Sh3BinaryEvaluator.h"
#include "Sh3Evaluator.h"

namespace aby3 {

// Rows per circuit evaluation (Sort.cpp:4)
constexpr u64 kMaxSendingSize = 1ull << 25;

// The reference's round schedule for lists of `length` (Sort.cpp:361-398):
// (d, r) per round.
std::vector<std::pair<u64, u64>> mergeSchedule(u64 length);

// One merge of a batch: lists [offA, offA + lenA) and [offA + lenA, + lenB)
// of the merge array (adjacent), merged in place into [offA, offA + lenA + lenB).
struct MergeSpec {
    u64 offA, lenA, lenB;
};
// Rows of each cmp_swap evaluation a batch / a multi-merge runs (chunks of
// kMaxSendingSize counted separately): the work accounting of bench jobs.
std::vector<u64> mergeBatchEvalRows(const std::vector<MergeSpec>& merges);
std::vector<u64> multiMergeEvalRows(std::vector<u64> lens, bool sequential = false);
// Run a batch of merges over the 64-bit sbMatrix `data` (one word per row).
void mergeBatch(sbMatrix& data, const std::vector<MergeSpec>& merges, int pIdx, Sh3Evaluator& eval,
                Sh3Runtime& runtime);

// Sort.cpp:327-406: merge two sorted arrays
int odd_even_merge(const sbMatrix& data1, const sbMatrix& data2, sbMatrix& res, int pIdx, Sh3Evaluator& eval,
                   Sh3Runtime& runtime);
// How a level of odd_even_multi_merge runs its pairwise merges: Batched
// (default) as one batch, every round of the level one cmp_swap evaluation
// over all of its merges; Sequential one merge after the other, as the
// reference's loop calls odd_even_merge (Sort.cpp:423-429) -- the same
// revealed result, and the reference's own order of randomness draws (so the
// reference's shares), at one evaluation per merge and round.
enum class MergeOrder { Batched, Sequential };
// Sort.cpp:413-437: merge k sorted arrays pairwise, level by level (odd k:
// the last two first).
int odd_even_multi_merge(std::vector<sbMatrix>& data, sbMatrix& sorted, int pIdx, Sh3Evaluator& eval,
                         Sh3Runtime& runtime, MergeOrder order = MergeOrder::Batched);
// The same over one array holding the lists back to back (list k has lens[k]
// rows): no per-list allocations, for many lists.
int odd_even_multi_merge(const sbMatrix& flat, const std::vector<u64>& lens, sbMatrix& sorted, int pIdx,
                         Sh3Evaluator& eval, Sh3Runtime& runtime, MergeOrder order = MergeOrder::Batched);
// Odd-even merge sort of `keys` (one 64-bit key per row): multi-merge of the
// keys as singleton lists (the C5 workload).
int odd_even_merge_sort(const sbMatrix& keys, sbMatrix& sorted, int pIdx, Sh3Evaluator& eval, Sh3Runtime& runtime);
// Sort.cpp:439-583: dim independent merges data1[i] with data2[i] as one batch
int high_dimensional_odd_even_merge(std::vector<sbMatrix>& data1, std::vector<sbMatrix>& data2,
                                    std::vector<sbMatrix>& sorted, int pIdx, Sh3Evaluator& eval, Sh3Runtime& runtime);
// Sort.cpp:585-628: data[dim][k] -> sorted[dim]; every level's merges over all
// pairs and dimensions form one batch (pair-major, then dimension).
int high_dimensional_odd_even_multi_merge(std::vector<std::vector<sbMatrix>>& data, std::vector<sbMatrix>& sorted,
                                          int pIdx, Sh3Evaluator& eval, Sh3Runtime& runtime,
                                          MergeOrder order = MergeOrder::Batched);

}  // namespace aby3
