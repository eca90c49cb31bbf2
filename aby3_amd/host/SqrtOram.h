// The square-root ORAM of aby3-Basic (SqrtOram.h, on the base classes of
// Oram/include/oram.h) over the GPU engine. Its bookkeeping -- indices, flags,
// the stash -- is host-held replicated shares exactly as in the reference
// (boolShare / boolIndex are pairs of share values there too); every
// comparison, AND / OR and dot product runs as a binary circuit on the device
// (int_eq, int_int_bitwiseAnd / Or through evalCircuit), and the memory is
// shuffled by efficient_shuffle_with_random_permutation (Shuffle.h).
//
// An access is round-latency bound (a handful of tiny circuits per level of
// the position map); the engine adds nothing to the reference's protocol.
// Revealed results are pinned by the reference's pos_map_test and
// sqrt_oram_test (aby3_tests/Test.cpp:771-981).
#pragma once
#include "Shuffle.h"

namespace aby3 {

constexpr u64 BITSIZE = 64;  // Basics.h:16

// Basics.h:28-97
struct boolShare {
    bool bshares[2] = {false, false};
    boolShare() = default;
    boolShare(bool s0, bool s1) : bshares{s0, s1} {}
    boolShare(bool plain, int pIdx);  // party 1 holds it in share 0, party 2 in share 1
};
// Basics.h:100-153
struct boolIndex {
    i64 indexShares[2] = {0, 0};
    boolIndex() = default;
    boolIndex(i64 s0, i64 s1) : indexShares{s0, s1} {}
    boolIndex(i64 plain, int pIdx);
};

// BoolBasic.cpp:64-100: A == public B, row-wise (1-bit result)
void bool_cipher_eq(int pIdx, const sbMatrix& A, const i64Matrix& plainB, sbMatrix& res, Sh3Evaluator& eval,
                    Sh3Runtime& runtime);
// BoolBasic.cpp:124-139 (local AND of the shares, reshared to next)
void bool_cipher_or(int pIdx, const boolShare& A, const boolShare& B, boolShare& res, Sh3Runtime& runtime);
void bool_cipher_not(int pIdx, const boolShare& A, boolShare& res);  // :373-391
void bool_init_false(int pIdx, boolShare& res);                      // :692-709
// BoolBasic.cpp:393-423: XOR over the rows of A AND B (one row out)
void bool_cipher_dot(int pIdx, const sbMatrix& A, const sbMatrix& B, sbMatrix& res, Sh3Evaluator& eval,
                     Sh3Runtime& runtime);
// BoolBasic.cpp:463-515: XOR over i of A[i] AND B[i] (B: one row per unit,
// a 1-bit B first expanded to all-ones masks)
void bool_cipher_dot(int pIdx, const std::vector<sbMatrix>& A, const sbMatrix& B, sbMatrix& res, Sh3Evaluator& eval,
                     Sh3Runtime& runtime);
// BoolBasic.cpp:425-461: flag ? trueVal : falseVal (64-bit rows)
void bool_cipher_selector(int pIdx, const boolShare& flag, const sbMatrix& trueVal, const sbMatrix& falseVal,
                          sbMatrix& res, Sh3Evaluator& eval, Sh3Runtime& runtime);
// BoolBasic.cpp:596-640: one-hot mask of the first false entry (log-depth OR prefix)
void bool_get_first_zero_mask(int pIdx, const std::vector<boolShare>& A, sbMatrix& res, Sh3Evaluator& eval,
                              Sh3Runtime& runtime);
// BoolBasic.cpp:772-783: (A >> k, A & (2^k - 1)) share-wise
void bool_shift_and_left(int pIdx, const boolIndex& A, u64 k, boolIndex& shifted, boolIndex& left);
// BoolBasic.cpp:895-903: open a shared index to every party
i64 back2plain(int pIdx, const boolIndex& x, Sh3Runtime& runtime);

// oram.h PackedIndex + SqrtOram.h:17-57
struct ABY3PackedIndex {
    u64 pack = 0;
    std::vector<boolIndex> packedIndices;
    boolIndex logicalIndex;
};

// SqrtOram.h:60-387 (PosMap, oram.h:89-160): the position map, linear below
// S packed entries, else a packed map over a recursive sub-map.
class ABY3PosMap {
public:
    ABY3PosMap(u64 n, u64 pack, u64 S, const std::vector<boolIndex>& permutation, int pIdx, Sh3Encryptor& enc,
               Sh3Evaluator& eval, Sh3Runtime& runtime);
    // the physical index of logical `index` (opened to every party)
    i64 access(const boolIndex& index, const boolShare& fake);
    bool linear() const { return mLinear; }

    // the state is public, as the reference's members are (read by the
    // share-level parity test, tests/cpp/test_oram.cpp)
    u64 n, pack, S, t = 0, map_len;
    std::vector<boolIndex> permutation;      // linear map
    std::vector<boolShare> usage_map;        // linear map
    std::vector<ABY3PackedIndex> packed_index, stash;
    std::unique_ptr<ABY3PosMap> subPosMap;
    boolIndex last_physical_index;  // the last access's physical index, before back2plain opens it

private:
    void linear_ram(const std::vector<sbMatrix>& data, const boolIndex& index, sbMatrix& res);
    bool mLinear;
    int pIdx;
    Sh3Encryptor* enc;
    Sh3Evaluator* eval;
    Sh3Runtime* runtime;
};

// SqrtOram.h:389-450 (SqrtOram, oram.h:203-275)
class ABY3SqrtOram {
public:
    ABY3SqrtOram(int n, int S, int pack, int pIdx, Sh3Encryptor& enc, Sh3Evaluator& eval, Sh3Runtime& runtime);
    // shuffles `data` into the ORAM memory and builds the position map
    void initiate(std::vector<sbMatrix>& data);
    sbMatrix access(const boolIndex& index);

    int n, S, pack, t = 0;
    std::vector<sbMatrix> shuffle_mem;
    std::unique_ptr<ABY3PosMap> posMap;

private:
    struct StashElement {
        sbMatrix data;
        boolIndex logicalIndex;
    };
    std::vector<StashElement> stash;
    int pIdx;
    Sh3Encryptor* enc;
    Sh3Evaluator* eval;
    Sh3Runtime* runtime;
};

}  // namespace aby3
