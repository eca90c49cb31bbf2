// aby3-Basic building blocks on the GPU engine (aby3-Basic/BuildingBlocks.cpp,
// BoolBasic.cpp, Sort.cpp). Same synchronous call style as the reference
// (each call runs its protocol to completion with .get()).
#pragma once
#include "Sh3BinaryEvaluator.h"
#include "Sh3Encryptor.h"
#include "Sh3Evaluator.h"
#include "Sort.h"

namespace aby3 {

// ---- arithmetic -> comparison (BuildingBlocks.cpp:464-742)
// res = MSB(diff): P0 reshares x0 + x2 (not randomized, as the reference),
// P1/P2 expose x1, then the MSB(a + b) circuit.
int fetch_msb(int pIdx, const si64Matrix& diffAB, sbMatrix& res, Sh3Evaluator& eval, Sh3Runtime& runtime);
// [A > B] = MSB(B - A)   (:525-532)
int cipher_gt(int pIdx, const si64Matrix& A, const si64Matrix& B, sbMatrix& res, Sh3Evaluator& eval,
              Sh3Runtime& runtime);
// cipher_gt for rows [rowOffset, rowOffset + A.rows()) of a totalRows-row
// comparison (A, B hold those rows): the circuit's masks are those rows'
// words (Sh3BinaryEvaluator::setCirRows), so res holds those rows of the
// unsplit comparison's shares -- one party's rows split over GPUs (SURVEY.md
// §8e). rowOffset is a multiple of 2048, A.rows() too unless the slice ends
// at totalRows.
int cipher_gt_rows(int pIdx, const si64Matrix& A, const si64Matrix& B, sbMatrix& res, Sh3Evaluator& eval,
                   Sh3Runtime& runtime, u64 rowOffset, u64 totalRows);
// [A >= B] = !MSB(A - B) (:593-602)
int cipher_ge(int pIdx, const si64Matrix& A, const si64Matrix& B, sbMatrix& res, Sh3Evaluator& eval,
              Sh3Runtime& runtime);
// [A == B] via the equality circuit on (-(x0 + x2), x1) (:698-742)
int circuit_cipher_eq(int pIdx, const si64Matrix& A, const si64Matrix& B, sbMatrix& res, Sh3Evaluator& eval,
                      Sh3Runtime& runtime);
// Hadamard product, the fork's cipher_mul (:398-404)
int cipher_mul(int pIdx, const si64Matrix& A, const si64Matrix& B, si64Matrix& res, Sh3Evaluator& eval,
               Sh3Runtime& runtime);
// a * b for a shared bit b (:334-391 / asyncMul(si64, sb))
int cipher_mul(int pIdx, const si64Matrix& A, const sbMatrix& B, si64Matrix& res, Sh3Evaluator& eval,
               Sh3Runtime& runtime);

// ---- boolean (BoolBasic.cpp:20-391)
// revealed semantics pinned by BoolTest.cpp:122: bool_cipher_lt(A, B) = [A < B]
void bool_cipher_lt(int pIdx, const sbMatrix& A, const sbMatrix& B, sbMatrix& res, Sh3Evaluator& eval,
                    Sh3Runtime& runtime);
void bool_cipher_eq(int pIdx, const sbMatrix& A, const sbMatrix& B, sbMatrix& res, Sh3Evaluator& eval,
                    Sh3Runtime& runtime);
void bool_cipher_and(int pIdx, const sbMatrix& A, const sbMatrix& B, sbMatrix& res, Sh3Evaluator& eval,
                     Sh3Runtime& runtime);
void bool_cipher_or(int pIdx, const sbMatrix& A, const sbMatrix& B, sbMatrix& res, Sh3Evaluator& eval,
                    Sh3Runtime& runtime);
void bool_cipher_add(int pIdx, const sbMatrix& A, const sbMatrix& B, sbMatrix& res, Sh3Evaluator& eval,
                     Sh3Runtime& runtime);
void bool_cipher_sub(int pIdx, const sbMatrix& A, const sbMatrix& B, sbMatrix& res, Sh3Evaluator& eval,
                     Sh3Runtime& runtime);
// local NOT: x1 is inverted (P1 flips share 0, P2 flips share 1) (:315-342)
void bool_cipher_not(int pIdx, const sbMatrix& A, sbMatrix& res);
// (max, min) of each row pair in one compare-and-swap circuit (:228-312)
void bool_cipher_max_min_split(int pIdx, const sbMatrix& A, const sbMatrix& B, sbMatrix& resMax, sbMatrix& resMin,
                               Sh3Evaluator& eval, Sh3Runtime& runtime);
void bool_cipher_max(int pIdx, const sbMatrix& A, const sbMatrix& B, sbMatrix& res, Sh3Evaluator& eval,
                     Sh3Runtime& runtime);
void bool_cipher_min(int pIdx, const sbMatrix& A, const sbMatrix& B, sbMatrix& res, Sh3Evaluator& eval,
                     Sh3Runtime& runtime);

// Boolean -> arithmetic (BoolBasic.cpp:517-593). One bit: the public-ones
// product pi_cb_mul (zero shares from enc's generator). More bits (at most 64):
// c = x + r with r = PRNG(P0's next seed).get<int32_t>() (P0 and P1 draw the
// same r from a fresh PRNG of that seed), c opened to P2, which reshares it as
// (c - t, t) with a private t; result shares (-r, t, c - t).
void bool2arith(int pIdx, const sbMatrix& boolInput, si64Matrix& res, Sh3Encryptor& enc, Sh3Evaluator& eval,
                Sh3Runtime& runtime);

// ---- large messages (aby3-Basic/Basic.cpp:3-62): a column of `len` i64
// sent to / received from a neighbour as messages of at most `chunk`
// elements (MAX_SENDING_SIZE in the reference). The receiver must use the
// same length and chunk size. toNext / fromPrev pick mNext / mPrev, as there.
constexpr u64 MAX_SENDING_SIZE = 1ull << 25;
// host columns (the reference's form): blocking, like its asyncSendFuture(..).get()
int large_data_sending(int pIdx, const i64Matrix& sharedA, Sh3Runtime& runtime, bool toNext,
                       u64 chunk = MAX_SENDING_SIZE);
int large_data_receiving(int pIdx, i64Matrix& res, Sh3Runtime& runtime, bool fromPrev, u64 chunk = MAX_SENDING_SIZE);
// device columns of this party: the chunks are enqueued on the party's
// stream (sends) / delivered on it (receives: usable by later work on the
// stream when the call returns)
int large_data_sending(int pIdx, const i64* sharedA, u64 len, Sh3Runtime& runtime, bool toNext,
                       u64 chunk = MAX_SENDING_SIZE);
int large_data_receiving(int pIdx, i64* res, u64 len, Sh3Runtime& runtime, bool fromPrev,
                         u64 chunk = MAX_SENDING_SIZE);

// ---- sort: Sort.h (odd_even_merge, odd_even_multi_merge, high_dimensional_*)

// Evaluate one library circuit on sbMatrix inputs (shared helper).
void evalCircuit(BetaCircuit* cir, const std::vector<const sbMatrix*>& in, const std::vector<sbMatrix*>& out,
                 Sh3Evaluator& eval, Sh3Runtime& runtime);
CircuitLibrary& basicLibrary();  // per-thread circuit cache

}  // namespace aby3
