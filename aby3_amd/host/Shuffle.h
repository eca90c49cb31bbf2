// The 3-party secret shuffle of aby3-Basic (Shuffle.cpp, after Asharov et al.,
// CCS'21 "advanced" variant) on the GPU engine: every party's masks are
// AES-CTR words of its prev / next common PRNG seeds, its two permutations are
// std::random_shuffle of 0..len-1 driven by PRNG(seed) (BoolBasic.cpp:925-934,
// restated on the host and cached per seed and length), and every
// mask-and-permute step is one gather launch over the packed units
// (aby3g_u64_xor_gather_units); the three rounds of messages are device
// payloads of at most MAX_SENDING_SIZE words (large_data_sending).
//
// Semantics kept from the reference, including its quirks:
//  * get_random_mask starts a fresh PRNG(seed) on every call, so every unit of
//    a vector gets the same mask (the first `unit` words of the stream), and
//    the parties' output masks equal their masking masks;
//  * the vector forms permute with the scattering plain_permutate
//    (tmp[p[i]] = x[i], Basics.h:324-332), the sbMatrix form with the
//    gathering one (res(i) = x(p[i]), BoolBasic.cpp:1033-1042) and uses the
//    first word of each row only (bit counts up to 64);
//  * the result is the input permuted by combine_permutation of the three
//    parties' permutations (Test.cpp:262-345).
#pragma once
#include "Basic.h"

namespace aby3 {

void get_permutation(size_t len, std::vector<size_t>& permutation, block seed);
void get_inverse_permutation(const std::vector<size_t>& permutation, std::vector<size_t>& inverse_permutation);
void combine_permutation(const std::vector<std::vector<size_t>>& permutation_list, std::vector<size_t>& final_permutation);

// Shuffle.cpp:14-226: T[i] a unit_len-word binary share each (i64Size words
// in Eigen's column-major order); Tres[i] the shuffled units.
int efficient_shuffle(std::vector<sbMatrix>& T, int pIdx, std::vector<sbMatrix>& Tres, Sh3Encryptor& enc,
                      Sh3Evaluator& eval, Sh3Runtime& runtime);
// Shuffle.cpp:229-385: the rows of T (bitCount <= 64).
int efficient_shuffle(sbMatrix& T, int pIdx, sbMatrix& Tres, Sh3Encryptor& enc, Sh3Evaluator& eval,
                      Sh3Runtime& runtime);
// Shuffle.cpp:388-903: the shuffle plus the binary shares of the permutation
// it applied (Pi[i] = shares of final_permutation[i]).
int efficient_shuffle_with_random_permutation(std::vector<sbMatrix>& T, int pIdx, std::vector<sbMatrix>& Tres,
                                              std::vector<si64>& Pi, Sh3Encryptor& enc, Sh3Evaluator& eval,
                                              Sh3Runtime& runtime);

// The packed forms the above run on: `len` units of `unit` words, device
// arrays [2][len][unit] (share 0 then share 1) of this party. Tres may not
// alias T. Pi (optional) receives the permutation's shares as [2][len].
int efficient_shuffle_units(const u64* T, u64 len, u64 unit, int pIdx, u64* Tres, Sh3Encryptor& enc,
                            Sh3Runtime& runtime);
int efficient_shuffle_rows(const u64* T, u64 len, int pIdx, u64* Tres, Sh3Encryptor& enc, Sh3Runtime& runtime);
int efficient_shuffle_with_random_permutation_units(const u64* T, u64 len, u64 unit, int pIdx, u64* Tres, u64* Pi,
                                                    Sh3Encryptor& enc, Sh3Runtime& runtime);

}  // namespace aby3
