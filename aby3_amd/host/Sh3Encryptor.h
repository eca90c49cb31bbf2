// Input sharing and reveal (aby3/sh3/Sh3Encryptor.h/.cpp), on device shares.
#pragma once
#include "Sh3Runtime.h"
#include "Sh3ShareGen.h"
#include "Sh3Types.h"

namespace aby3 {

class Sh3Encryptor {
public:
    void init(u64 partyIdx, block prevSeed, block nextSeed);
    void init(u64 partyIdx, CommPkg& comm, block seed);

    // x_i = getShare() + m (owner) / getShare() (others); send x_i to next,
    // receive x_{i-1} from prev (Sh3Encryptor.cpp:229-279).
    Sh3Task localIntMatrix(Sh3Task dep, const i64Matrix& m, si64Matrix& dest);
    Sh3Task remoteIntMatrix(Sh3Task dep, si64Matrix& dest);
    // Rows [rowOffset, rowOffset + dest.rows()) of the sharing of a
    // totalRows-row matrix (m holds those rows): the draws of the whole
    // matrix are taken from the share stream and the slice's rows used, so
    // the slice's shares are those rows of the unsplit sharing and the
    // stream ends where the unsplit sharing leaves it (a party whose rows are
    // split over GPUs; DESIGN.md §6 "Row split")
    Sh3Task localIntMatrixRows(Sh3Task dep, const i64Matrix& m, si64Matrix& dest, u64 rowOffset, u64 totalRows);
    Sh3Task remoteIntMatrixRows(Sh3Task dep, si64Matrix& dest, u64 rowOffset, u64 totalRows);
    // binary: x_i = getBinaryShare() ^ m (Sh3Encryptor.cpp:282-340)
    Sh3Task localBinMatrix(Sh3Task dep, const i64Matrix& m, sbMatrix& dest);
    Sh3Task remoteBinMatrix(Sh3Task dep, sbMatrix& dest);
    // fixed point: m scaled by 2^D then shared (Sh3Encryptor localFixedMatrix)
    Sh3Task localFixedMatrix(Sh3Task dep, const std::vector<double>& m, u64 rows, u64 cols, u64 D,
                             si64Matrix& dest);

    // reveal to this party: receive x_{i+1} from next, dest = x_i + x_{i-1} + x_{i+1}
    // (Sh3Encryptor.cpp:497-505); sbMatrix variant XORs (:527-535)
    Sh3Task reveal(Sh3Task dep, const si64Matrix& x, i64Matrix& dest);
    Sh3Task reveal(Sh3Task dep, const sbMatrix& x, i64Matrix& dest);
    // sender side of reveal to partyIdx (:516-525)
    Sh3Task reveal(Sh3Task dep, u64 partyIdx, const si64Matrix& x);
    Sh3Task reveal(Sh3Task dep, u64 partyIdx, const sbMatrix& x);
    Sh3Task revealAll(Sh3Task dep, const si64Matrix& x, i64Matrix& dest);
    Sh3Task revealAll(Sh3Task dep, const sbMatrix& x, i64Matrix& dest);

    u64 mPartyIdx = (u64)-1;
    Sh3ShareGen mShareGen;

private:
    // totalRows 0: dest is the whole matrix
    Sh3Task shareImpl(Sh3Task dep, const i64Matrix* m, SharedMat& dest, int kind, u64 rowOffset = 0,
                      u64 totalRows = 0);
    Sh3Task revealImpl(Sh3Task dep, const SharedMat& x, i64Matrix& dest, bool binary);
    Sh3Task revealSend(Sh3Task dep, u64 partyIdx, const SharedMat& x);
};

}  // namespace aby3
