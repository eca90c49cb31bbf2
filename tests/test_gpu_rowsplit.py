"""One party's rows split over GPUs (optional): the truncated
share GEMM of C2 and the comparison of C3 run as `shards` row slices, each a
three-party session of its own (the jobs' shard parameters:
localIntMatrixRows + Sh3Evaluator::asyncMulRows; cipher_gt_rows, whose
circuit masks are the slice's words of every AND gate's draws). Every
party's shares of every slice must be exactly those rows of the unsplit
job's shares -- over two steps, so the slices also leave the parties'
randomness streams where the unsplit job does. The slices run one after the other on cuda:0 (the boxes have one GPU);
on a node each would run on its own GPU with no exchange between them."""
import numpy as np
import pytest

from aby3_amd import native as nt


def _shares(params, steps, job=nt.JOB_MUL_TRUNC):
    with nt.Session(job, params, probe=False) as s:
        s.run(steps)
        assert s.check()
        return [s.result(p) for p in range(3)]


@pytest.mark.gpu
@pytest.mark.parametrize("mkn,d,shards", [
    ((256, 200, 130), 16, 2),
    ((257, 64, 96), 8, 3),      # uneven slices (85, 86, 86 rows)
    ((1024, 1024, 1024), 16, 2),  # C2
    ((5, 32, 16), 16, 8),       # more slices than some have rows (empty slices)
])
def test_row_split_share_exact(gpu, mkn, d, shards):
    M, K, N = mkn
    base = [M, K, N, d, 1, 1]
    ref = _shares(base, 2)
    got = [[[], []] for _ in range(3)]
    for k in range(shards):
        for p, (s0, s1) in enumerate(_shares(base + [k, shards], 2)):
            rows = M * (k + 1) // shards - M * k // shards
            assert s0.size == rows * N and s1.size == rows * N
            got[p][0].append(s0)
            got[p][1].append(s1)
    for p in range(3):
        for sh in range(2):
            want = ref[p][sh].reshape(M, N)
            have = np.concatenate(got[p][sh]).reshape(M, N)
            bad = np.argwhere(want != have)
            assert bad.size == 0, f"party {p} share {sh}: {len(bad)} entries differ, first at {bad[0]}"


@pytest.mark.gpu
def test_row_split_rejects_bad_shards(gpu):
    with pytest.raises(nt.NativeError):
        nt.Session(nt.JOB_MUL_TRUNC, [64, 64, 64, 16, 1, 1, 2, 2], probe=False)
    with pytest.raises(nt.NativeError):  # Hadamard products are not split
        nt.Session(nt.JOB_MUL_TRUNC, [64, 64, 64, 16, 0, 1, 0, 2], probe=False)


def _msb_edges(rows, shards):
    return [rows if k == shards else rows * k // shards // 2048 * 2048 for k in range(shards + 1)]


@pytest.mark.gpu
@pytest.mark.parametrize("rows,shards", [
    (3 * 2048 + 100, 2),
    (3 * 2048 + 100, 3),
    (1000, 2),          # the first slice empty
    (1 << 20, 2),       # C3
    (1 << 20, 4),
])
def test_row_split_comparison_share_exact(gpu, rows, shards):
    ref = _shares([rows], 2, nt.JOB_MSB)
    e = _msb_edges(rows, shards)
    got = [[[], []] for _ in range(3)]
    for k in range(shards):
        for p, (s0, s1) in enumerate(_shares([rows, k, shards], 2, nt.JOB_MSB)):
            assert s0.size == e[k + 1] - e[k] and s1.size == e[k + 1] - e[k]
            got[p][0].append(s0)
            got[p][1].append(s1)
    for p in range(3):
        for sh in range(2):
            have = np.concatenate(got[p][sh])
            bad = np.flatnonzero(ref[p][sh] != have)
            assert bad.size == 0, f"party {p} share {sh}: {bad.size} rows differ, first {bad[0]}"
