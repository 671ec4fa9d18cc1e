"""Layout of the pruned harmonic sum's segmented cells (csrc/hip/hs_kernels.hpp,
written by pass 3 in csrc/hip/fft_passes.hip, staged by hs_load in
csrc/hip/harmonic_sum.hip), replayed in numpy: every cell is written by exactly
one pass-3 lane group and holds exactly the bins hs_cell8 maps to it; the
32-bit magic division and the two-cell cover of each aligned 8-bin cell that
the staging uses are exact. The GPU side is checked bit for bit against the
CPU harmonic sum in tests/test_gpu_kernels.py."""
import numpy as np
import pytest


def seg_index(k, C):
    k3, c = k // C, k % C
    return k3 * (C // 8 + 1) + np.where(c <= C // 2, c >> 3, ((c - 1) >> 3) + 1)


@pytest.mark.parametrize("C,L", [(24576, 256), (4096, 64), (6144, 512), (16384, 128)])
def test_segmented_cells_layout(C, L):
    M, half, cseg = C * L, C // 2, C // 8 + 1
    k = np.arange(M + 1, dtype=np.int64)
    idx = seg_index(k, C)
    assert np.all(np.diff(idx) >= 0) and idx[-1] == L * cseg
    # pass 3: workgroup c0 (rows c0..c0+7 <= C/2) writes, per k3, the cell of its
    # direct bins and (c0 != C/2) the cell of its mirror bins; bin M alone
    writes = {}
    for c0 in range(0, half + 1, 8):
        rows = np.arange(c0, c0 + 8)
        rows = rows[rows <= half]
        for k3 in range(L):
            direct = rows + C * k3  # row 0 (self-mirror) emits every k3 itself
            writes.setdefault(k3 * cseg + c0 // 8, []).append(direct)
            if c0 != half:
                mrows = rows[(rows != 0) & (rows != half)]
                writes.setdefault((L - 1 - k3) * cseg + (C - c0) // 8, []).append(M - mrows - C * k3)
    writes.setdefault(L * cseg, []).append(np.array([M]))
    assert all(len(v) == 1 for v in writes.values()), "a cell written by two lane groups"
    assert sorted(writes) == sorted(set(idx.tolist()))
    for cell, (bins,) in writes.items():
        assert np.all(idx[bins] == cell)
    counts = np.bincount(idx)
    assert sum(len(v[0]) for v in writes.values()) == counts.sum()


@pytest.mark.parametrize("C,L", [(24576, 256), (4096, 64), (6144, 512)])
def test_segmented_cells_staging_cover(C, L):
    M, c8, h8 = C * L, C // 8, C // 16
    magic = (1 << 40) // c8 + 1
    assert magic < 1 << 32
    idx = seg_index(np.arange(M + 8, dtype=np.int64), C)
    m = np.arange((M + 8) // 8, dtype=np.int64)
    k3 = ((m * magic) >> 32) >> 8  # __umulhi(m, magic) >> 8
    np.testing.assert_array_equal(k3, m // c8)
    x0 = m + k3
    x1 = x0 + ((m - k3 * c8) >= h8)
    np.testing.assert_array_equal(x0, idx[8 * m])
    np.testing.assert_array_equal(x1, idx[8 * m + 7])
