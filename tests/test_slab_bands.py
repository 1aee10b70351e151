"""slab_bands (drtvam_amd/optimize.py): the (row band, slice range) parts of a banded planar
iteration, on synthetic row -> slice maps (CPU): ranges on whole forward / adjoint / 64-slice bin
blocks, one contiguous band of rows per range, bands tiling the rows in either row order, unmapped
rows absorbed, and None where the map has no banded structure."""
import numpy as np

from drtvam_amd.optimize import slab_bands


def _check(parts, m, nz, R):
    rows = sorted((r0, r1) for r0, r1, _, _ in parts)
    assert rows[0][0] == 0 and rows[-1][1] == R and all(a[1] == b[0] for a, b in zip(rows, rows[1:]))
    assert parts[0][2] == 0 and parts[-1][3] == nz and all(a[3] == b[2] for a, b in zip(parts, parts[1:]))
    for r0, r1, z0, z1 in parts:  # every mapped row of the band lies in the band's slices, and vice versa
        band = m[r0:r1]
        assert np.all((band < 0) | ((band >= z0) & (band < z1)))
        assert not np.any((np.delete(m, np.arange(r0, r1)) >= z0) & (np.delete(m, np.arange(r0, r1)) < z1))


def test_bottom_up_rows():
    nz = R = 400
    m = np.arange(R)
    parts = slab_bands(m, nz, 3, 32, 8, R)
    assert [(z0, z1) for _, _, z0, z1 in parts] == [(0, 128), (128, 256), (256, 400)]
    _check(parts, m, nz, R)


def test_top_down_rows_with_unmapped_edges():
    nz, R = 192, 210
    m = np.full(R, -1)
    m[9:201] = np.arange(nz)[::-1]  # row 9 feeds the top slice; rows 0..8 and 201..209 miss the grid
    parts = slab_bands(m, nz, 3, 32, 8, R)
    assert len(parts) == 3
    _check(parts, m, nz, R)
    assert parts[0][0] > parts[-1][0]  # slice order runs against row order


def test_two_rows_per_slice_and_single_range():
    nz, R = 128, 256
    m = np.repeat(np.arange(nz), 2)
    parts = slab_bands(m, nz, 2, 32, 8, R)
    _check(parts, m, nz, R)
    assert slab_bands(m, nz, 2, 40, 8, R) is None  # 320-slice blocks: one range, nothing to band


def test_interleaved_rows_rejected():
    nz = R = 128
    m = np.arange(R)
    m[10], m[100] = m[100], m[10]  # a row of the last range inside the first band
    assert slab_bands(m, nz, 2, 32, 8, R) is None


def test_balanced_slabs_cover_and_balance():
    """The slab split: contiguous slabs that tile the film, one per rank, whose
    largest cost is the least any contiguous split reaches (brute force on small cases)."""
    import itertools
    import numpy as np
    from drtvam_amd.optimize import balanced_slabs
    rng = np.random.default_rng(0)
    for n, w in [(10, 3), (12, 4), (9, 2), (7, 7), (16, 5)]:
        c = rng.uniform(1.0, 1.5, n)
        e = balanced_slabs(c, w)
        assert e[0][0] == 0 and e[-1][1] == n and all(a < b for a, b in e)
        assert all(e[i][1] == e[i + 1][0] for i in range(w - 1))
        got = max(c[a:b].sum() for a, b in e)
        best = min(max(c[a:b].sum() for a, b in zip((0,) + cut, cut + (n,)))
                   for cut in itertools.combinations(range(1, n), w - 1))
        assert got <= best + 1e-9


def test_slab_costs_weigh_target_slices():
    """Slices holding target voxels cost more (their adjoint tiles are marched); the box target's
    8-rank split gives the two end slabs, which hold the empty slices, more slices."""
    from drtvam_amd.optimize import balanced_slabs, slab_costs
    from drtvam_amd.utils import analytic_target
    t = analytic_target((400, 400, 400), (-5.0, -5.0, -5.0), (5.0, 5.0, 5.0))
    c = slab_costs(t)
    assert c[0] == 1.0 and c[200] > 1.2
    e = balanced_slabs(c, 8)
    sizes = [b - a for a, b in e]
    assert sizes[0] > 50 and sizes[-1] > 50 and max(sizes[1:-1]) < 50
