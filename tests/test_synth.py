"""Synthetic workloads: sizes of SURVEY.md §8(d) and mesh validity."""
import numpy as np
import pytest

from parmmg_amd import configs, synth


@pytest.mark.parametrize("w,old,new", [
    (configs.CFG2, (175616, 998250), 205379),
    (configs.CFG3, (3442951, 20250000), 4096000),
    (configs.CFG4, (17112472, 101056368), 20345904),
    (configs.CFG5, (84027672, 500720718), 100544625),
])
def test_config_sizes_match_survey(w, old, new):
    (np_o, ne_o, _), (np_n, _, _) = w.counts()
    assert (np_o, ne_o) == old
    assert np_n == new


def test_algorithmic_bytes_cfg3_cfg4():
    # cfg3 B ~ 1.81 GB, cfg4 B ~ 9.01 GB
    assert abs(configs.CFG3.algorithmic_bytes() / 1e9 - 1.81) < 0.01
    assert abs(configs.CFG4.algorithmic_bytes() / 1e9 - 9.01) < 0.01


def _check_mesh(m):
    P = m.xyz
    T = m.tetv - 1
    a, b, c, d = P[T[:, 0]], P[T[:, 1]], P[T[:, 2]], P[T[:, 3]]
    vol = np.einsum("ij,ij->i", b - a, np.cross(c - a, d - a))
    assert (vol > 0).all()
    # adjacency symmetry + shared faces
    k, i = np.nonzero(m.adja)
    code = m.adja[k, i]
    kk, ii = code // 4 - 1, code % 4
    assert np.array_equal(m.adja[kk, ii], 4 * (k + 1) + i)
    fa = np.sort(np.where(np.arange(4)[None, :] != i[:, None], m.tetv[k], 0), 1)[:, 1:]
    fb = np.sort(np.where(np.arange(4)[None, :] != ii[:, None], m.tetv[kk], 0), 1)[:, 1:]
    assert np.array_equal(fa, fb)
    # closed boundary surface
    assert (m.adjt > 0).all()
    t, e = np.nonzero(m.adjt)
    c2 = m.adjt[t, e]
    assert np.array_equal(m.adjt[c2 // 3 - 1, c2 % 3], 3 * (t + 1) + e)
    assert m.nt == int((m.adja == 0).sum())


@pytest.mark.parametrize("kind,n,jit", [(synth.CUBE, 3, 0.0), (synth.CUBE, 5, 0.2), (synth.SHELL, 8, 0.0),
                                        (synth.SHELL, 16, 0.0)])
def test_lattice_valid(kind, n, jit):
    _check_mesh(synth.lattice(kind, n, jitter=jit))


def test_boundary_points_on_exact_surface():
    m = synth.lattice(synth.SHELL, 12, jitter=0.2)
    r = np.linalg.norm(m.xyz, axis=1)
    b = m.isbdy == 1
    assert np.allclose(np.minimum(np.abs(r[b] - 0.5), np.abs(r[b] - 1.0)), 0, atol=1e-14)
    assert ((r[~b] > 0.5) & (r[~b] < 1.0)).all()
    c = synth.lattice(synth.CUBE, 7, jitter=0.2)
    onf = np.any((c.xyz == 0.0) | (c.xyz == 1.0), axis=1)
    assert np.array_equal(onf, c.isbdy == 1)


def test_jitter_deterministic():
    a = synth.lattice(synth.CUBE, 6, jitter=0.2, seed=11)
    b = synth.lattice(synth.CUBE, 6, jitter=0.2, seed=11)
    c = synth.lattice(synth.CUBE, 6, jitter=0.2, seed=12)
    assert np.array_equal(a.xyz, b.xyz)
    assert not np.array_equal(a.xyz, c.xyz)


def test_fields_spd_and_slab_diagonal():
    m = synth.lattice(synth.CUBE, 6)
    for w in (synth.F_ANI, synth.F_TENSOR):
        t = synth.solution(w, m.xyz)
        M = t[:, [0, 1, 2, 1, 3, 4, 2, 4, 5]].reshape(-1, 3, 3)
        assert (np.linalg.eigvalsh(M) > 0).all()
    ani = synth.solution(synth.F_ANI, m.xyz)
    slab = m.xyz[:, 0] < 0.1
    assert (ani[slab][:, [1, 2, 4]] == 0).all()


def test_mmg_like_numbering_is_a_permutation():
    """bench.py's Mmg-like numbering: a permutation, one point in ~six
    appended at the end, both parts in the generator's order."""
    n = 100_000
    perm = synth.mmg_like_perm(n)
    assert np.array_equal(np.sort(perm), np.arange(n))
    cut = int(np.argmax(np.diff(perm) < 0)) + 1  # the appended part starts where the order restarts
    head, tail = perm[:cut], perm[cut:]
    assert np.all(np.diff(head) > 0) and np.all(np.diff(tail) > 0)
    assert 0.14 < tail.size / n < 0.19


def _volumes(m):
    tv = m.tetv.astype(np.int64) - 1
    x = m.xyz
    return np.einsum("ij,ij->i", x[tv[:, 1]] - x[tv[:, 0]], np.cross(x[tv[:, 2]] - x[tv[:, 0]], x[tv[:, 3]] - x[tv[:, 0]]))


def test_valid_jitter_keeps_every_tetra_positive():
    """The shell's radial map leaves slivers along the planes |y_i| = |y_j|
    that the plain jitter inverts (the r05 iteration-2 background: 0.23 % of
    its tetra, 2655 walks cycling to the step cap); synth_vertices_valid caps
    each vertex's displacement so that the jittered lattice stays a valid
    mesh, with boundary vertices still on their spheres."""
    plain = synth.lattice(synth.SHELL, 24, jitter=0.2, seed=7, with_trias=False)
    assert (_volumes(plain) <= 0).sum() > 0
    for kind, n in ((synth.SHELL, 24), (synth.SHELL, 40), (synth.CUBE, 20)):
        m = synth.lattice(kind, n, jitter=0.2, seed=7, with_trias=False, valid=True)
        assert (_volumes(m) > 0).all()
        ref = synth.lattice(kind, n, jitter=0.0, with_tetra=False)
        assert not np.array_equal(m.xyz, ref.xyz)  # still jittered
        b = m.isbdy.astype(bool)
        if kind == synth.SHELL:
            r = np.abs(np.linalg.norm(m.xyz[b], axis=1))
            assert np.all(np.isclose(r, 1.0) | np.isclose(r, 0.5))
