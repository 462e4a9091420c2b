"""The CPU oracle against known answers (CPU only).

No value-level golden data for this path exists in the reference (SURVEY.md
§4, §8(c)), and the reference cannot be built here (Mmg is absent), so the
oracle is pinned by analytic known answers computed independently with numpy
on the reference's own fixtures (libexamples/adaptation_example0, copied to
tests/golden/) and on synthetic lattices, plus the committed regression
vectors of tests/golden/make_golden.py.  Parity with the reference binary at
the Mmg arithmetic boundary (MMG5_invmat, MMG5_orvol, MMG5_EPS) is unpinned.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O
from parmmg_amd import synth
from parmmg_amd.synth import Mesh

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


# ------------------------------------------------------------------ MMG5_invmat restatement

def test_invmat_general_matches_numpy():
    rng = np.random.default_rng(3)
    for _ in range(200):
        A = rng.normal(size=(3, 3))
        M = A @ A.T + 0.5 * np.eye(3)
        m = M[[0, 0, 0, 1, 1, 2], [0, 1, 2, 1, 2, 2]]
        ok, mi = O.invmat(m)
        Mi = np.linalg.inv(M)
        assert ok
        np.testing.assert_allclose(mi, Mi[[0, 0, 0, 1, 1, 2], [0, 1, 2, 1, 2, 2]], rtol=1e-10, atol=1e-12)


def test_invmat_diagonal_shortcut_and_failures():
    ok, mi = O.invmat(np.array([4.0, 1e-7, -1e-7, 2.0, 5e-7, 8.0]))  # |offdiag| < EPS: exact diagonal inverse
    assert ok and np.array_equal(mi, [0.25, 0, 0, 0.5, 0, 0.125])
    ok, _ = O.invmat(np.zeros(6))  # zero matrix -> failure... through the diagonal shortcut: 1/0
    assert ok  # the reference's shortcut fires first (max offdiag 0 < EPS) and returns inf entries
    ok, _ = O.invmat(np.array([0.0, 1.0, 0.0, 0.0, 0.0, 0.0]))  # singular, off-diagonal above EPS
    assert not ok


# ------------------------------------------------------------------ cube fixture of the reference

def _p1_numpy(bg_xyz, bg_tetv, vals, x, ani):
    """Independent P1 (or inverse-tensor) interpolation: first tetra (index
    order) whose barycentric coordinates are all > -1e-9."""
    P = bg_xyz[bg_tetv - 1]  # (ne, 4, 3)
    for k in range(bg_tetv.shape[0]):
        A = np.vstack([P[k].T, np.ones(4)])
        lam = np.linalg.solve(A, np.r_[x, 1.0])
        if lam.min() > -1e-9:
            rows = vals[bg_tetv[k] - 1]
            if not ani:
                return lam @ rows
            inv = np.array([np.linalg.inv(r[[0, 1, 2, 1, 3, 4, 2, 4, 5]].reshape(3, 3)) for r in rows])
            M = np.linalg.inv(np.tensordot(lam, inv, 1))
            return M[[0, 0, 0, 1, 1, 2], [0, 1, 2, 1, 2, 2]]
    raise AssertionError("point outside")


def test_cube_fixture_known_answers():
    g = np.load(os.path.join(GOLD, "cube_refine8.npz"))
    bg = Mesh(0, 0, g["bg_xyz"], g["bg_tetv"], g["bg_adja"], g["bg_triv"], g["bg_adjt"], None)
    fields = [g[f"field{j}"] for j in range(int(g["nfield"]))]
    B = O.Background(bg, g["met"], fields)
    r = O.run(B, g["new_xyz"], g["pclass"], g["visit"])
    # cube-met.sol is the constant iso size 0.5
    np.testing.assert_allclose(r["met"][:, 0], 0.5, rtol=1e-15)
    for i, x in enumerate(g["new_xyz"]):
        # scalar x^2+y+z and vector (x,0,0) of cube-solphys.sol: P1 interpolant
        np.testing.assert_allclose(r["fields"][0][i], _p1_numpy(g["bg_xyz"], g["bg_tetv"], fields[0], x, False),
                                   rtol=1e-13, atol=1e-14)
        np.testing.assert_allclose(r["fields"][1][i], _p1_numpy(g["bg_xyz"], g["bg_tetv"], fields[1], x, False),
                                   rtol=1e-13, atol=1e-14)
        # tensor field: inverse of the interpolated inverses (interpmesh_pmmg.c:247-270)
        np.testing.assert_allclose(r["fields"][2][i], _p1_numpy(g["bg_xyz"], g["bg_tetv"], fields[2], x, True),
                                   rtol=1e-12, atol=1e-12)
    # (x,0,0) is affine: the P1 interpolation reproduces it
    np.testing.assert_allclose(r["fields"][1][:, 0], g["new_xyz"][:, 0], atol=1e-15)


@pytest.mark.parametrize("name", ["cube_refine8", "lattice_4_5_aniso"])
def test_golden_regression(name):
    g = np.load(os.path.join(GOLD, f"{name}.npz"))
    bg = Mesh(0, 0, g["bg_xyz"], g["bg_tetv"], g["bg_adja"], g["bg_triv"], g["bg_adjt"], None)
    fields = [g[f"field{j}"] for j in range(int(g["nfield"]))]
    B = O.Background(bg, g["met"], fields)
    r = O.run(B, g["new_xyz"], g["pclass"], g["visit"], O.MODE_FAITHFUL)
    assert np.array_equal(r["elem"], g["out_elem"])
    assert np.array_equal(r["hit"], g["out_hit"])
    assert np.array_equal(r["met"], g["out_met"], equal_nan=True)
    for j in range(len(fields)):
        assert np.array_equal(r["fields"][j], g[f"out_field{j}"], equal_nan=True)


# ------------------------------------------------------------------ synthetic lattices

def _case(kind, n_old, n_new, req_every=0, mode=O.MODE_FAITHFUL):
    bg = synth.lattice(kind, n_old)
    new = synth.lattice(kind, n_new, jitter=0.2)
    met = synth.solution(synth.F_ANI, bg.xyz)
    fs = [synth.solution(w, bg.xyz) for w in (synth.F_AFFINE, synth.F_AFFINE_VEC, synth.F_CONST_TENSOR)]
    pc = synth.classes(new, req_every)
    B = O.Background(bg, met, fs)
    return bg, new, B, pc, O.run(B, new.xyz, pc, synth.visit_order(new), mode)


@pytest.mark.parametrize("kind,n_old,n_new", [(synth.CUBE, 6, 7), (synth.CUBE, 5, 9), (synth.SHELL, 8, 12)])
def test_affine_fields_reproduced(kind, n_old, n_new):
    bg, new, B, pc, r = _case(kind, n_old, n_new)
    x = new.xyz
    vol = pc == 1
    np.testing.assert_allclose(r["fields"][0][vol, 0], 1 + 2 * x[vol, 0] - 3 * x[vol, 1] + 0.5 * x[vol, 2],
                               rtol=0, atol=1e-13)
    vec = np.c_[x[:, 0] + x[:, 1], 2 * x[:, 1] - x[:, 2], 3 * x[:, 2] + x[:, 0] - 1]
    np.testing.assert_allclose(r["fields"][1][vol], vec[vol], atol=1e-13)
    # constant SPD tensor: inverse-tensor interpolation returns it
    np.testing.assert_allclose(r["fields"][2][pc != 0], np.tile([4.0, 1.0, 0.5, 3.0, 0.25, 2.0], ((pc != 0).sum(), 1)),
                               rtol=1e-13)


def test_every_volume_point_located_and_accepted():
    bg, new, B, pc, r = _case(synth.CUBE, 7, 8, req_every=5)
    assert (r["hit"][pc == 0] == 0).all()
    vol = np.nonzero(pc == 1)[0]
    assert set(np.unique(r["hit"][vol])) == {1}
    for i in vol:
        assert O.tetra_minbary(B, r["elem"][i], new.xyz[i]) > -O.EPS
        assert r["minbary"][i] == O.tetra_minbary(B, r["elem"][i], new.xyz[i])
    bdy = np.nonzero(pc == 2)[0]
    assert set(np.unique(r["hit"][bdy])) <= {4, 5, 6, 7, 8}


def test_eval_in_element_reproduces_run():
    bg, new, B, pc, r = _case(synth.SHELL, 8, 12, mode=O.MODE_FRESH)
    for i in np.nonzero(pc)[0]:
        met, fr = O.eval_in_element(B, new.xyz[i], pc[i] == 2, r["elem"][i], r["hit"][i], r["loc"][i])
        assert np.array_equal(met, r["met"][i], equal_nan=True)
        for j, f in enumerate(fr):
            assert np.array_equal(f, r["fields"][j][i], equal_nan=True)


def test_exhaustive_and_closest_semantics():
    """Points outside the domain: stuck walk -> exhaustive scan -> closest
    tetra by |bary_min|*vol and the nearest vertex (locate_pmmg.c:737-770)."""
    bg = synth.lattice(synth.CUBE, 4)
    met = synth.solution(synth.F_ISO, bg.xyz)
    B = O.Background(bg, met, [])
    x = np.array([[1.2, 0.5, 0.5], [0.5, -0.3, 0.2], [0.999999, 0.5, 0.5]])
    pc = np.ones(3, np.uint8)
    r = O.run(B, x, pc, np.arange(1, 4, dtype=np.int32))
    assert list(r["hit"][:2]) == [3, 3]
    for i in range(2):
        # same metric value as the brute-force closest tetra (exact ties are
        # broken by evaluation order in the reference, by index here)
        kb = O.closest_tetra(B, x[i])
        assert O.closest_value(B, r["elem"][i], x[i]) == O.closest_value(B, kb, x[i])
        assert O.first_accepting_tetra(B, x[i]) == 0
    assert r["hit"][2] in (1, 2)


def test_faithful_vs_fresh_cone_state():
    """The reference's cone test reads point flags left by earlier queries;
    FRESH mode (what the HIP module implements) differs only at cone hits."""
    bg, new, B, pc, rf = _case(synth.SHELL, 8, 12, mode=O.MODE_FAITHFUL)
    rr = O.run(B, new.xyz, pc, synth.visit_order(new), O.MODE_FRESH)
    diff = rr["hit"] != rf["hit"]
    assert (~diff | np.isin(rf["hit"], [7, 8]) | np.isin(rr["hit"], [7, 8])).all()


def test_threaded_driver_matches_sequential():
    """orc_interp_mesh_mt (CPU baseline) = sequential runs over ranges: every
    point is processed, and where both runs pick the same element the values
    are bit-identical (warm starts differ per range, so near-face points may
    legitimately land in another accepting element)."""
    from parmmg_amd import synth

    bg = synth.lattice(synth.CUBE, 6)
    new = synth.lattice(synth.CUBE, 7, jitter=0.2, with_trias=False)
    met = synth.solution(synth.F_ANI, bg.xyz)
    fields = [synth.solution(synth.F_SCALAR, bg.xyz), synth.solution(synth.F_TENSOR, bg.xyz)]
    B = O.Background(bg, met, fields, 0.01)
    pc = synth.classes(new)
    order = np.arange(1, new.np + 1, dtype=np.int32)
    seq = O.run(B, new.xyz, pc, order)
    mt = O.run(B, new.xyz, pc, order, threads=4)
    act = pc != 0
    assert mt["nvisited"] == new.np
    assert ((mt["hit"] != 0) == act).all()
    same = act & (seq["elem"] == mt["elem"]) & (seq["hit"] == mt["hit"])
    assert same.sum() > 0.95 * act.sum()
    np.testing.assert_array_equal(seq["met"][same], mt["met"][same])
    for a, b in zip(seq["fields"], mt["fields"]):
        np.testing.assert_array_equal(a[same], b[same])


def test_invmat_failure_case_on_the_oracle():
    """tests/parity.invmat_failure_case on the oracle alone: every failure
    path of MMG5_invmat is reached and leaves its rows at the NaN sentinel
    (src/interpmesh_pmmg.c:98-107, 177-187, 258-267) — the case the GPU test
    test_invmat_failures_leave_rows_untouched compares against."""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from parity import check, invmat_failure_case

    case, vol, srf = invmat_failure_case()
    new, pc = case["new"], case["pclass"]
    out = O.run(case["B"], new.xyz, pc, synth.visit_order(new), O.MODE_FRESH)
    skip = pc == 0
    met_nan = np.isnan(out["met"]).all(axis=1) & ~skip
    ten_nan = np.isnan(out["fields"][2]).all(axis=1) & ~skip
    assert met_nan.sum() > 2 and ten_nan.sum() > 2
    for f in out["fields"][:2]:
        assert not np.isnan(f[~skip]).any()
    assert met_nan[vol] and ten_nan[vol] and met_nan[srf] and ten_nan[srf]
    assert out["hit"][vol] == 1 and out["hit"][srf] == 5
    for h in (1, 4, 5):
        assert (met_nan & (out["hit"] == h)).any(), h
    # the final inversion fails although every vertex tensor inverts
    for i in (vol, srf):
        k = int(out["elem"][i])
        vv = case["bg"].tetv[k - 1] if out["hit"][i] == 1 else case["bg"].triv[k - 1]
        for v in vv:
            assert O.invmat(case["met"][v - 1])[0]
    # the oracle's own run meets the contract check() applies to the GPU
    hit = out["hit"].astype(np.int32) | (np.maximum(out["loc"], 0).astype(np.int32) << 4)
    rep = check(case, dict(met=out["met"], fields=out["fields"], elem=out["elem"], hit=hit.astype(np.int8)))
    assert rep["n"] == int((~skip).sum()) and rep["exact"] == rep["n"]


def test_oracle_reaches_the_stale_reevaluation():
    """The reference's stale re-evaluation after a failed exhaustive tria
    search (src/locate_pmmg.c:505-509: `ptr` still at the last tria, the
    closest tria's normal and index): on the constructed fixture every point
    takes it (HIT_BDY_STALE = 10, element = the closest tria 1), in both
    oracle modes, with the values of that arithmetic restated independently
    in numpy (tests/parity.py::stale_case)."""
    from parity import stale_case

    case, exp = stale_case()
    n = case["new"].xyz.shape[0]
    for mode in (O.MODE_FAITHFUL, O.MODE_FRESH):
        r = O.run(case["B"], case["new"].xyz, case["pclass"], np.arange(1, n + 1, dtype=np.int32), mode)
        assert (r["hit"] == 10).all() and (r["elem"] == exp["elem"]).all(), (r["hit"], r["elem"])
        assert np.allclose(r["met"], exp["met"], rtol=1e-13, atol=0)
        assert np.allclose(r["fields"][0], exp["fields"][0], rtol=1e-13, atol=1e-14)
