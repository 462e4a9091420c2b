"""Graded and stretched meshes: the reference's
anisotropic runs remesh a torus around a planar shock
(cmake/testing/pmmg_tests.cmake:52-63), whose adapted meshes are strongly
graded and stretched.  synth.graded maps a cube lattice so that the cell
size grows 1000x away from three planes and shears it.

CPU tests: the meshes are valid (positive volumes, boundary points on the
surface), graded >= 10^3 with elements stretched >= 50:1, and the oracle
meets the parity contract's premises on them (every point located, P1
exactness of an affine field).  GPU tests: the module against the oracle on
every point (tests/parity.py contract), the fp32 filter walk's hand-overs
counted."""
import numpy as np
import pytest

from oracle import oracle as O
from parity import check, run_gpu
from parmmg_amd import configs, synth


def _case(n_old, n_new, grade=configs.GRADE, fields=(synth.F_SCALAR, synth.F_VECTOR, synth.F_TENSOR, synth.F_AFFINE)):
    w = configs.Workload("graded-small", synth.CUBE, n_old, n_new, synth.F_ANI, fields, grade=grade)
    bg, new = configs.build_meshes(w, with_new_tetra=True)
    met = synth.solution(w.metric, bg.xyz)
    fs = [synth.solution(f, bg.xyz) for f in w.fields]
    pc = synth.classes(new)
    B = O.Background(bg, met, fs, w.hausd)
    vis = synth.visit_order(new)
    ref = O.run(B, new.xyz, pc, vis, O.MODE_FRESH)
    return dict(bg=bg, new=new, met=met, fields=fs, pclass=pc, B=B, hausd=w.hausd, ref=ref)


def test_graded_mesh_is_valid_graded_and_stretched():
    bg = synth.graded(synth.lattice(synth.CUBE, 24), configs.GRADE[0], configs.GRADE[2], configs.GRADE[3])
    st = synth.cell_stats(bg)
    assert st["min_volume"] > 0.0
    assert st["size_grading"] >= 300.0   # cube root of the volume ratio (1000^3 -> 1000 at the limit)
    assert st["max_aspect"] >= 50.0
    # the clustering planes: spacing along each axis graded by >= 10^3
    t = np.linspace(0.0, 1.0, 1001)
    for d in range(3):
        z = synth.shock_map(t, configs.GRADE[0][d], configs.GRADE[2][d])
        dz = np.diff(z)
        assert np.all(dz > 0) and dz.max() / dz.min() >= 900.0
    # signed volumes stay positive (orientation kept by the monotone map)
    p = bg.xyz[bg.tetv - 1]
    vol = np.einsum("ij,ij->i", p[:, 1] - p[:, 0], np.cross(p[:, 2] - p[:, 0], p[:, 3] - p[:, 0]))
    assert (vol > 0).all()


def test_graded_new_boundary_points_on_the_background_surface():
    w = configs.Workload("g", synth.CUBE, 10, 13, synth.F_ANI, (), grade=configs.GRADE)
    bg, new = configs.build_meshes(w)
    b = new.xyz[new.isbdy == 1]
    x, z0 = b[:, 0], b[:, 2] - configs.GRADE[3] * (b[:, 0] - 0.5)  # undo the shear
    on = (np.isclose(x, 0) | np.isclose(x, 1) | np.isclose(b[:, 1], 0) | np.isclose(b[:, 1], 1)
          | np.isclose(z0, 0) | np.isclose(z0, 1))
    assert on.all()


def test_oracle_on_graded_mesh_locates_every_point_and_is_p1_exact():
    case = _case(8, 11)
    ref = case["ref"]
    act = case["pclass"] != 0
    assert (ref["hit"][act] != 0).all()
    # the affine field is reproduced exactly (to rounding) wherever a volume point is located
    vol = act & ((ref["hit"] & 15) <= 2)
    exact = synth.solution(synth.F_AFFINE, case["new"].xyz)[:, 0]
    np.testing.assert_allclose(ref["fields"][3][vol, 0], exact[vol], rtol=1e-9, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("n_old,n_new", [(8, 11), (20, 23), (40, 45)])
def test_graded_parity(n_old, n_new):
    case = _case(n_old, n_new)
    for tet8 in (False, True):
        gpu = run_gpu(case, tet8=tet8)
        rep = check(case, gpu)
        st = gpu["stats"]
        print(n_old, n_new, tet8, rep, "nvol_exact", st["nvol_exact"], "stepmax", st["stepmax"],
              "steps/pt", st["steps_total"] / max(1, st["nvol"] + st["nbdy"]))
        assert rep["n"] == int((case["pclass"] != 0).sum())
        assert rep["class_i"] == rep["class_i_same"]
