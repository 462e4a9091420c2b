"""Load-balancing weights from the interpolated metric: PMMG_computeWgt /
PMMG_computeWgt_mesh (reference src/metis_pmmg.c:242-300), the oracle
restatement pinned by known answers (CPU) and the device kernels
(pmmg_hip_compute_wgt_mesh / _faces) against it (GPU).

Tolerance: 1e-13 relative — the device's exp / log1p are not the host libm's
(each within an ulp), the rest of the arithmetic keeps the reference's order."""
import math

import numpy as np
import pytest

from oracle import oracle as O
from parmmg_amd import synth

HUGE = 1.0e6  # PMMG_WGTVAL_HUGEINT
MG_PARBDY = 1 << 6


def _regular_tetra(edge=1.0):
    a = edge
    xyz = np.array([[0, 0, 0], [a, 0, 0], [a / 2, a * math.sqrt(3) / 2, 0],
                    [a / 2, a * math.sqrt(3) / 6, a * math.sqrt(2.0 / 3.0)]], np.float64)
    return xyz, np.array([1, 2, 3, 4], np.int32)


def test_no_metric_is_hugeint():
    xyz, v = _regular_tetra()
    assert O.face_wgt(xyz, v, 0, None) == HUGE


@pytest.mark.parametrize("h,expect", [(1.0, 1.0), (1.25, math.exp(28 * 0.6 / 3)), (2.0, HUGE),
                                      (0.5, math.exp(-28 * (3 * (0.5 - 1.0)) / 3))])
def test_constant_iso_metric_known_answers(h, expect):
    """Unit edges in a constant size h: len = 1/h per edge (MMG5_lenedgCoor_iso
    with h1 == h2), res = 3 (len - 1) or 3 (1/len - 1)."""
    xyz, v = _regular_tetra()
    met = np.full((4, 1), h)
    for f in range(4):
        w = O.face_wgt(xyz, v, f, met)
        assert w == pytest.approx(min(expect, HUGE), rel=1e-13)


def test_graded_iso_metric_matches_formula():
    """h1 != h2: len = l log(h2/h1) / (h2 - h1) (MMG5_lenedgCoor_iso)."""
    xyz, v = _regular_tetra(0.7)
    met = np.array([[0.5], [0.9], [1.3], [0.6]])
    f = 0  # face 0 = vertices 1, 2, 3 (MMG5_iarf[0] = edges 5, 4, 3)
    res = 0.0
    for a, b in ((2, 3), (1, 3), (1, 2)):
        l = np.linalg.norm(xyz[b] - xyz[a])
        h1, h2 = met[a, 0], met[b, 0]
        ln = l / (h2 - h1) * math.log1p(h2 / h1 - 1.0)
        res += ln - 1.0 if ln <= 1.0 else 1.0 / ln - 1.0
    assert O.face_wgt(xyz, v, f, met) == pytest.approx(min(1.0 / math.exp(28 * res / 3), HUGE), rel=1e-13)


def test_identity_tensor_equals_unit_iso():
    xyz, v = _regular_tetra(0.9)
    iso = np.ones((4, 1))
    ani = np.tile([1.0, 0, 0, 1.0, 0, 1.0], (4, 1))
    for f in range(4):
        assert O.face_wgt(xyz, v, f, ani) == pytest.approx(O.face_wgt(xyz, v, f, iso), rel=1e-15)


def test_mesh_weights_sum_tagged_faces_and_leave_others():
    xyz, v = _regular_tetra()
    tetv = np.array([v, v, [0, 0, 0, 0]], np.int32)
    xt = np.array([1, 0, 1], np.int32)
    ftag = np.array([[MG_PARBDY, 0, MG_PARBDY, 1], [MG_PARBDY] * 4, [MG_PARBDY] * 4], np.uint16)
    q = O.compute_wgt_mesh(xyz, tetv, xt, ftag, None, MG_PARBDY, np.array([7.0, 8.0, 9.0]))
    np.testing.assert_array_equal(q, [2 * HUGE, 8.0, 9.0])  # no xtetra / unused: untouched


def _case(ani, n=6, seed=3):
    bg = synth.lattice(synth.CUBE, n, jitter=0.15, seed=seed)
    met = synth.solution(synth.F_ANI if ani else synth.F_ISO, bg.xyz)
    rng = np.random.default_rng(seed)
    xt = (rng.random(bg.ne) < 0.6).astype(np.int32)
    ftag = np.where(rng.random((bg.ne, 4)) < 0.5, MG_PARBDY, 0).astype(np.uint16) | 1
    return bg, met, xt, ftag


@pytest.mark.gpu
@pytest.mark.parametrize("ani", [False, True, None])
def test_device_weights_match_oracle(ani):
    from parmmg_amd.transfer import TransferContext

    bg, met, xt, ftag = _case(bool(ani))
    if ani is None:
        met = None
    qual0 = np.linspace(0.5, 1.5, bg.ne)
    want = O.compute_wgt_mesh(bg.xyz, bg.tetv, xt, ftag, met, MG_PARBDY, qual0)
    faces = np.array([(k + 1, f) for k in range(0, bg.ne, 3) for f in range(4)], np.int32)
    want_f = np.array([O.face_wgt(bg.xyz, bg.tetv[k - 1], f, met) for k, f in faces])
    with TransferContext(0) as ctx:
        d = [ctx.upload(a) for a in (bg.xyz, bg.tetv, xt, ftag, qual0, faces)]
        dm = None if met is None else ctx.upload(met)
        q = ctx.compute_wgt_mesh(d[0], d[1], d[2], d[3], dm, MG_PARBDY, d[4]).download()
        wf = ctx.compute_wgt_faces(d[0], d[1], d[5], dm).download()
    np.testing.assert_array_equal(q[xt == 0], qual0[xt == 0])
    np.testing.assert_allclose(q, want, rtol=1e-13, atol=0)
    np.testing.assert_allclose(wf, want_f, rtol=1e-13, atol=0)
    print("exact:", int((q == want).sum()), "of", q.size, "faces exact:", int((wf == want_f).sum()), "of", wf.size)
