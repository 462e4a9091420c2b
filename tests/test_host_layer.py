"""The C host layer's CPU-side pieces (csrc/pmmg_host.c), called through the
C-ABI on the CPU (no device needed):

* the point classification of the reference's visitation loop
  (src/interpmesh_pmmg.c:535-550), against a direct Python restatement;
* PMMG_copyMetricsAndFields_point (src/interpmesh_pmmg.c:311-446): frozen
  (MG_REQ) rows copied at the same index, or through permNodGlob when the
  mesh was renumbered (SCOTCH, src/libparmmg1.c:692-715), the metric only
  when inputMet == 1 and hsiz <= 0;
* MMG3D_Set_constantSize's fill (restated from Mmg, unpinned).
"""
import numpy as np
import pytest

from parmmg_amd import synth
from parmmg_amd.transfer import (TAG_BDY, TAG_NUL, TAG_REQ, classify_points, copy_metrics_and_fields_point,
                                 set_constant_metric)


def _classify_ref(tetv, tag, np_):
    pc = np.zeros(np_, np.uint8)
    seen = np.zeros(np_, bool)
    for v in tetv:
        if v[0] <= 0:
            continue
        for ip in v:
            if seen[ip - 1]:
                continue
            seen[ip - 1] = True
            t = int(tag[ip - 1])
            if t >= TAG_NUL or t & TAG_REQ:
                continue
            pc[ip - 1] = 2 if t & TAG_BDY else 1
    return pc


def test_classify_points_matches_the_visitation_loop():
    new = synth.lattice(synth.CUBE, 6, jitter=0.1)
    rng = np.random.default_rng(1)
    tag = np.where(new.isbdy == 1, TAG_BDY, 0).astype(np.uint16)
    tag[rng.choice(new.np, 30, replace=False)] |= TAG_REQ
    tag[rng.choice(new.np, 10, replace=False)] = TAG_NUL
    tetv = new.tetv.copy()
    tetv[rng.choice(new.ne, 40, replace=False), 0] = 0  # unused tetra (!MG_EOK)
    g = dict(xyz=new.xyz, tag=tag, tetv=tetv, met=None, fields=[])
    pc = classify_points(g)
    np.testing.assert_array_equal(pc, _classify_ref(tetv, tag, new.np))
    assert (pc == 1).any() and (pc == 2).any() and (pc == 0).any()


def _groups(np_old=40, np_new=50, seed=0):
    rng = np.random.default_rng(seed)
    old_met = rng.uniform(1, 2, (np_old, 6))
    old_f = [rng.uniform(-1, 1, (np_old, 1)), rng.uniform(-1, 1, (np_old, 3))]
    tag = np.zeros(np_old, np.uint16)
    tag[::3] |= TAG_REQ
    tag[5] = TAG_NUL | TAG_REQ  # invalid point: never copied

    class M:
        np, ne, nt = np_old, 0, 0
        xyz = tetv = adja = triv = adjt = None

    old = dict(mesh=M(), met=old_met, fields=old_f, tag=tag)
    new = dict(xyz=np.zeros((np_new, 3)), tag=np.zeros(np_new, np.uint16), tetv=np.zeros((0, 4), np.int32),
               met=np.full((np_new, 6), np.nan), fields=[np.full((np_new, 1), np.nan), np.full((np_new, 3), np.nan)])
    return old, new


def _valid_req(tag):
    return np.nonzero((tag < TAG_NUL) & ((tag & TAG_REQ) != 0))[0]


@pytest.mark.parametrize("renum", [0, 1])
def test_copy_required_same_index_without_renumbering(renum):
    old, new = _groups()
    # no permutation array: same index whatever renum says; renum without a
    # permutation array also keeps the index (src/interpmesh_pmmg.c:321)
    assert copy_metrics_and_fields_point(old, new, None, renum=renum, input_met=1) == 1
    req = _valid_req(old["tag"])
    np.testing.assert_array_equal(new["met"][req], old["met"][req])
    for a, b in zip(new["fields"], old["fields"]):
        np.testing.assert_array_equal(a[req], b[req])
    rest = np.setdiff1d(np.arange(new["met"].shape[0]), req)
    assert np.isnan(new["met"][rest]).all()


def test_copy_required_through_perm_nod_glob():
    old, new = _groups()
    np_old, np_new = old["met"].shape[0], new["met"].shape[0]
    perm = np.zeros(np_old + 1, np.int32)
    perm[1:] = np.random.default_rng(3).permutation(np_new)[:np_old] + 1
    # renum == 0: the permutation is ignored (src/interpmesh_pmmg.c:321)
    assert copy_metrics_and_fields_point(old, new, perm, renum=0) == 1
    req = _valid_req(old["tag"])
    np.testing.assert_array_equal(new["met"][req], old["met"][req])
    old, new = _groups()
    assert copy_metrics_and_fields_point(old, new, perm, renum=1) == 1
    dst = perm[req + 1] - 1
    np.testing.assert_array_equal(new["met"][dst], old["met"][req])
    np.testing.assert_array_equal(new["fields"][1][dst], old["fields"][1][req])
    assert np.isnan(np.delete(new["met"], dst, axis=0)).all()


def test_copy_required_metric_only_with_input_metric_and_no_hsiz():
    old, new = _groups()
    assert copy_metrics_and_fields_point(old, new, None, input_met=0) == 1
    assert np.isnan(new["met"]).all()
    req = _valid_req(old["tag"])
    np.testing.assert_array_equal(new["fields"][0][req], old["fields"][0][req])
    old, new = _groups()
    new["hsiz"] = 0.1
    assert copy_metrics_and_fields_point(old, new, None, input_met=1) == 1
    assert np.isnan(new["met"]).all()


def test_copy_required_rejects_targets_out_of_range():
    old, new = _groups()
    perm = np.full(old["met"].shape[0] + 1, new["met"].shape[0] + 5, np.int32)
    assert copy_metrics_and_fields_point(old, new, perm, renum=1) == 0


@pytest.mark.parametrize("ani", [0, 1])
def test_constant_metric(ani):
    n = 20
    tag = np.zeros(n, np.uint16)
    tag[3] = TAG_NUL
    met = np.full((n, 6 if ani else 1), np.nan)
    g = dict(xyz=np.zeros((n, 3)), tag=tag, tetv=np.zeros((0, 4), np.int32), met=met, fields=[], hsiz=0.2,
             hmin=0.0, hmax=0.0, ani=ani)
    assert set_constant_metric(g) == 1
    ok = np.arange(n) != 3
    if ani:
        q = 1.0 / (0.2 * 0.2)
        np.testing.assert_array_equal(met[ok], np.tile([q, 0, 0, q, 0, q], (n - 1, 1)))
    else:
        np.testing.assert_array_equal(met[ok, 0], 0.2)
    assert np.isnan(met[3]).all()  # !MG_VOK points untouched
    # hsiz outside the user bounds: MMG5_Compute_constantSize's "Mismatched
    # options" error (the metric is left untouched), inside them: accepted
    before = met.copy()
    g.update(hmin=0.3, hmax=0.0)
    assert set_constant_metric(g) == 0
    g.update(hmin=0.0, hmax=0.1)
    assert set_constant_metric(g) == 0
    np.testing.assert_array_equal(met[ok], before[ok])
    g.update(hmin=0.1, hmax=0.3)
    assert set_constant_metric(g) == 1
    np.testing.assert_array_equal(met[ok, 0], 1.0 / (0.2 * 0.2) if ani else 0.2)
    # the array must have the size info.ani asks for
    g["met"] = np.zeros((n, 1 if ani else 6))
    assert set_constant_metric(g) == 0
