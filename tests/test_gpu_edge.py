"""Edge cases and full-size properties of the HIP module (runs on the MI355X).

Full-size checks follow tests/parity.py's contract through size-independent
properties (the oracle cannot replay 4M points in seconds): every point
processed, affine fields reproduced exactly by the P1 interpolation (bit
tolerance 1e-13 absolute), a constant SPD tensor reproduced by the
inverse-tensor interpolation, acceptance and values of a random sample
checked against the oracle, and determinism across runs.
"""
import numpy as np
import pytest

from parity import check, make_case, run_dev, run_gpu
from parmmg_amd import configs, synth
from parmmg_amd.transfer import TransferContext, pack_tet8

C = synth.CUBE


@pytest.mark.gpu
def test_zero_new_points():
    case = make_case(kind=C, n_old=4, n_new=3, with_ref=False)
    with TransferContext(0) as ctx:
        bg = case["bg"]
        ctx.set_background(bg.xyz, bg.tetv, bg.adja, bg.triv, bg.adjt, case["hausd"])
        ctx.set_solutions(case["met"], case["fields"])
        st = ctx.locate_interp(np.zeros((0, 3)), np.zeros(0, np.uint8), np.zeros((0, 6)),
                               [np.zeros((0, f.shape[1])) for f in case["fields"]])
        assert st.nvol == 0 and st.nbdy == 0


@pytest.mark.gpu
def test_all_points_skipped():
    case = make_case(kind=C, n_old=4, n_new=5, with_ref=False)
    case["pclass"][:] = 0
    gpu = run_gpu(case)
    assert (gpu["hit"] == 0).all() and np.isnan(gpu["met"]).all()


@pytest.mark.gpu
def test_background_without_trias_volume_only():
    """nt = 0 is allowed when no surface query is submitted."""
    import dataclasses

    case = make_case(kind=C, n_old=5, n_new=6)
    case["pclass"] = np.where(case["pclass"] == 2, 0, case["pclass"]).astype(np.uint8)
    bg_notri = dataclasses.replace(case["bg"], triv=np.zeros((0, 3), np.int32), adjt=np.zeros((0, 3), np.int32))
    gpu = run_gpu(dict(case, bg=bg_notri))
    rep = check(case, gpu)
    assert rep["n"] == int((case["pclass"] == 1).sum())


@pytest.mark.gpu
@pytest.mark.parametrize("fields", [
    (synth.F_VECTOR, synth.F_SCALAR, synth.F_TENSOR, synth.F_VECTOR),                 # generic layout path
    (synth.F_SCALAR,) * 7,                                                              # metric + 7 fields (slot limit)
])
def test_unusual_slot_layouts(fields):
    case = make_case(kind=C, n_old=5, n_new=6, metric=synth.F_ISO, fields=fields)
    for kw in ({}, dict(tet8=True)):
        gpu = run_gpu(case, **kw)
        rep = check(case, gpu)
        assert rep["class_i"] == rep["class_i_same"]


@pytest.mark.gpu
def test_too_many_fields_rejected():
    case = make_case(kind=C, n_old=3, n_new=3, metric=synth.F_ISO, fields=(synth.F_SCALAR,) * 8, with_ref=False)
    with TransferContext(0) as ctx:
        bg = case["bg"]
        ctx.set_background(bg.xyz, bg.tetv, bg.adja, bg.triv, bg.adjt, case["hausd"])
        with pytest.raises(RuntimeError):
            ctx.set_solutions(case["met"], case["fields"])


def _full_size(w, seed=synth.SEED):
    bg = synth.lattice(w.kind, w.n_old)
    new = synth.lattice(w.kind, w.n_new, jitter=w.jitter_new, seed=seed)
    met = synth.solution(w.metric, bg.xyz)
    fields = [synth.solution(f, bg.xyz) for f in (synth.F_AFFINE, synth.F_AFFINE_VEC, synth.F_CONST_TENSOR)]
    pc = synth.classes(new)
    return bg, new, met, fields, pc


def _run_dev(ctx, bg, new, met, fields, pc, hausd, separate=False):
    return run_dev(ctx, bg, new.xyz, met, fields, pc, hausd, separate)


@pytest.mark.gpu
def test_full_size_cfg3_properties():
    """cfg3 (20.25M background tetra, 4.1M new points) with fields whose exact
    answers are known: affine scalar and vector (P1 reproduces them), constant
    SPD tensor (the inverse-tensor interpolation returns it)."""
    w = configs.CFG3
    bg, new, met, fields, pc = _full_size(w)
    with TransferContext(0) as ctx:
        mo, fo, el, hit, st = _run_dev(ctx, bg, new, met, fields, pc, w.hausd)
        mo2, fo2, el2, hit2, _ = _run_dev(ctx, bg, new, met, fields, pc, w.hausd, separate=True)
    act = pc != 0
    assert ((hit & 15) != 0).sum() == act.sum()
    assert ((hit & 15)[~act] == 0).all()
    assert st.nvol_exhaust + st.nvol_closest < 0.001 * act.sum()
    x = new.xyz
    vol = pc == 1
    np.testing.assert_allclose(fo[0][vol, 0], 1 + 2 * x[vol, 0] - 3 * x[vol, 1] + 0.5 * x[vol, 2], rtol=0,
                               atol=1e-12)
    vec = np.c_[x[:, 0] + x[:, 1], 2 * x[:, 1] - x[:, 2], 3 * x[:, 2] + x[:, 0] - 1]
    np.testing.assert_allclose(fo[1][vol], vec[vol], rtol=0, atol=1e-12)
    np.testing.assert_allclose(fo[2][act], np.tile([4.0, 1.0, 0.5, 3.0, 0.25, 2.0], (int(act.sum()), 1)),
                               rtol=1e-12)
    # metric: SPD, finite on every processed point
    assert np.isfinite(mo[act]).all()
    # separate tetv / adja arrays give bit-identical results (same kernels, same elements)
    np.testing.assert_array_equal(el, el2)
    np.testing.assert_array_equal(mo, mo2)
    for a, b in zip(fo, fo2):
        np.testing.assert_array_equal(a, b)


@pytest.mark.gpu
def test_full_size_cfg3_sample_against_oracle_and_determinism():
    """A random sample of cfg3's points checked against the oracle (acceptance
    of the chosen element + values bit-for-bit), and two runs bit-identical."""
    from oracle import oracle as O

    w = configs.CFG3
    bg, new, met, fields, pc = _full_size(w)
    fields = [synth.solution(f, bg.xyz) for f in w.fields]
    with TransferContext(0) as ctx:
        mo, fo, el, hit, st = _run_dev(ctx, bg, new, met, fields, pc, w.hausd)
        mo2, fo2, el2, hit2, _ = _run_dev(ctx, bg, new, met, fields, pc, w.hausd)
    np.testing.assert_array_equal(el, el2)
    np.testing.assert_array_equal(hit, hit2)
    np.testing.assert_array_equal(mo, mo2)
    case = dict(B=O.Background(bg, met, fields, w.hausd), new=new, pclass=pc, met=met, fields=fields)
    rep = check(case, dict(met=mo, fields=fo, elem=el, hit=hit), max_points=3000)
    assert rep["n"] == 3000 and rep["maxrel"] <= 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("n", [39, 101, 127])
def test_query_order_detection(n):
    """Input order is kept for a lattice numbering whatever its row length
    (n=127: 128^3 points, a row length an evenly strided sample would alias
    with) and for an Mmg-like one, and Morton binning is chosen for a
    shuffled numbering of a group of at least 2^20 points (n=39: 64k points,
    a small group, keeps the input order untested: kSmallGroup); results are
    the same either way."""
    case = make_case(kind=C, n_old=8, n_new=n, with_ref=False)
    a = run_gpu(case)
    assert a["stats"]["sorted"] == 0
    rng = np.random.default_rng(3)
    perm = rng.permutation(case["new"].np)
    import dataclasses
    shuf = dict(case)
    shuf["new"] = dataclasses.replace(case["new"], xyz=np.ascontiguousarray(case["new"].xyz[perm]))
    shuf["pclass"] = np.ascontiguousarray(case["pclass"][perm])
    b = run_gpu(shuf)
    assert b["stats"]["sorted"] == (1 if case["new"].np >= 1 << 20 else 0)
    np.testing.assert_array_equal(b["elem"], a["elem"][perm])
    np.testing.assert_array_equal(b["met"], a["met"][perm])
    # an Mmg-like numbering (the inserted sixth appended) keeps its input order
    perm = synth.mmg_like_perm(case["new"].np)
    mmg = dict(case)
    mmg["new"] = dataclasses.replace(case["new"], xyz=np.ascontiguousarray(case["new"].xyz[perm]))
    mmg["pclass"] = np.ascontiguousarray(case["pclass"][perm])
    m = run_gpu(mmg)
    assert m["stats"]["sorted"] == 0
    np.testing.assert_array_equal(m["elem"], a["elem"][perm])
