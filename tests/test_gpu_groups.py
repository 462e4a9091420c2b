"""Many groups in one call (pmmg_hip_locate_interp_groups): the loop of
src/interpmesh_pmmg.c:690 over a rank's groups as one enqueue, groups spread
over the context's lanes.  Every group's outputs must be bit-identical to one
pmmg_hip_locate_interp per group, and meet the oracle contract."""
import os

import numpy as np
import pytest

from parity import check, make_case, run_gpu
from parmmg_amd import synth
from parmmg_amd.transfer import TransferContext, pack_tet8

C, S = synth.CUBE, synth.SHELL
GROUPS = [dict(kind=C, n_old=6, n_new=7), dict(kind=S, n_old=8, n_new=12),
          dict(kind=C, n_old=5, n_new=9, metric=None, fields=(synth.F_TENSOR, synth.F_AFFINE_VEC)),
          dict(kind=C, n_old=7, n_new=5, metric=synth.F_ISO, fields=(synth.F_SCALAR,)),
          dict(kind=S, n_old=12, n_new=8, metric=synth.F_ISO, fields=(synth.F_SCALAR, synth.F_AFFINE))]


def _device_group(ctx, case, tet8=True):
    bg, new = case["bg"], case["new"]
    npn = new.np
    g = dict(xyz=ctx.upload(bg.xyz), triv=ctx.upload(bg.triv), adjt=ctx.upload(bg.adjt), hausd=case["hausd"],
             met=None if case["met"] is None else ctx.upload(case["met"]),
             fields=[ctx.upload(f) for f in case["fields"]], xyz_new=ctx.upload(new.xyz),
             pclass=ctx.upload(case["pclass"]),
             met_out=None if case["met"] is None else ctx.upload(np.full((npn, case["met"].shape[1]), np.nan)),
             fields_out=[ctx.upload(np.full((npn, f.shape[1]), np.nan)) for f in case["fields"]],
             elem_out=ctx.upload(np.zeros(npn, np.int32)), hit_out=ctx.upload(np.zeros(npn, np.int8)))
    if tet8:
        g["tet8"] = ctx.upload(pack_tet8(bg.tetv, bg.adja))
    else:
        g["tetv"], g["adja"] = ctx.upload(bg.tetv), ctx.upload(bg.adja)
    return g


def _download(g):
    return dict(met=None if g["met_out"] is None else g["met_out"].download(),
                fields=[f.download() for f in g["fields_out"]], elem=g["elem_out"].download(),
                hit=g["hit_out"].download())


def _same(a, b):
    np.testing.assert_array_equal(a["elem"], b["elem"])
    np.testing.assert_array_equal(a["hit"], b["hit"])
    for x, y in zip(([a["met"]] if a["met"] is not None else []) + a["fields"],
                    ([b["met"]] if b["met"] is not None else []) + b["fields"]):
        assert np.array_equal(x, y, equal_nan=True)


@pytest.fixture(scope="module")
def cases():
    return [make_case(**spec) for spec in GROUPS]


@pytest.fixture(scope="module")
def singles(cases):
    return [run_gpu(c, tet8=True) for c in cases]


@pytest.mark.gpu
@pytest.mark.parametrize("lanes", ["1", "2", "3"])
@pytest.mark.parametrize("sync", [True, False])
def test_groups_match_single_calls(cases, singles, lanes, sync, monkeypatch):
    monkeypatch.setenv("PMMG_HIP_GROUP_LANES", lanes)  # read by pmmg_hip_create
    with TransferContext(0) as ctx:
        gs = [_device_group(ctx, c, tet8=(i % 2 == 0)) for i, c in enumerate(cases)]
        for rep in range(2):  # the second call reuses the lanes and their buffers
            st = ctx.locate_interp_groups(gs, sync=sync)
            if not sync:
                ctx.sync()
            for case, g, one in zip(cases, gs, singles):
                out = _download(g)
                _same(out, one)
                rep_ = check(case, out)
                assert rep_["class_i"] == rep_["class_i_same"]
        if sync:
            assert st.nvol == sum(s["stats"]["nvol"] for s in singles)
            assert st.nbdy == sum(s["stats"]["nbdy"] for s in singles)
            assert st.steps_total == sum(s["stats"]["steps_total"] for s in singles)
            assert st.stepmax == max(s["stats"]["stepmax"] for s in singles)


@pytest.mark.gpu
def test_groups_invalid_group_reports_its_index(cases):
    with TransferContext(0) as ctx:
        gs = [_device_group(ctx, c) for c in cases[:3]]
        gs[2] = dict(gs[2], met=None, met_out=None, fields=[], fields_out=[])  # valid: nothing but locate
        bad = dict(gs[1])
        bad["fields_out"] = []  # two fields in, no outputs
        with pytest.raises(RuntimeError, match="group 1"):
            ctx.locate_interp_groups([gs[0], bad, gs[2]])
        ctx.sync()
        # the context stays usable
        ctx.locate_interp_groups(gs[:1])
        _same(_download(gs[0]), run_gpu(cases[0], tet8=True))


@pytest.mark.gpu
def test_groups_call_leaves_the_context_background(cases):
    """the groups call's lane 0 used to be the context itself, so a
    later single call ran against the last group's arrays.  The lanes are
    contexts of their own now: a single call after a groups call still uses
    the context's own (host-mode) background and solutions."""
    case = cases[1]
    with TransferContext(0) as ctx:
        bg = case["bg"]
        ctx.set_background(bg.xyz, bg.tetv, bg.adja, bg.triv, bg.adjt, case["hausd"])
        ctx.set_solutions(case["met"], case["fields"])
        gs = [_device_group(ctx, c) for c in cases[:3]]
        ctx.locate_interp_groups(gs, sync=True)
        new = case["new"]
        npn = new.np
        mo = np.full((npn, case["met"].shape[1]), np.nan)
        fo = [np.full((npn, f.shape[1]), np.nan) for f in case["fields"]]
        el, hit = np.zeros(npn, np.int32), np.zeros(npn, np.int8)
        ctx.locate_interp(new.xyz, case["pclass"], mo, fo, el, hit)
        out = dict(met=mo, fields=fo, elem=el, hit=hit)
        _same(out, run_gpu(case, tet8=False))
        rep = check(case, out)
        assert rep["class_i"] == rep["class_i_same"]


@pytest.mark.gpu
def test_groups_after_release_scratch(cases, singles):
    """pmmg_hip_release_scratch between calls: the lanes and the binning /
    snapshot scratch are re-created on demand, the outputs unchanged; a
    Morton-binned single call and a device adjacency build after it too."""
    with TransferContext(0) as ctx:
        gs = [_device_group(ctx, c) for c in cases]
        for rep in range(2):
            ctx.locate_interp_groups(gs, sync=True)
            for g, one in zip(gs, singles):
                _same(_download(g), one)
            ctx.release_scratch()
    case = cases[1]
    with TransferContext(0, sort=True) as ctx:
        a = run_gpu(case, ctx=ctx)
        ctx.release_scratch()
        b = run_gpu(case, ctx=ctx)
        _same(a, b)
        assert a["stats"]["sorted"] == 1 and b["stats"]["sorted"] == 1
        bg = case["bg"]
        tetv = ctx.upload(bg.tetv)
        adja, _ = ctx.build_adjacency(bg.np, tetv, adja=True, tet8=False)
        ctx.release_scratch()
        adja2, _ = ctx.build_adjacency(bg.np, tetv, adja=True, tet8=False)
        np.testing.assert_array_equal(adja.download(), bg.adja)
        np.testing.assert_array_equal(adja2.download(), bg.adja)
