"""Output records (pmmg_hip_locate_interp_rec): the new points' values
written as records of the packed input layout, [metric | field 0 | ...] per
point — the layout a resident ParMmg pipeline keeps across iterations (the
records a step writes are the next background's records).  Every record
must equal, bit for bit, the rows pmmg_hip_locate_interp writes into the
per-solution arrays, in every query order and gather mode; what the
reference leaves untouched (skipped points, failed MMG5_invmat rows) keeps
the caller's previous content."""
import numpy as np
import pytest

from parity import invmat_failure_case, make_case
from parmmg_amd import synth
from parmmg_amd.transfer import TransferContext, pack_solutions, pack_tet8

# the packed records hold at most 16 doubles per vertex: aniso metric + scalar + vector + tensor
PACKABLE = (synth.F_SCALAR, synth.F_VECTOR, synth.F_TENSOR)
SENT = np.frombuffer(np.uint64(0x7FF4A5A5A5A5A5A5).tobytes(), np.float64)[0]  # a NaN no arithmetic makes


def _both(case, sort=None, env=None):
    """arrays-out and records-out runs of the same packed-input transfer"""
    import os
    bg, new = case["bg"], case["new"]
    met, fields = case["met"], case["fields"]
    sizes = ([met.shape[1]] if met is not None else []) + [f.shape[1] for f in fields]
    RS = (sum(sizes) + 1) & ~1
    saved = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        ctx = TransferContext(0, sort=sort)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    with ctx:
        d = [ctx.upload(bg.xyz), ctx.upload(pack_tet8(bg.tetv, bg.adja)), ctx.upload(bg.triv), ctx.upload(bg.adjt)]
        rec = ctx.upload(pack_solutions(met, fields))
        q, pc = ctx.upload(new.xyz), ctx.upload(case["pclass"])
        n = new.np
        ctx.set_background_tet8(d[0], d[1], d[2], d[3], case["hausd"])
        ctx.set_solutions_packed(rec, 0 if met is None else met.shape[1], [f.shape[1] for f in fields])
        outs = [ctx.upload(np.full((n, s), SENT)) for s in sizes]
        el, hit = ctx.upload(np.zeros(n, np.int32)), ctx.upload(np.zeros(n, np.int8))
        st = ctx.locate_interp(q, pc, outs[0] if met is not None else None, outs[1:] if met is not None else outs,
                               el, hit)
        a = dict(rows=[o.download() for o in outs], elem=el.download(), hit=hit.download(), stats=st.as_dict())
        ro = ctx.upload(np.full((n, RS), SENT))
        el2, hit2 = ctx.upload(np.zeros(n, np.int32)), ctx.upload(np.zeros(n, np.int8))
        ctx.locate_interp_rec(q, pc, ro, el2, hit2)
        r = ro.download()
        b = dict(rows=[], elem=el2.download(), hit=hit2.download())
        o = 0
        for s in sizes:
            b["rows"].append(np.ascontiguousarray(r[:, o:o + s]))
            o += s
        pad = r[:, o:]
    return a, b, pad


def _same(a, b):
    np.testing.assert_array_equal(a["elem"], b["elem"])
    np.testing.assert_array_equal(a["hit"], b["hit"])
    for x, y in zip(a["rows"], b["rows"]):
        assert np.array_equal(x.view(np.uint64), y.view(np.uint64))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["input", "morton", "input-2pass", "morton-2pass"])
@pytest.mark.parametrize("spec", [dict(kind=synth.CUBE, n_old=6, n_new=7, fields=PACKABLE),
                                  dict(kind=synth.SHELL, n_old=8, n_new=12, req_every=9, fields=PACKABLE),
                                  dict(kind=synth.CUBE, n_old=7, n_new=9, metric=synth.F_ISO,
                                       fields=(synth.F_SCALAR,)),
                                  dict(kind=synth.CUBE, n_old=5, n_new=8, metric=synth.F_ISO,
                                       fields=(synth.F_SCALAR, synth.F_VECTOR, synth.F_TENSOR))])
def test_records_equal_arrays(spec, mode):
    case = make_case(**spec, with_ref=False)
    sort = mode.startswith("morton")
    env = {"PMMG_HIP_PACKPASS": "2" if mode.endswith("2pass") else "1"}
    a, b, pad = _both(case, sort=sort, env=env)
    _same(a, b)
    skipped = case["pclass"] == 0
    for x in b["rows"]:  # skipped points' records untouched
        assert np.all(x[skipped].view(np.uint64) == np.uint64(0x7FF4A5A5A5A5A5A5))
    assert np.all(pad.view(np.uint64) == np.uint64(0x7FF4A5A5A5A5A5A5))  # the record's padding double


@pytest.mark.gpu
def test_records_leave_failed_inversions_untouched():
    case, vol, srf = invmat_failure_case()
    a, b, _ = _both(case)
    _same(a, b)
    # the metric (slot 0) and the tensor field (slot 3) rows of both points stay at the sentinel
    for i in (vol, srf):
        assert np.all(b["rows"][0][i].view(np.uint64) == np.uint64(0x7FF4A5A5A5A5A5A5))
        assert np.all(b["rows"][3][i].view(np.uint64) == np.uint64(0x7FF4A5A5A5A5A5A5))
        assert not np.isnan(b["rows"][1][i]).any()  # the scalar row is written


@pytest.mark.gpu
def test_records_need_packed_input():
    case = make_case(kind=synth.CUBE, n_old=4, n_new=5, with_ref=False)
    with TransferContext(0) as ctx:
        bg = case["bg"]
        ctx.set_background(ctx.upload(bg.xyz), ctx.upload(bg.tetv), ctx.upload(bg.adja), ctx.upload(bg.triv),
                           ctx.upload(bg.adjt), case["hausd"])
        ctx.set_solutions(ctx.upload(case["met"]), [ctx.upload(f) for f in case["fields"]])
        n = case["new"].np
        with pytest.raises(RuntimeError, match="packed input records"):
            ctx.locate_interp_rec(ctx.upload(case["new"].xyz), ctx.upload(case["pclass"]),
                                  ctx.empty((n, 16), np.float64))
