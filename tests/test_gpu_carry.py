"""Carry-over of the new mesh into the next iteration (pmmg_hip_keep /
pmmg_hip_carry_over, C host layer pmmg_interp_metrics_and_fields_carry):
ParMmg's adapted groups become the next iteration's old groups
(src/libparmmg1.c:653 -> PMMG_update_oldGrps, src/grpsplit_pmmg.c:1224-1248).
The second iteration, fed from the rows kept on the device, must give outputs
bit-identical to a cold run that uploads everything, while uploading far
fewer bytes."""
import numpy as np
import pytest

from parity import make_case
from parmmg_amd import synth
from parmmg_amd.transfer import TAG_BDY, TAG_REQ, TransferContext, interp_metrics_and_fields

C = synth.CUBE


def _new_group(mesh, req_every=0):
    tag = np.where(mesh.isbdy == 1, TAG_BDY, 0).astype(np.uint16)
    if req_every:
        tag[::req_every] |= TAG_REQ
    return dict(xyz=mesh.xyz, tag=tag, tetv=mesh.tetv, met=np.full((mesh.np, 6), np.nan),
                fields=[np.full((mesh.np, k), np.nan) for k in (1, 3, 6)], ani=1,
                elem=np.zeros(mesh.np, np.int32), hit=np.zeros(mesh.np, np.int8))


class _Mesh:
    """an old group's mesh: the adapted mesh of the previous iteration
    (connectivity only: adjacency and boundary trias built on the device)"""

    def __init__(self, xyz, tetv):
        self.xyz, self.tetv = np.ascontiguousarray(xyz), np.ascontiguousarray(tetv, np.int32)
        self.np, self.ne, self.nt = self.xyz.shape[0], self.tetv.shape[0], 0
        self.adja = self.triv = self.adjt = None


def _old_from(mesh, g, hausd):
    return dict(mesh=mesh, met=g["met"], fields=g["fields"], hausd=hausd, device_adjacency=True,
                device_boundary=True)


def _outputs(g):
    return [g["met"]] + list(g["fields"]) + [g["elem"], g["hit"]]


@pytest.mark.gpu
@pytest.mark.parametrize("renumber", [False, True])
def test_second_iteration_from_kept_rows_is_bit_identical(renumber):
    case = make_case(kind=C, n_old=6, n_new=7, fields=(synth.F_SCALAR, synth.F_VECTOR, synth.F_TENSOR),
                     with_ref=False)
    B = case["new"]
    nxt = synth.lattice(C, 5, jitter=0.2, seed=synth.SEED + 7)
    old1 = dict(mesh=case["bg"], met=case["met"], fields=case["fields"], hausd=case["hausd"])
    with TransferContext(0) as ctx:
        # iteration 1 (cold), its new group kept on the device
        g1 = _new_group(B, req_every=9)
        ier, _ = interp_metrics_and_fields(ctx, [old1], [g1], input_met=1, carry=(False, None))
        assert ier == 1
        req = (g1["tag"] & TAG_REQ) != 0
        assert np.isnan(g1["met"][req]).all()
        # the host fills the skipped (MG_REQ) rows as PMMG_copyMetricsAndFields_point would
        g1["met"][req] = 1.0 + np.arange(req.sum())[:, None]
        for f in g1["fields"]:
            f[req] = -2.0
        # iteration 2: old group = the adapted mesh B with the rows just written
        xyz, tetv = B.xyz, B.tetv
        met, fields = g1["met"], g1["fields"]
        src = None
        if renumber:  # load balancing renumbered B and brought some vertices in from elsewhere
            rng = np.random.default_rng(5)
            p = rng.permutation(B.np)                # new vertex i = kept point p[i]
            inv = np.empty_like(p)
            inv[p] = np.arange(B.np)
            xyz, tetv = B.xyz[p], (inv[B.tetv - 1] + 1).astype(np.int32)
            met, fields = met[p].copy(), [f[p].copy() for f in fields]
            src = (p + 1).astype(np.int32)
            moved = rng.choice(B.np, 25, replace=False)
            src[moved] = 0                           # rows from the host, which differ from the kept ones
            met[moved] *= 1.5
            for f in fields:
                f[moved] += 0.25
        mesh2 = _Mesh(xyz, tetv)
        old2 = _old_from(mesh2, dict(met=met, fields=fields), case["hausd"])
        g2 = _new_group(nxt)
        ctx.bytes_up(reset=True)
        ier, st = interp_metrics_and_fields(ctx, [old2], [g2], input_met=1,
                                            carry=(True, None if src is None else [src]))
        assert ier == 1
        up_carried = ctx.bytes_up(reset=True)
    with TransferContext(0) as cold:
        g2c = _new_group(nxt)
        ier, stc = interp_metrics_and_fields(cold, [old2], [g2c], input_met=1)
        assert ier == 1
        up_cold = cold.bytes_up()
    for a, b in zip(_outputs(g2), _outputs(g2c)):
        assert np.array_equal(a, b, equal_nan=True)
    assert st.nvol == stc.nvol and st.nbdy == stc.nbdy and st.nvol > 0
    # the vertices and solution rows of the old group did not go up again,
    # but for the skipped (1 in 9) and moved-in (25) rows and the map
    rows = B.xyz.nbytes + met.nbytes + sum(f.nbytes for f in fields)
    assert up_carried <= up_cold - 0.7 * rows, (up_carried, up_cold, rows)


@pytest.mark.gpu
def test_carry_over_errors_and_dropped_slots():
    case = make_case(kind=C, n_old=5, n_new=6, fields=(synth.F_SCALAR,), with_ref=False)
    B = case["new"]
    with TransferContext(0) as ctx:
        with pytest.raises(RuntimeError, match="holds nothing"):
            ctx.carry_over(0, B.np)
        with pytest.raises(RuntimeError, match="keep"):
            ctx.keep(0)  # nothing to keep yet
        ctx.set_background(case["bg"].xyz, case["bg"].tetv, case["bg"].adja, case["bg"].triv, case["bg"].adjt,
                           case["hausd"])
        ctx.set_solutions(case["met"], case["fields"])
        mo, fo = np.zeros((B.np, 6)), [np.zeros((B.np, 1))]
        ctx.locate_interp(B.xyz, case["pclass"], mo, fo)
        ctx.keep(3)
        with pytest.raises(RuntimeError, match="without a map"):
            ctx.carry_over(3, B.np + 1)
        with pytest.raises(RuntimeError, match="out of"):
            ctx.carry_over(3, 4, np.array([1, 2, B.np + 1, 0], np.int32))
        ctx.carry_over(3, B.np)
        with pytest.raises(RuntimeError, match="armed carry-over is for"):
            ctx.set_background(case["bg"].xyz, case["bg"].tetv, None, None, None, case["hausd"])
        ctx.carry_over(3, 0)  # dropped
        with pytest.raises(RuntimeError, match="holds nothing"):
            ctx.carry_over(3, B.np)


@pytest.mark.gpu
def test_carry_consumes_its_slot_and_disarms_on_failure():
    """the identity carry swaps the kept vertex buffer into the
    background, so the slot is consumed at once — a later carry of it fails
    instead of feeding the previous background's vertices; an armed carry
    rejects set_solutions_packed; a failed armed call disarms."""
    from parmmg_amd.transfer import pack_solutions
    case = make_case(kind=C, n_old=5, n_new=6, fields=(synth.F_SCALAR,), with_ref=False)
    B = case["new"]
    bg = case["bg"]
    with TransferContext(0) as ctx:
        def first_iteration():
            ctx.set_background(bg.xyz, bg.tetv, bg.adja, bg.triv, bg.adjt, case["hausd"])
            ctx.set_solutions(case["met"], case["fields"])
            ctx.locate_interp(B.xyz, case["pclass"], np.zeros((B.np, 6)), [np.zeros((B.np, 1))])
            ctx.keep(1)

        first_iteration()
        mo, fo = np.zeros((B.np, 6)), [np.zeros((B.np, 1))]
        ctx.carry_over(1, B.np)
        ctx.set_background(B.xyz, B.tetv, None, None, None, case["hausd"])  # takes the slot's vertices
        with pytest.raises(RuntimeError, match="carry-over is armed"):
            ctx.set_solutions_packed(pack_solutions(mo, fo), 6, [1])
        with pytest.raises(RuntimeError, match="holds nothing"):
            ctx.carry_over(1, B.np)  # consumed by the set_background above
        # disarmed: a plain set_solutions uploads again and the context works
        ctx.set_solutions(mo, fo)
        first_iteration()
        ctx.carry_over(1, B.np)
        with pytest.raises(RuntimeError, match="armed carry-over is for"):
            ctx.set_background(B.xyz[:-1].copy(), B.tetv, None, None, None, case["hausd"])  # wrong size: disarms
        # disarmed without touching the slot: plain host calls work, and the
        # slot can still be carried
        ctx.set_background(bg.xyz, bg.tetv, bg.adja, bg.triv, bg.adjt, case["hausd"])
        ctx.set_solutions(case["met"], case["fields"])
        ctx.carry_over(1, B.np)
        ctx.carry_over(1, 0)  # dropped (its buffers freed)
        with pytest.raises(RuntimeError, match="holds nothing"):
            ctx.carry_over(1, B.np)
