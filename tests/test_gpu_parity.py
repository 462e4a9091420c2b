"""Parity of the HIP module with the CPU oracle (runs on the MI355X).

Sizes are chosen so the oracle's per-point checks finish in seconds; the
contract is documented in tests/parity.py."""
import numpy as np
import pytest

from parity import check, invmat_failure_case, make_case, run_gpu
from parmmg_amd import synth

C, S = synth.CUBE, synth.SHELL

CASES = {
    "cube-ani-6-7": dict(kind=C, n_old=6, n_new=7),
    "cube-iso-req-8-11": dict(kind=C, n_old=8, n_new=11, metric=synth.F_ISO,
                              fields=(synth.F_SCALAR, synth.F_AFFINE), req_every=7),
    "shell-ani-8-12": dict(kind=S, n_old=8, n_new=12),
    "shell-iso-12-16": dict(kind=S, n_old=12, n_new=16, metric=synth.F_ISO, fields=(synth.F_SCALAR,)),
    "cube-jitterbg-10-13": dict(kind=C, n_old=10, n_new=13, jitter_old=0.15),
    "cube-nomet-tensor-5-9": dict(kind=C, n_old=5, n_new=9, metric=None, fields=(synth.F_TENSOR, synth.F_AFFINE_VEC)),
    "cube-coarse-new-9-4": dict(kind=C, n_old=9, n_new=4),
}


def _packable(case):
    """metric + fields of at most 16 doubles, no tensor across doubles 8/9, a
    compiled layout (pick_layout in pmmg_hip.hip)"""
    sizes = ([case["met"].shape[1]] if case["met"] is not None else []) + [f.shape[1] for f in case["fields"]]
    return tuple(sizes) in {(6, 1, 3, 6), (1, 1), (1, 1, 1, 1, 1, 1), (1, 1, 1), (6,), (1,), (6, 1)}


def _packed_variant(case):
    """the same geometry and metric with trailing fields dropped until the slot
    layout has a packed-record kernel (the default cases carry 17 doubles)"""
    from oracle import oracle as O
    c = dict(case, fields=list(case["fields"]))
    while c["fields"] and not _packable(c):
        c["fields"].pop()
    assert _packable(c), "no packable prefix"
    c["B"] = O.Background(c["bg"], c["met"], c["fields"], c["hausd"])
    return c


# the shipped paths: query order chosen on the device, forced Morton bins,
# forced input order; separate tetv/adja arrays or packed tet8 records
# (morton-fine: the fine binning cells auto mode picks for a numbering
# without coherence)
FINE = {"PMMG_HIP_BINBITS": "7"}
ONEPASS = {"PMMG_HIP_PACKPASS": "1"}  # packed records in one gather pass (the default picks by record size)
MODES = {"auto": {}, "morton": dict(sort=True), "nosort": dict(sort=False), "tet8": dict(tet8=True),
         "tet8-morton": dict(tet8=True, sort=True), "packed": dict(tet8=True, packed=True, env=ONEPASS),
         "packed-morton": dict(tet8=True, packed=True, sort=True, env=ONEPASS),
         "morton-fine": dict(sort=True, env=FINE), "packed-morton-fine": dict(tet8=True, packed=True, sort=True,
                                                                              env={**FINE, **ONEPASS}),
         # packed records gathered in two passes over the record halves (PMMG_HIP_PACKPASS=2)
         "packed2": dict(tet8=True, packed=True, env={"PMMG_HIP_PACKPASS": "2"}),
         "packed2-morton": dict(tet8=True, packed=True, sort=True, env={"PMMG_HIP_PACKPASS": "2"})}


@pytest.mark.gpu
@pytest.mark.parametrize("mode", sorted(MODES))
@pytest.mark.parametrize("name", sorted(CASES))
def test_parity_small(name, mode):
    case = make_case(**CASES[name])
    if MODES[mode].get("packed") and not _packable(case):
        # no packed-record kernel for this slot layout: refused, never computed another way
        with pytest.raises(RuntimeError, match="slot layout not supported"):
            run_gpu(case, **MODES[mode])
        case = _packed_variant(case)
    gpu = run_gpu(case, **MODES[mode])
    rep = check(case, gpu)
    print(name, mode, rep, gpu["stats"])
    assert rep["n"] == int((case["pclass"] != 0).sum())
    assert rep["class_i"] == rep["class_i_same"]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["auto", "morton"])
def test_fallback_paths_outside_domain(mode):
    """Points pushed outside the background make the walks get stuck; the
    exhaustive / closest kernels must reproduce the reference semantics."""
    case = make_case(kind=C, n_old=5, n_new=6, with_ref=False)
    new = case["new"]
    rng = np.random.default_rng(7)
    vol = np.nonzero(case["pclass"] == 1)[0]
    bdy = np.nonzero(case["pclass"] == 2)[0]
    pick_v = rng.choice(vol, 10, replace=False)
    pick_b = rng.choice(bdy, 10, replace=False)
    new.xyz[pick_v, 0] = 1.0 + rng.uniform(0.001, 0.2, 10)   # outside the cube: closest tetra
    new.xyz[pick_b[:5], 2] = -0.05                            # beyond hausd: exhaustive -> stale/closest
    new.xyz[pick_b[5:], 2] = -0.004                           # within hausd of the bottom face
    case["B"] = __import__("oracle.oracle", fromlist=["Background"]).Background(
        case["bg"], case["met"], case["fields"], case["hausd"])
    gpu = run_gpu(case, **MODES[mode])
    rep = check(case, gpu)
    print(rep, gpu["stats"])
    assert gpu["stats"]["nvol_closest"] + gpu["stats"]["nvol_exhaust"] >= 1


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["auto", "morton-fine", "packed"])
def test_invmat_failures_leave_rows_untouched(mode):
    """Every MMG5_invmat failure path of the reference's interpolators
    leaves the output row untouched (src/interpmesh_pmmg.c:98-107, 177-187,
    258-267): the oracle's rows stay at their NaN sentinel exactly where
    invmat returned 0, and the GPU's rows are identical (check() compares
    every point bit for bit, NaN with NaN)."""
    case, vol, srf = invmat_failure_case()
    gpu = run_gpu(case, **MODES[mode])
    rep = check(case, gpu)
    print(rep, gpu["stats"])
    skip = case["pclass"] == 0
    met_nan = np.isnan(gpu["met"]).all(axis=1) & ~skip
    ten_nan = np.isnan(gpu["fields"][2]).all(axis=1) & ~skip
    assert met_nan.sum() > 2 and ten_nan.sum() > 2
    for f in gpu["fields"][:2]:  # scalar and vector fields never fail
        assert not np.isnan(f[~skip]).any()
    # the final inversion's failure at both midpoints (volume and surface edge)
    assert met_nan[vol] and ten_nan[vol] and met_nan[srf] and ten_nan[srf]
    code = gpu["hit"].astype(np.int32) & 15
    assert code[vol] == 1 and code[srf] == 5  # VOL_WALK, BDY_EDGE
    # the vertex-tensor failures reach volume, surface-face and surface-edge hits
    for h in (1, 4, 5):
        assert (met_nan & (code == h)).any(), h


@pytest.mark.gpu
@pytest.mark.parametrize("device_built", [False, True])
def test_host_layer_groups_and_hsiz(device_built):
    """C host layer (PMMG_interpMetricsAndFields mirror): two groups, REQ
    points skipped, hsiz > 0 replaces the metric by a constant.  With
    device_built the adjacency and the boundary trias are not handed over:
    the module builds them on the device (MMG3D_hashTetra / MMG5_chkBdryTria
    results), with identical outputs."""
    from parmmg_amd.transfer import TAG_BDY, TAG_REQ, TransferContext, interp_metrics_and_fields

    olds, news, cases = [], [], []
    for n_old, n_new in ((5, 6), (6, 5)):
        case = make_case(kind=C, n_old=n_old, n_new=n_new, with_ref=False)
        new = case["new"]
        tag = np.where(new.isbdy == 1, TAG_BDY, 0).astype(np.uint16)
        tag[::11] |= TAG_REQ
        olds.append(dict(mesh=case["bg"], met=case["met"], fields=case["fields"], hausd=case["hausd"],
                         device_adjacency=device_built, device_boundary=device_built))
        met = np.full((new.np, 6), np.nan)
        fs = [np.full((new.np, f.shape[1]), np.nan) for f in case["fields"]]
        news.append(dict(xyz=new.xyz, tag=tag, tetv=new.tetv, met=met, fields=fs, ani=1,
                         elem=np.zeros(new.np, np.int32), hit=np.zeros(new.np, np.int8)))
        cases.append(case)
    with TransferContext(0) as ctx:
        ier, st = interp_metrics_and_fields(ctx, olds, news, input_met=1)
        assert ier == 1
        for case, g in zip(cases, news):
            req = (g["tag"] & TAG_REQ) != 0
            assert np.isnan(g["met"][req]).all()
            case["pclass"] = np.where(req, 0, np.where(case["new"].isbdy == 1, 2, 1)).astype(np.uint8)
            rep = check(case, dict(met=g["met"], fields=g["fields"], elem=g["elem"], hit=g["hit"]))
            assert rep["n"] == int((~req).sum())
        # hsiz > 0: constant metric, fields still interpolated
        for g in news:
            g["met"][:] = np.nan
            g["hsiz"], g["hmax"] = 0.04, 0.05
        ier, st = interp_metrics_and_fields(ctx, olds, news, input_met=1)
        assert ier == 1
        for g in news:
            np.testing.assert_array_equal(g["met"][:, 0], np.full(g["met"].shape[0], 1.0 / 0.04 ** 2))
            np.testing.assert_array_equal(g["met"][:, 1], 0.0)
        # hsiz above hmax: MMG5_Compute_constantSize's mismatched options -> the call fails
        for g in news:
            g["hsiz"], g["hmax"] = 0.05, 0.04
        ier, st = interp_metrics_and_fields(ctx, olds, news, input_met=1)
        assert ier == 0


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cube-ani-6-7", "shell-ani-8-12", "cube-jitterbg-10-13", "cube-nomet-tensor-5-9"])
def test_filter_walk_vs_exact_walk(name, monkeypatch):
    """PMMG_HIP_FILTER_STEPS=0 (test-only) hands every volume query straight
    to the exact fp64 walk (k_vol_walk_exact); both paths meet the contract,
    locate every class (i) point in the same tetra, and give bit-identical
    values wherever they chose the same tetra."""
    case = make_case(**CASES[name])
    outs = {}
    for val in ("0", None):
        if val is None:
            monkeypatch.delenv("PMMG_HIP_FILTER_STEPS", raising=False)
        else:
            monkeypatch.setenv("PMMG_HIP_FILTER_STEPS", val)  # read by pmmg_hip_create
        outs[val] = run_gpu(case, tet8=True)
        rep = check(case, outs[val])
        assert rep["n"] == int((case["pclass"] != 0).sum()) and rep["class_i"] == rep["class_i_same"]
    a, b = outs["0"], outs[None]
    assert a["stats"]["nvol_exact"] == a["stats"]["nvol"]
    same = a["elem"] == b["elem"]
    assert same.mean() > 0.99
    for x, y in zip(([a["met"]] if a["met"] is not None else []) + a["fields"],
                    ([b["met"]] if b["met"] is not None else []) + b["fields"]):
        assert np.array_equal(x[same], y[same], equal_nan=True)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cube-ani-6-7", "shell-ani-8-12", "cube-jitterbg-10-13", "shell-iso-12-16"])
def test_packed_records_bit_identical(name):
    """Packed per-vertex solution records give bit-identical outputs to the
    one-array-per-solution layout (same kernels' arithmetic, other gathers)."""
    case = make_case(**dict(CASES[name], fields=(synth.F_SCALAR, synth.F_VECTOR, synth.F_TENSOR))
                     if CASES[name].get("metric", synth.F_ANI) == synth.F_ANI else CASES[name], with_ref=False)
    assert _packable(case)
    a = run_gpu(case, tet8=True)
    for env in (ONEPASS, {"PMMG_HIP_PACKPASS": "2"}, {}):  # one gather per record, one per half, by size
        b = run_gpu(case, tet8=True, packed=True, env=env)
        np.testing.assert_array_equal(a["elem"], b["elem"])
        np.testing.assert_array_equal(a["hit"], b["hit"])
        for x, y in zip(([a["met"]] if a["met"] is not None else []) + a["fields"],
                        ([b["met"]] if b["met"] is not None else []) + b["fields"]):
            assert np.array_equal(x, y, equal_nan=True)
