"""Every BASELINE.json config through the HIP module, checked against the
oracle (runs on the MI355X).

* cfg1: the reference's own libexamples cube (tests/golden/cube_refine8.npz,
  made by tests/golden/make_golden.py from cube.mesh / cube-met.sol /
  cube-solphys.sol) and the aniso lattice fixture: the module against the
  committed oracle outputs.
* cfg2 (1M tetra) and cfg3 (20M tetra): every point, against a full oracle run
  in the reference's visitation order.
* cfg4 (100M-tetra shell, the bench config) and cfg5 (500M-tetra cube): the
  full-size module run, checked on a contiguous range of the reference's
  visitation order (the oracle walks it with its warm start, like one rank).

Contract (tests/parity.py): class (i) points in the identical tetra, every
chosen element accepted by the reference's test for its hit kind, values of
the reference interpolator in it within 1e-12 relative (and the bit-exact
count reported), identical values wherever the oracle chose the same element.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O
from parity import check, run_dev
from parmmg_amd import configs, synth
from parmmg_amd.synth import Mesh
from parmmg_amd.transfer import TransferContext

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
THREADS = min(16, os.cpu_count() or 1)


def _check_against(B, new_xyz, pc, gpu, ref, idx):
    """oracle.check_batch over idx (0-based) + identical values where the
    oracle chose the same element and hit kind; asserts the contract."""
    rep = O.check_batch(B, new_xyz, pc, gpu["elem"], gpu["hit"], gpu["met"], gpu["fields"], idx=idx, ref=ref,
                        threads=THREADS)
    same = (gpu["elem"][idx] == ref["elem"][idx]) & ((gpu["hit"][idx] & 15) == (ref["hit"][idx] & 15))
    ident = np.ones(idx.shape[0], bool)
    for a, b in zip(([gpu["met"]] if gpu["met"] is not None else []) + gpu["fields"],
                    ([ref["met"]] if ref["met"] is not None else []) + ref["fields"]):
        ident &= np.all((a[idx] == b[idx]) | (np.isnan(a[idx]) & np.isnan(b[idx])), axis=1)
    rep["same_element"] = int(same.sum())
    rep["same_element_identical"] = int((same & ident).sum())
    print(rep)
    assert rep["unprocessed"] == 0 and rep["accept_fail"] == 0 and rep["value_fail"] == 0, rep
    assert rep["n"] == idx.shape[0]
    assert rep["class_i"] > 0 and rep["class_i"] == rep["class_i_same"], rep
    assert rep["maxrel"] <= 1e-12
    assert rep["same_element"] == rep["same_element_identical"], rep
    return rep


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cube_refine8", "lattice_4_5_aniso"])
def test_golden_fixture_on_gpu(name):
    """cfg1: the reference's libexamples cube (and the aniso lattice fixture)
    through the module; outputs against the committed oracle outputs."""
    g = np.load(os.path.join(GOLD, f"{name}.npz"))
    bg = Mesh(0, 0, g["bg_xyz"], g["bg_tetv"], g["bg_adja"], g["bg_triv"], g["bg_adjt"], None)
    new = Mesh(0, 0, g["new_xyz"], np.zeros((0, 4), np.int32), np.zeros((0, 4), np.int32),
               np.zeros((0, 3), np.int32), np.zeros((0, 3), np.int32), None)
    fields = [g[f"field{j}"] for j in range(int(g["nfield"]))]
    met = g["met"]
    ref = dict(elem=g["out_elem"], hit=g["out_hit"], minbary=g["out_minbary"], met=g["out_met"],
               fields=[g[f"out_field{j}"] for j in range(len(fields))])
    B = O.Background(bg, met, fields, 0.01)
    case = dict(bg=bg, new=new, met=met, fields=fields, pclass=g["pclass"], B=B, hausd=0.01, ref=ref)
    for tet8 in (False, True):
        from parity import run_gpu
        gpu = run_gpu(case, tet8=tet8)
        rep = check(case, gpu)
        print(name, tet8, rep, gpu["stats"])
        assert rep["n"] == int((g["pclass"] != 0).sum())
        assert rep["class_i"] == rep["class_i_same"]
        # same element and hit kind as the committed oracle output -> same bits
        same = (gpu["elem"] == ref["elem"]) & ((gpu["hit"] & 15) == (ref["hit"] & 15)) & (g["pclass"] != 0)
        assert same.any()
        for a, b in zip([gpu["met"]] + gpu["fields"], [ref["met"]] + ref["fields"]):
            assert np.array_equal(a[same], b[same], equal_nan=True)


def _config_parity(w, sample: int = 0):
    """The config's full-size workload (bench.py's synthetic meshes and
    solutions) through the module, checked against an oracle run over the
    reference's visitation order (a contiguous range of it when sample > 0)."""
    bg, new = configs.build_meshes(w, seed=synth.SEED, with_new_tetra=True)
    visit = synth.visit_order(new)
    pc = synth.classes(new)
    new_xyz = new.xyz
    del new  # the new tetra are only needed for the visitation order
    if sample and visit.shape[0] > sample:
        s0 = visit.shape[0] // 3
        visit = np.ascontiguousarray(visit[s0:s0 + sample])
    met = synth.solution(w.metric, bg.xyz)
    fields = [synth.solution(f, bg.xyz) for f in w.fields]
    with TransferContext(0) as ctx:
        mo, fo, el, hit, st = run_dev(ctx, bg, new_xyz, met, fields, pc, w.hausd)
    gpu = dict(met=mo, fields=fo, elem=el, hit=hit)
    act = pc != 0
    assert ((hit & 15) != 0).sum() == act.sum() and ((hit & 15)[~act] == 0).all()
    B = O.Background(bg, met, fields, w.hausd)
    ref = O.run(B, new_xyz, pc, visit, O.MODE_FRESH, threads=THREADS)
    idx = np.nonzero(ref["hit"] != 0)[0].astype(np.int32)
    assert idx.shape[0] == int(act[visit - 1].sum())
    rep = _check_against(B, new_xyz, pc, gpu, ref, idx)
    print(w.name, "stats", st.as_dict())
    return rep, st


@pytest.mark.gpu
def test_cfg2_full_size_every_point():
    """cfg2 (1M-tetra cube, iso metric + scalar): every point of the module's
    run against a full oracle run."""
    rep, st = _config_parity(configs.CFG2)
    assert rep["n"] > 200_000


@pytest.mark.gpu
def test_cfg3_full_size_every_point():
    """cfg3 (20M-tetra cube, aniso metric + 3 fields): every point, with the
    class (i) identity asserted at size."""
    rep, st = _config_parity(configs.CFG3)
    assert rep["n"] > 4_000_000


@pytest.mark.gpu
def test_cfg4_full_size_visit_range():
    """cfg4 (100M-tetra shell, the bench config): the full-size run checked on
    a 1M-point range of the reference's visitation order."""
    rep, st = _config_parity(configs.CFG4, sample=1_000_000)
    assert rep["n"] > 900_000 and st.nbdy > 0


@pytest.mark.gpu
@pytest.mark.skipif(os.environ.get("PMMG_TEST_CFG5", "1") == "0", reason="PMMG_TEST_CFG5=0")
def test_cfg5_full_size_visit_range():
    """cfg5 (500M-tetra cube, iso metric + 5 fields): the full-size run on one
    GPU checked on a 300k-point range of the reference's visitation order."""
    rep, st = _config_parity(configs.CFG5, sample=300_000)
    assert rep["n"] > 250_000


@pytest.mark.gpu
def test_cfgG_graded_full_size_visit_range():
    """cfgG: cfg3's lattices graded 1000x towards three planes (the new mesh's
    planes moved against the background's) and sheared — elements from ~1:1
    to ~1000:1, the geometry of the reference's anisotropic torus-with-shock
    runs.  The full-size module run, checked on a 1M-point range of the
    reference's visitation order (the oracle runs ~30k points/s per 8 threads
    on this mesh: every point would take minutes); the fp32 filter walk's
    hand-overs to the exact walk (nvol_exact) stay a small fraction: its
    margin holds on these elements."""
    rep, st = _config_parity(configs.CFGG, sample=1_000_000)
    assert rep["n"] > 900_000
    print("cfgG nvol_exact", st.nvol_exact, "stepmax", st.stepmax, "steps/pt",
          st.steps_total / max(1, st.nvol + st.nbdy))
    assert st.nvol_exact < 0.01 * st.nvol


@pytest.mark.gpu
def test_cfg3_shuffled_numbering_auto_order():
    """cfg3's new points shuffled: the coherence test picks the Morton order,
    which (below 2^23 queries) runs beside the input order's lists on a
    stream of its own, each order with its own volume / surface launch.  Every
    point is located, and a point located in the same element as in the
    input-order call gets bit-identical rows."""
    w = configs.CFG3
    bg, new = configs.build_meshes(w, seed=synth.SEED, with_new_tetra=False)
    pc = synth.classes(new)
    met = synth.solution(w.metric, bg.xyz)
    fields = [synth.solution(f, bg.xyz) for f in w.fields]
    perm = np.random.default_rng(7).permutation(new.np)
    with TransferContext(0) as ctx:
        a = run_dev(ctx, bg, new.xyz, met, fields, pc, w.hausd)
        b = run_dev(ctx, bg, np.ascontiguousarray(new.xyz[perm]), met, fields, np.ascontiguousarray(pc[perm]),
                    w.hausd)
    assert a[4].sorted == 0 and b[4].sorted == 1
    inv = np.argsort(perm)
    el_b, hit_b = b[2][inv], b[3][inv]
    act = pc != 0
    assert ((hit_b & 15) != 0).sum() == act.sum()
    same = act & (a[2] == el_b) & (a[3] == hit_b)
    assert same.sum() > 0.99 * act.sum()
    for x, y in zip([a[0]] + a[1], [b[0]] + b[1]):
        assert np.array_equal(x[same].view(np.uint64), y[inv][same].view(np.uint64))


@pytest.mark.gpu
def test_split_volume_stage_bit_identical_to_fused(monkeypatch):
    """The split volume stage (PMMG_HIP_VOLSPLIT=1: a walk kernel writing
    located records, an interpolation kernel per chunk on its own stream —
    measured slower than the fused kernel and not the default)
    gives the fused kernel's outputs bit for bit, in input order and in the
    Morton order of a shuffled numbering, with the reference's arrays and
    with packed records."""
    w = configs.CFG3
    bg, new = configs.build_meshes(w, seed=synth.SEED, with_new_tetra=False)
    pc = synth.classes(new)
    met = synth.solution(w.metric, bg.xyz)
    fields = [synth.solution(f, bg.xyz) for f in w.fields]
    perm = np.random.default_rng(11).permutation(new.np)
    orders = [(new.xyz, pc), (np.ascontiguousarray(new.xyz[perm]), np.ascontiguousarray(pc[perm]))]
    res = {}
    for split in ("0", "1"):
        monkeypatch.setenv("PMMG_HIP_VOLSPLIT", split)
        monkeypatch.setenv("PMMG_HIP_VOLCHUNKS", "3")
        with TransferContext(0) as ctx:
            res[split] = [run_dev(ctx, bg, q, met, fields, c, w.hausd) for q, c in orders]
            res[split].append(run_dev(ctx, bg, new.xyz, met, fields, pc, w.hausd, packed=True))
    for a, b in zip(res["0"], res["1"]):
        assert a[4].sorted == b[4].sorted
        assert np.array_equal(a[2], b[2]) and np.array_equal(a[3], b[3])
        wr = (a[3] & 15) != 0
        assert wr.sum() == (pc != 0).sum()
        for x, y in zip([a[0]] + a[1], [b[0]] + b[1]):
            assert np.array_equal(x[wr].view(np.uint64), y[wr].view(np.uint64))
    assert res["0"][1][4].sorted == 1
