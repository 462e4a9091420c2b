"""Halo-sharded background (parmmg_amd/shard.py, csrc/pmmg_shard.c).

Each rank of a Morton split transfers its points against the halo shard of
the background around its range; mapped back to group ids, the union of the
ranks' results must satisfy the same parity contract (tests/parity.py) as a
transfer against the whole group: identical tetra for class (i) points,
accepted elements otherwise, reference values in the chosen element.
The CPU cases run the oracle on the shards; the GPU case runs the HIP module.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O
from parity import check, make_case
from parmmg_amd import ranks, shard, synth

BDY_CODES = set(range(4, 12))


def _shards(case, world, halo=shard.DEFAULT_HALO, mode="box"):
    """mode box: Morton ranges, each against its range's box; cells: Morton
    ranges against the cells of their points; rcb: bench.py's default split
    (recursive coordinate bisection) against the cells of its points"""
    new, pc = case["new"], case["pclass"]
    split = ranks.rcb_shards if mode == "rcb" else ranks.morton_shards
    for mine in split(new.xyz, pc, world):
        if mode == "rcb":
            mode_ = "cells"
        else:
            mode_ = mode
        if mode_ == "cells":
            yield mine, shard.halo_shard_cells(case["bg"], new.xyz[mine], halo, hausd=case["hausd"])
        else:
            lo, hi = shard.range_box(new.xyz[mine])
            yield mine, shard.halo_shard(case["bg"], lo, hi, halo)


def _empty_result(case):
    npn = case["new"].np
    return dict(met=None if case["met"] is None else np.full((npn, case["met"].shape[1]), np.nan),
                fields=[np.full((npn, f.shape[1]), np.nan) for f in case["fields"]],
                elem=np.zeros(npn, np.int32), hit=np.zeros(npn, np.int8))


def _scatter(full, mine, sh, met, fields, elem, hit):
    code = hit.astype(np.int32) & 15
    is_tria = np.isin(code, list(BDY_CODES))
    full["elem"][mine] = sh.to_group_elem(elem, is_tria)
    full["hit"][mine] = hit
    if met is not None:
        full["met"][mine] = met
    for f, g in zip(full["fields"], fields):
        f[mine] = g


def test_shard_of_everything_is_the_group():
    bg = synth.lattice(synth.SHELL, 8)
    lo, hi = bg.xyz.min(axis=0), bg.xyz.max(axis=0)
    sh = shard.halo_shard(bg, lo, hi, 0.0)
    m = sh.mesh
    for a, b in ((m.xyz, bg.xyz), (m.tetv, bg.tetv), (m.adja, bg.adja), (m.triv, bg.triv), (m.adjt, bg.adjt)):
        assert np.array_equal(a, b)
    assert np.array_equal(sh.tet_gid, np.arange(1, bg.ne + 1))


@pytest.mark.parametrize("kind,n", [(synth.CUBE, 7), (synth.SHELL, 12)])
def test_shard_structure(kind, n):
    bg = synth.lattice(kind, n)
    lo, hi = np.array([-0.1, -0.2, 0.0]), np.array([0.35, 0.3, 0.6])
    sh = shard.halo_shard(bg, lo, hi)
    m = sh.mesh
    assert 0 < m.ne < bg.ne and np.all(np.diff(sh.tet_gid) > 0) and np.all(np.diff(sh.vert_gid) > 0)
    # connectivity and coordinates are the group's, renumbered
    assert np.array_equal(sh.vert_gid[m.tetv - 1], bg.tetv[sh.tet_gid - 1])
    assert np.array_equal(m.xyz, bg.xyz[sh.vert_gid - 1])
    assert np.array_equal(sh.vert_gid[m.triv - 1], bg.triv[sh.tria_gid - 1])
    # adjacency: symmetric, the group's where the neighbour is kept, 0 across the cut
    a = m.adja
    k, f = np.nonzero(a > 0)
    nb, nf = a[k, f] // 4 - 1, a[k, f] % 4
    assert np.array_equal(a[nb, nf], 4 * (k + 1) + f)
    assert np.array_equal(sh.tet_gid[nb], bg.adja[sh.tet_gid[k] - 1, f] // 4)
    cut = (a == 0) & (bg.adja[sh.tet_gid - 1] > 0)
    assert cut.any()
    # every kept tetra meets the grown box; every tetra meeting the box is kept
    box = lambda xyz, tv: (xyz[tv - 1].min(axis=1), xyz[tv - 1].max(axis=1))
    tl, th = box(bg.xyz, bg.tetv)
    meets = np.all((th >= lo - sh.halo) & (tl <= hi + sh.halo), axis=1)
    assert np.array_equal(np.nonzero(meets)[0] + 1, sh.tet_gid)


def test_cell_shard_structure():
    """pmmg_shard_mark_cells keeps exactly the tetra whose box grown by the
    halo meets the range's box and an occupied cell (numpy restatement), a
    subset of the box shard, with the same renumbered connectivity."""
    bg = synth.lattice(synth.SHELL, 12)
    new = synth.lattice(synth.SHELL, 16, jitter=0.2, with_trias=False, with_tetra=False)
    pc = synth.classes(new)
    for mine in ranks.morton_shards(new.xyz, pc, 4):
        q = new.xyz[mine]
        sh = shard.halo_shard_cells(bg, q, hausd=0.01)
        h = sh.halo
        cell = 1.0 * h
        g_lo = bg.xyz.min(axis=0) - cell
        g_n = np.maximum(1, np.ceil((bg.xyz.max(axis=0) + cell - g_lo) / cell).astype(np.int64))
        occ = np.zeros(tuple(g_n[::-1]), bool)
        c = np.clip(np.floor((q - g_lo) / cell).astype(np.int64), 0, g_n - 1)
        occ[c[:, 2], c[:, 1], c[:, 0]] = True
        tl, th = bg.xyz[bg.tetv - 1].min(axis=1), bg.xyz[bg.tetv - 1].max(axis=1)
        lo, hi = shard.range_box(q)
        a = np.maximum(np.floor((tl - h - g_lo) / cell).astype(np.int64), 0)
        b = np.minimum(np.floor((th + h - g_lo) / cell).astype(np.int64), g_n - 1)
        inbox = np.all((th >= lo - h) & (tl <= hi + h), axis=1)
        keep = np.zeros(bg.ne, bool)
        for k in np.nonzero(inbox)[0]:
            keep[k] = occ[a[k, 2]:b[k, 2] + 1, a[k, 1]:b[k, 1] + 1, a[k, 0]:b[k, 0] + 1].any()
        assert np.array_equal(np.nonzero(keep)[0] + 1, sh.tet_gid)
        assert np.array_equal(sh.vert_gid[sh.mesh.tetv - 1], bg.tetv[sh.tet_gid - 1])
        box = shard.halo_shard(bg, lo, hi, hausd=0.01)
        assert set(sh.tet_gid.tolist()) <= set(box.tet_gid.tolist())


@pytest.mark.parametrize("mode", ["box", "cells", "rcb"])
@pytest.mark.parametrize("kind,n_old,n_new,world", [(synth.CUBE, 6, 7, 2), (synth.CUBE, 5, 9, 3),
                                                    (synth.SHELL, 8, 12, 2), (synth.SHELL, 8, 12, 4)])
def test_halo_shards_oracle_parity(kind, n_old, n_new, world, mode):
    """Oracle on each rank's halo shard == contract of a transfer on the group."""
    case = make_case(kind=kind, n_old=n_old, n_new=n_new)
    full = _empty_result(case)
    nshard = 0
    for mine, sh in _shards(case, world, mode=mode):
        B = O.Background(sh.mesh, None if case["met"] is None else sh.rows(case["met"]),
                         [sh.rows(f) for f in case["fields"]], case["hausd"])
        q = np.ascontiguousarray(case["new"].xyz[mine])
        r = O.run(B, q, case["pclass"][mine], np.arange(1, len(mine) + 1, dtype=np.int32), O.MODE_FRESH)
        hit = (r["hit"].astype(np.int32) | (np.maximum(r["loc"], 0).astype(np.int32) << 4)).astype(np.int8)
        _scatter(full, mine, sh, r["met"], r["fields"], r["elem"], hit)
        nshard += sh.mesh.ne
    rep = check(case, full)
    assert rep["n"] == int((case["pclass"] != 0).sum()) and rep["class_i"] == rep["class_i_same"] > 0
    assert nshard < world * case["bg"].ne  # not replicas


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["box", "cells"])
@pytest.mark.parametrize("kind,n_old,n_new,world", [(synth.CUBE, 6, 7, 3), (synth.SHELL, 12, 16, 4)])
def test_halo_shards_gpu_parity(kind, n_old, n_new, world, mode):
    from parmmg_amd.transfer import TransferContext

    case = make_case(kind=kind, n_old=n_old, n_new=n_new)
    full = _empty_result(case)
    with TransferContext(0) as ctx:
        for mine, sh in _shards(case, world, mode=mode):
            m = sh.mesh
            ctx.set_background(m.xyz, m.tetv, m.adja, m.triv, m.adjt, case["hausd"])
            ctx.set_solutions(None if case["met"] is None else sh.rows(case["met"]),
                              [sh.rows(f) for f in case["fields"]])
            n = len(mine)
            met = None if case["met"] is None else np.full((n, case["met"].shape[1]), np.nan)
            fo = [np.full((n, f.shape[1]), np.nan) for f in case["fields"]]
            elem, hit = np.zeros(n, np.int32), np.zeros(n, np.int8)
            ctx.locate_interp(np.ascontiguousarray(case["new"].xyz[mine]), np.ascontiguousarray(case["pclass"][mine]),
                              met, fo, elem, hit)
            _scatter(full, mine, sh, met, fo, elem, hit)
    rep = check(case, full)
    assert rep["n"] == int((case["pclass"] != 0).sum()) and rep["class_i"] == rep["class_i_same"] > 0


def _halo_worker(rank, world, port, q):
    import os

    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    ri = ranks.init("gloo")
    case = make_case(kind=synth.SHELL, n_old=8, n_new=12, with_ref=False)  # the same problem on every rank
    shards = ranks.rcb_shards(case["new"].xyz, case["pclass"], world)  # bench.py's default split
    mine = shards[rank]
    sh = shard.halo_shard_cells(case["bg"], case["new"].xyz[mine], hausd=case["hausd"])  # as bench.py --shard halo
    B = O.Background(sh.mesh, sh.rows(case["met"]), [sh.rows(f) for f in case["fields"]], case["hausd"])
    r = O.run(B, np.ascontiguousarray(case["new"].xyz[mine]), case["pclass"][mine],
              np.arange(1, len(mine) + 1, dtype=np.int32), O.MODE_FRESH)
    code = r["hit"].astype(np.int32)
    gid = sh.to_group_elem(r["elem"], np.isin(code, list(BDY_CODES)))
    hit = code | (np.maximum(r["loc"], 0).astype(np.int32) << 4)
    rows = np.concatenate([gid[:, None], hit[:, None], r["met"]] + r["fields"], axis=1).astype(np.float64)
    got = ranks.allgather_rows(ri, torch.from_numpy(rows), [len(s) for s in shards]).numpy()
    q.put((rank, got, sh.mesh.ne))
    ranks.finalize(ri)


def test_gloo_two_ranks_halo_shards():
    """world 2 (gloo): each rank transfers its Morton range against its own halo
    shard; the gathered results meet the group's parity contract."""
    import torch.multiprocessing as mp
    from test_ranks import _free_port

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_halo_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {r: (g, ne) for r, g, ne in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    case = make_case(kind=synth.SHELL, n_old=8, n_new=12)
    assert np.array_equal(out[0][0], out[1][0])
    assert all(ne < case["bg"].ne for _, ne in out.values())
    order = np.concatenate(ranks.rcb_shards(case["new"].xyz, case["pclass"], world))
    got = out[0][0]
    full = _empty_result(case)
    full["elem"][order] = got[:, 0].astype(np.int32)
    full["hit"][order] = got[:, 1].astype(np.int8)
    c = 2
    full["met"][order] = got[:, c:c + case["met"].shape[1]]
    c += case["met"].shape[1]
    for f in full["fields"]:
        f[order] = got[:, c:c + f.shape[1]]
        c += f.shape[1]
    rep = check(case, full)
    assert rep["n"] == len(order) and rep["class_i"] == rep["class_i_same"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["box", "cells", "rcb"])
@pytest.mark.parametrize("kind,n_old,n_new,world", [(synth.CUBE, 64, 70, 4), (synth.SHELL, 64, 72, 3)])
def test_halo_shards_gpu_match_group_run_large(kind, n_old, n_new, world, mode):
    """Million-tetra sizes: every rank's halo-shard transfer, mapped to group
    ids, agrees with the transfer on the whole group — same element and
    bit-identical values wherever both walks accepted the same tetra (the
    walk path may differ near the cut), and otherwise an element the group
    accepts with the reference values in it (oracle spot checks)."""
    from parmmg_amd.transfer import TransferContext

    case = make_case(kind=kind, n_old=n_old, n_new=n_new, with_ref=False)
    bg, new, pc = case["bg"], case["new"], case["pclass"]
    B = case["B"]
    with TransferContext(0) as ctx:
        ctx.set_background(bg.xyz, bg.tetv, bg.adja, bg.triv, bg.adjt, case["hausd"])
        ctx.set_solutions(case["met"], case["fields"])
        whole = _empty_result(case)
        ctx.locate_interp(new.xyz, pc, whole["met"], whole["fields"], whole["elem"], whole["hit"])
        parts = _empty_result(case)
        for mine, sh in _shards(case, world, mode=mode):
            m = sh.mesh
            ctx.set_background(m.xyz, m.tetv, m.adja, m.triv, m.adjt, case["hausd"])
            ctx.set_solutions(sh.rows(case["met"]), [sh.rows(f) for f in case["fields"]])
            n = len(mine)
            met = np.full((n, case["met"].shape[1]), np.nan)
            fo = [np.full((n, f.shape[1]), np.nan) for f in case["fields"]]
            elem, hit = np.zeros(n, np.int32), np.zeros(n, np.int8)
            ctx.locate_interp(np.ascontiguousarray(new.xyz[mine]), np.ascontiguousarray(pc[mine]), met, fo, elem, hit)
            _scatter(parts, mine, sh, met, fo, elem, hit)
    done = pc != 0
    assert (parts["elem"][done] > 0).all() and ((parts["hit"][done].astype(np.int32) & 15) != 0).all()
    same = done & (parts["elem"] == whole["elem"]) & (parts["hit"] == whole["hit"])
    # near the cut the walks may take other paths (more cut faces for cell shards: 0.1 % of the points)
    assert same.sum() >= 0.995 * done.sum(), (int(same.sum()), int(done.sum()))
    for a, b in zip([parts["met"]] + parts["fields"], [whole["met"]] + whole["fields"]):
        assert np.array_equal(a[same], b[same], equal_nan=True)
    # the rest: accepted elements and reference values (oracle, per point)
    rest = np.nonzero(done & ~same)[0][:5000]
    for i in rest:
        code = int(parts["hit"][i]) & 15
        if code == 1:  # volume walk: the group accepts the element
            assert O.tetra_minbary(B, int(parts["elem"][i]), new.xyz[i]) > -O.EPS
        met_r, fr = O.eval_in_element(B, new.xyz[i], pc[i] == 2, int(parts["elem"][i]), code,
                                      (int(parts["hit"][i]) >> 4) & 3)
        np.testing.assert_allclose(parts["met"][i], met_r, rtol=1e-12)
        for f, g in zip(parts["fields"], fr):
            np.testing.assert_allclose(f[i], g, rtol=1e-12)


@pytest.mark.gpu
@pytest.mark.skipif(os.environ.get("PMMG_TEST_CFG5", "1") == "0", reason="PMMG_TEST_CFG5=0: skipped (~55 s, ~80 GB "
                    "of host memory)")
def test_halo_shards_gpu_cfg5_full_size():
    """cfg5 at full size (500.7M tetra, 100.5M new points, iso metric + 5
    fields): the group on one GPU, then its two RCB parts against their halo
    shards one after the other on the same GPU (the split bench.py --gpus 2
    --shard halo runs across two).  Mapped to group ids, the parts agree
    with the group: same element and bit-identical rows wherever both walks
    accepted the same tetra, elsewhere an element the group accepts with the
    reference interpolator's values (oracle, 2000 points)."""
    import time

    from parmmg_amd import configs
    from parmmg_amd.transfer import TransferContext

    t0 = time.time()
    w = configs.CFG5
    bg, new = configs.build_meshes(w, seed=synth.SEED)
    pc = synth.classes(new)
    met = synth.solution(w.metric, bg.xyz)
    fields = [synth.solution(f, bg.xyz) for f in w.fields]
    case = dict(bg=bg, new=new, pclass=pc, met=met, fields=fields, hausd=w.hausd)
    print(f"cfg5: {bg.ne} tetra, {new.np} points, built in {time.time() - t0:.0f} s", flush=True)
    with TransferContext(0) as ctx:
        ctx.set_background(bg.xyz, bg.tetv, bg.adja, bg.triv, bg.adjt, w.hausd)
        ctx.set_solutions(met, fields)
        whole = _empty_result(case)
        st = ctx.locate_interp(new.xyz, pc, whole["met"], whole["fields"], whole["elem"], whole["hit"])
        print(f"group run: {st.ms_total:.2f} ms on the device, {time.time() - t0:.0f} s, {st.as_dict()}", flush=True)
        parts = _empty_result(case)
        for r, mine in enumerate(ranks.rcb_shards(new.xyz, pc, 2)):
            sh = shard.halo_shard_cells(bg, new.xyz[mine], hausd=w.hausd)
            m = sh.mesh
            print(f"part {r}: {len(mine)} points, shard {m.ne} tetra ({m.ne / bg.ne:.1%}), {time.time() - t0:.0f} s",
                  flush=True)
            ctx.set_background(m.xyz, m.tetv, m.adja, m.triv, m.adjt, w.hausd)
            ctx.set_solutions(sh.rows(met), [sh.rows(f) for f in fields])
            n = len(mine)
            mo = np.full((n, met.shape[1]), np.nan)
            fo = [np.full((n, f.shape[1]), np.nan) for f in fields]
            elem, hit = np.zeros(n, np.int32), np.zeros(n, np.int8)
            st = ctx.locate_interp(np.ascontiguousarray(new.xyz[mine]), np.ascontiguousarray(pc[mine]), mo, fo, elem,
                                   hit)
            print(f"part {r}: {st.ms_total:.2f} ms on the device, {st.as_dict()}", flush=True)
            _scatter(parts, mine, sh, mo, fo, elem, hit)
            del sh, m
    done = pc != 0
    assert (parts["elem"][done] > 0).all() and ((parts["hit"][done].astype(np.int32) & 15) != 0).all()
    same = done & (parts["elem"] == whole["elem"]) & (parts["hit"] == whole["hit"])
    print(f"same element as the group: {int(same.sum())} of {int(done.sum())}", flush=True)
    assert same.sum() >= 0.995 * done.sum(), (int(same.sum()), int(done.sum()))
    for a, b in zip([parts["met"]] + parts["fields"], [whole["met"]] + whole["fields"]):
        assert np.array_equal(a[same], b[same], equal_nan=True)
    B = O.Background(bg, met, fields, w.hausd)
    rest = np.nonzero(done & ~same)[0][:2000]
    for i in rest:
        code = int(parts["hit"][i]) & 15
        if code == 1:
            assert O.tetra_minbary(B, int(parts["elem"][i]), new.xyz[i]) > -O.EPS
        met_r, fr = O.eval_in_element(B, new.xyz[i], pc[i] == 2, int(parts["elem"][i]), code,
                                      (int(parts["hit"][i]) >> 4) & 3)
        np.testing.assert_allclose(parts["met"][i], met_r, rtol=1e-12)
        for f, g in zip(parts["fields"], fr):
            np.testing.assert_allclose(f[i], g, rtol=1e-12)
    print(f"checked {len(rest)} of the rest against the oracle; {time.time() - t0:.0f} s", flush=True)
