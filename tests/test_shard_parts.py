"""Halo shards built from the ranks' parts of a group (VERDICT r04 item 6:
no rank holds the whole group).  pmmg_shard_part_pack + pmmg_shard_assemble
(csrc/pmmg_shard.c) must give, bit for bit, the shard halo_shard_cells
builds from the whole group: the same local numbering (ascending global
ids), coordinates, adjacency (cut faces and edges as walls), trias and
global id maps, and the vertex rows travel with it."""
import numpy as np
import pytest

from parity import make_case
from parmmg_amd import ranks, shard, synth


def _same_shard(a: shard.HaloShard, b: shard.HaloShard):
    for x, y in ((a.mesh.xyz, b.mesh.xyz), (a.mesh.tetv, b.mesh.tetv), (a.mesh.adja, b.mesh.adja),
                 (a.mesh.triv, b.mesh.triv), (a.mesh.adjt, b.mesh.adjt), (a.tet_gid, b.tet_gid),
                 (a.vert_gid, b.vert_gid), (a.tria_gid, b.tria_gid)):
        assert x.shape == y.shape and np.array_equal(x, y)


def _problem(kind, n_old, n_new):
    case = make_case(kind=kind, n_old=n_old, n_new=n_new, with_ref=False)
    bg = case["bg"]
    sol = np.concatenate([case["met"]] + case["fields"], axis=1)
    h = max(-shard.DEFAULT_HALO * shard.max_tet_extent(bg), 1.01 * case["hausd"])
    grid = shard.grid_for(bg.xyz.min(axis=0), bg.xyz.max(axis=0), h)
    return case, bg, sol, h, grid


@pytest.mark.parametrize("kind,n_old,n_new,world", [(synth.CUBE, 10, 12, 3), (synth.SHELL, 12, 16, 4),
                                                    (synth.CUBE, 8, 9, 1)])
def test_parts_assemble_to_the_whole_group_shard(kind, n_old, n_new, world):
    case, bg, sol, h, (g_lo, cell, g_n) = _problem(kind, n_old, n_new)
    parts = [shard.part_of(bg, sol, r, world) for r in range(world)]
    assert sum(p.tet_gid.shape[0] for p in parts) == bg.ne
    for mine in ranks.rcb_shards(case["new"].xyz, case["pclass"], world):
        q = case["new"].xyz[mine]
        whole = shard.halo_shard_cells(bg, q, h, hausd=case["hausd"])
        reg = shard.region_of(q, g_lo, cell, g_n, h)
        got = shard.assemble([shard.pack_part(p, reg) for p in parts], sol.shape[1], kind, n_old, h)
        _same_shard(got, whole)
        assert np.array_equal(got.sol, sol[whole.vert_gid - 1])
        assert whole.mesh.ne < bg.ne or world == 1


def test_assemble_rejects_inconsistent_buffers():
    case, bg, sol, h, (g_lo, cell, g_n) = _problem(synth.CUBE, 6, 7)
    reg = shard.region_of(case["new"].xyz[:50], g_lo, cell, g_n, h)
    buf = shard.pack_part(shard.part_of(bg, sol, 0, 2), reg)
    with pytest.raises(ValueError):
        shard.assemble([buf], sol.shape[1] + 1)  # another K
    with pytest.raises(ValueError):
        shard.assemble([buf[:-8]], sol.shape[1])  # truncated


def _parts_worker(rank, world, port, q):
    import os

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    ri = ranks.init("gloo")
    case, bg, sol, h, (g_lo, cell, g_n) = _problem(synth.SHELL, 12, 16)
    part = shard.part_of(bg, sol, rank, world)  # all this rank holds of the group
    mine = ranks.rcb_shards(case["new"].xyz, case["pclass"], world)[rank]
    sh = shard.shard_from_parts(ri, part, case["new"].xyz[mine], h, g_lo, cell, g_n, synth.SHELL, 12)
    # the halo and the grid from the parts alone (parts_frame's all-reduces, hausd floor)
    frame = shard.parts_frame(ri, part, shard.DEFAULT_HALO, case["hausd"])
    sh2 = shard.shard_from_parts(ri, part, case["new"].xyz[mine], shard.DEFAULT_HALO, kind=synth.SHELL, n=12,
                                 hausd=case["hausd"])
    whole = shard.halo_shard_cells(bg, case["new"].xyz[mine], h, hausd=case["hausd"])
    try:
        _same_shard(sh, whole)
        _same_shard(sh2, whole)
        ok = bool(np.array_equal(sh.sol, sol[whole.vert_gid - 1])) and bool(np.array_equal(sh2.sol, sh.sol))
        ok = ok and frame[0] == h and np.array_equal(frame[1], g_lo) and frame[2] == cell and \
            np.array_equal(frame[3], g_n)
    except AssertionError:
        ok = False
    q.put((rank, ok, sh.mesh.ne, part.tet_gid.shape[0]))
    ranks.finalize(ri)


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_shards_from_parts(world):
    """world 2 / 3 (gloo): every rank holds only its part of the group; the
    all-to-all of packed parts gives each rank the same shard as the whole-
    group builder."""
    import torch.multiprocessing as mp
    from test_ranks import _free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_parts_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _, _ in out), out
