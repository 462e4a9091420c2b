"""The bench's multi-rank path on CPU (gloo, world_size 2): every rank owns
its own group (weak scaling, no data-path collective), the only reductions are
the barrier, max of the step time and sum of the points."""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

from parmmg_amd import configs, ranks, synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    ri = ranks.init("gloo")
    assert ri.distributed and ri.world == world and ri.rank == rank
    # per-rank group, as bench.build_workload makes it (seed + rank)
    new = synth.lattice(synth.CUBE, 4, jitter=0.2, seed=synth.SEED + rank, with_trias=False)
    pclass = synth.classes(new)
    npts = int((pclass != 0).sum())
    ranks.barrier(ri)
    elapsed = 0.5 + rank  # rank 1 is the slow one
    agg = ranks.aggregate(ri, npts, elapsed, steps=5)
    q.put((rank, npts, float(new.xyz.sum()), agg))
    ranks.finalize(ri)


def test_gloo_two_ranks_weak_aggregate():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, n0, s0, a0), (r1, n1, s1, a1) = out
    assert a0 == a1  # every rank sees the same reduced numbers
    assert a0["points_per_step"] == n0 + n1
    assert a0["elapsed_s"] == 1.5
    np.testing.assert_allclose(a0["ms_per_step"], 1.5 / 5 * 1e3)
    np.testing.assert_allclose(a0["mpts_per_s"], (n0 + n1) / (1.5 / 5) / 1e6)
    assert s0 != s1  # each rank jitters its own group


def test_single_process_no_group(monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    ri = ranks.init("nccl")  # world 1: no process group, no device touched
    assert not ri.distributed
    agg = ranks.aggregate(ri, 1000, 2.0, steps=4)
    assert agg["points_per_step"] == 1000 and agg["ms_per_step"] == 500.0


def test_bench_configs_fit_one_gpu():
    """Every bench workload's resident footprint fits a 288 GB GPU with room."""
    for w in configs.SHORT.values():
        (np_o, ne_o, nt_o), (np_n, _, _) = w.counts()
        b = np_o * (24 + 8 * w.K) + ne_o * 32 + nt_o * 24 + np_n * (24 + 1 + 8 * w.K + 4 + 1)
        assert b < 200e9, (w.name, b)


def test_morton_shards_partition_and_locality():
    new = synth.lattice(synth.CUBE, 12, jitter=0.2, with_trias=False)
    pclass = synth.classes(new, req_every=7)
    for world in (1, 2, 3, 8):
        sh = ranks.morton_shards(new.xyz, pclass, world)
        allidx = np.concatenate(sh)
        assert sorted(allidx.tolist()) == np.nonzero(pclass != 0)[0].tolist()  # every processed point once
        # equal cost: a surface point weighs BDY_WEIGHT volume points
        cost = [int(np.where(pclass[s] == 2, ranks.BDY_WEIGHT, 1).sum()) for s in sh]
        assert max(cost) - min(cost) <= ranks.BDY_WEIGHT
        sizes = [len(s) for s in ranks.morton_shards(new.xyz, pclass, world, bdy_weight=1)]
        assert max(sizes) - min(sizes) <= 1
        codes = ranks.morton_codes(new.xyz[np.nonzero(pclass != 0)[0]])
        cmin = [int(ranks.morton_codes(new.xyz)[s].min()) for s in sh]
        assert cmin == sorted(cmin)  # contiguous Morton ranges in rank order
        assert codes.dtype == np.uint32


def test_rcb_shards_partition_and_boxes():
    """Recursive coordinate bisection: every processed point once, equal cost
    per rank, and on a shell compact boxes (a Morton range's box can hold
    two pieces far apart)."""
    new = synth.lattice(synth.SHELL, 16, jitter=0.2, with_trias=False)
    pclass = synth.classes(new, req_every=7)
    for world in (1, 2, 3, 8):
        sh = ranks.rcb_shards(new.xyz, pclass, world)
        allidx = np.concatenate(sh)
        assert sorted(allidx.tolist()) == np.nonzero(pclass != 0)[0].tolist()
        cost = [int(np.where(pclass[s] == 2, ranks.BDY_WEIGHT, 1).sum()) for s in sh]
        assert max(cost) - min(cost) <= 2 * ranks.BDY_WEIGHT
        assert all(np.all(np.diff(s) > 0) for s in sh)  # input order kept inside a part
    # 8 parts of a shell: the octants, boxes of half the shell's extent
    sh = ranks.rcb_shards(new.xyz, pclass, 8)
    ext = np.ptp(new.xyz, axis=0)
    for s in sh:
        assert np.all(np.ptp(new.xyz[s], axis=0) <= 0.51 * ext)


def _gather_worker(rank, world, port, q):
    """One rank of the Morton split with a replicated background: the oracle
    transfers this rank's contiguous Morton range (as the module does on its
    GPU), and {elem, hit, K doubles} rows are all-gathered."""
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from parity import make_case
    from oracle import oracle as O

    ri = ranks.init("gloo")
    case = make_case(kind=synth.SHELL, n_old=8, n_new=12, with_ref=False)  # the same problem on every rank
    sh = ranks.morton_shards(case["new"].xyz, case["pclass"], world)
    mine = sh[rank]
    r = O.run(case["B"], np.ascontiguousarray(case["new"].xyz[mine]), case["pclass"][mine],
              np.arange(1, len(mine) + 1, dtype=np.int32), O.MODE_FRESH)
    hit = r["hit"].astype(np.int32) | (np.maximum(r["loc"], 0).astype(np.int32) << 4)
    rows = np.concatenate([r["elem"][:, None], hit[:, None], r["met"]] + r["fields"], axis=1).astype(np.float64)
    got = ranks.allgather_rows(ri, torch.from_numpy(rows), [len(s) for s in sh]).numpy()
    q.put((rank, got))
    ranks.finalize(ri)


def test_gloo_two_ranks_morton_allgather():
    """world 2 (gloo), Morton ranges against a replicated background: every
    rank transfers its range, the all-gathered rows are identical on both
    ranks and meet the group's parity contract (tests/parity.py)."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from parity import check, make_case

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(out[0], out[1])
    case = make_case(kind=synth.SHELL, n_old=8, n_new=12)
    order = np.concatenate(ranks.morton_shards(case["new"].xyz, case["pclass"], world))
    got = out[0]
    n = case["new"].np
    full = dict(elem=np.zeros(n, np.int32), hit=np.zeros(n, np.int8),
                met=np.full((n, case["met"].shape[1]), np.nan), fields=[np.full((n, f.shape[1]), np.nan)
                                                                         for f in case["fields"]])
    full["elem"][order] = got[:, 0].astype(np.int32)
    full["hit"][order] = got[:, 1].astype(np.int8)
    c = 2 + case["met"].shape[1]
    full["met"][order] = got[:, 2:c]
    for f in full["fields"]:
        f[order] = got[:, c:c + f.shape[1]]
        c += f.shape[1]
    rep = check(case, full)
    assert rep["n"] == len(order) and rep["class_i"] == rep["class_i_same"] > 0
