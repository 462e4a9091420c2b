"""Benchmark of the old->new mesh transfer step (PMMG_interpMetricsAndFields).

One step = one full pmmg_hip_locate_interp over one group: frame + seed
grids + query order + volume/surface locate + metric/field interpolation +
fallbacks, with every input already resident in HBM (device-mode C-ABI).

N = 1: the whole cfg4 group on one GPU.  N > 1 (torchrun, one process per
GPU), default ``--shard halo``: every rank owns a compact part of the new
points (recursive coordinate bisection into boxes of equal cost, ``--split
rcb``; ``--split morton`` keeps the north_star's contiguous Morton ranges)
against the halo shard of the background around that part (SURVEY.md
§8(e)); the located elements and interpolated rows are collected with an
RCCL all-gather after the timed steps (reported separately, outside the
step: ParMmg consumes results per rank) and checked on rank 0 against an
oracle run over a sample of the whole group (``parity``).  Strong scaling:
`value` = points of the whole problem / max-over-ranks step time.
``--shard morton`` replicates the background instead; ``--shard group``
gives every rank its own group (weak scaling, ParMmg's per-group sharding).

After the timed steps (rank 0, N = 1): the CPU baseline runs the oracle — a C
restatement of the reference path — over ALL new points in the reference's
visitation order on the host cores, and the GPU outputs of the last step are
checked against that same run point by point (``parity``: class (i) identity,
acceptance of every chosen element, values of the reference interpolator in
it, bit-exact count and max relative error).

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from parmmg_amd import configs, ranks, synth  # noqa: E402
from parmmg_amd.transfer import TransferContext, pack_solutions, pack_tet8  # noqa: E402

METRIC = "new-mesh points located+interpolated/sec (Mpts/s) and HBM GB/s, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
BOX_CPU_SHARE = 16     # host CPUs a one-GPU lease of the GPU pool gives a job


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_workload(w: configs.Workload, rank: int):
    t0 = time.time()
    bg, new = configs.build_meshes(w, seed=synth.SEED + rank)
    met = synth.solution(w.metric, bg.xyz)
    fields = [synth.solution(f, bg.xyz) for f in w.fields]
    pclass = synth.classes(new)
    log(f"[bench r{rank}] workload {w.name}: bg {bg.ne} tets / {bg.np} verts / {bg.nt} trias, new {new.np} verts, "
        f"K={w.K}, generated in {time.time() - t0:.1f}s")
    return bg, new, met, fields, pclass


def pmc_traffic(workload: str):
    """HBM bytes per call of the volume stage from the newest committed
    rocprofv3 PMC summary (profiles/rNN*/pmc_<workload>.json, made by
    tools/prof_summary.py from FETCH_SIZE / WRITE_SIZE passes of this bench),
    or (None, None)."""
    import glob

    def order(path):  # round, then the run tag as named: r03a .. r03z, r03aa .. r03zz
        tag = os.path.basename(os.path.dirname(path))
        return tag[:3], len(tag), tag

    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"pmc_{workload}.json")), key=order)
    if not paths:
        return None, None
    try:
        with open(paths[-1]) as f:
            d = json.load(f)
        return d.get("k_vol_hbm_bytes_per_call"), os.path.relpath(paths[-1], ROOT)
    except Exception:
        return None, None


def cgroup_cpus() -> float | None:
    """The CPU quota of this process's cgroup (cgroup v2 cpu.max: quota /
    period), or None when unlimited / unreadable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return None if q == "max" else int(q) / int(p)
    except (OSError, ValueError):
        return None


def host_cores() -> tuple[int, int]:
    """(threads used, CPUs visible): every host core this process can use —
    the CPUs of its affinity mask, bounded by its cgroup's CPU quota (a
    one-GPU box shows all 256 CPUs of the machine but grants the job 16 of
    them through cpu.max; more threads than that are throttled, not
    faster).  Without a quota: the affinity mask, capped at the pool's
    per-GPU share."""
    try:
        vis = len(os.sched_getaffinity(0))
    except AttributeError:
        vis = os.cpu_count() or 1
    env = int(os.environ.get("PMMG_CPU_THREADS", "0"))
    quota = cgroup_cpus()
    usable = min(vis, max(1, int(quota))) if quota else min(vis, BOX_CPU_SHARE)
    return (env or usable), vis


def cpu_baseline(w, bg, met, fields, pclass, new, budget_s: float):
    """The oracle (C restatement of the reference path) on this host's cores:
    the per-iteration precompute (faceAreas, triaNormals, nodeTrias, inside
    the reference's tim=2 timer, src/libparmmg1.c:823-836) split over the
    threads, then ALL new points in the reference's visitation order (first
    appearance in new-tetra order, src/interpmesh_pmmg.c:535-541) cut into one
    contiguous range per thread, each a sequential reference run with warm
    start and private visited flags (one MPI rank per group).  Returns the
    report and the oracle's per-point outputs (the parity reference)."""
    from oracle import oracle as O

    threads, visible = host_cores()
    t0 = time.time()
    new_t = synth.lattice(w.kind, w.n_new, jitter=w.jitter_new, seed=synth.SEED, with_trias=False)
    order = synth.visit_order(new_t)
    del new_t
    log(f"[bench] visit order of {order.shape[0]} points in {time.time() - t0:.1f}s; oracle on {threads} threads")
    B = O.Background(bg, met, fields, w.hausd)
    r = O.run(B, new.xyz, pclass, order, budget_s=budget_s, threads=threads)
    t_pre, t_loc = r["t_precompute"], r["t_locate"]
    nproc = int((r["hit"] != 0).sum())
    ntot = int((pclass != 0).sum())
    t_full = t_pre + t_loc * ntot / max(nproc, 1)
    frac = nproc / max(ntot, 1)
    rep = {
        "value": round(ntot / t_full / 1e6, 4),
        "unit": "Mpts/s",
        "cores": threads,
        "cpus_visible": visible,
        "cgroup_cpu_quota": cgroup_cpus(),
        "kind": "port",
        "sample": f"oracle (C restatement of the reference path) as {threads} threads = every usable host core "
                  f"({visible} CPUs visible, cgroup cpu.max quota {cgroup_cpus()} CPUs), one contiguous range of the "
                  f"reference's "
                  f"visitation order each (like MPI ranks), on {w.name}: precompute over {bg.ne} tets "
                  f"({t_pre:.2f}s) + locate/interp of {nproc} of {ntot} points ({100 * frac:.1f}%, {t_loc:.2f}s)"
                  + ("" if nproc == ntot else ", rate extrapolated to all points"),
        "t_precompute_s": round(t_pre, 3),
        "t_locate_s": round(t_loc, 3),
        "points_timed": nproc,
        "points_total": ntot,
    }
    return rep, B, r


def parity_report(B, new, pclass, gpu, ref) -> dict:
    """The GPU outputs of the last step against the oracle run of the CPU
    baseline, over every point the oracle processed (tests/parity.py
    contract, oracle.check_batch)."""
    from oracle import oracle as O

    threads, _ = host_cores()
    idx = np.nonzero(ref["hit"] != 0)[0].astype(np.int32)
    t0 = time.time()
    rep = O.check_batch(B, new.xyz, pclass, gpu["elem"], gpu["hit"], gpu["met"], gpu["fields"], idx=idx, ref=ref,
                        threads=threads)
    # points whose element and hit kind equal the oracle's must carry the
    # oracle's own values bit for bit
    same = (gpu["elem"][idx] == ref["elem"][idx]) & ((gpu["hit"][idx] & 15) == (ref["hit"][idx] & 15))
    ident = np.ones(idx.shape[0], bool)
    for a, b in zip(([gpu["met"]] if gpu["met"] is not None else []) + gpu["fields"],
                    ([ref["met"]] if ref["met"] is not None else []) + ref["fields"]):
        ident &= np.all((a[idx] == b[idx]) | (np.isnan(a[idx]) & np.isnan(b[idx])), axis=1)
    out = {
        "what": "GPU outputs of the timed step vs the oracle run of cpu_baseline, every point it processed",
        "points": int(idx.shape[0]), "checked": rep["n"], "exact": rep["exact"],
        "class_i": rep["class_i"], "class_i_same": rep["class_i_same"],
        "accept_fail": rep["accept_fail"], "value_fail": rep["value_fail"], "unprocessed": rep["unprocessed"],
        "maxrel": rep["maxrel"], "rel_tol": 1e-12,
        "same_element_as_oracle": int(same.sum()),
        "same_element_values_identical": int((same & ident).sum()),
        "hits": rep["hits"],
        "ok": bool(rep["accept_fail"] == 0 and rep["value_fail"] == 0 and rep["unprocessed"] == 0
                   and rep["class_i"] == rep["class_i_same"] and rep["maxrel"] <= 1e-12
                   and int((same & ~ident).sum()) == 0),
        "check_s": round(time.time() - t0, 2),
    }
    return out


def allgather_timing(ri, ctx, d_mo, d_fo, d_elem, d_hit, sh, counts, rank: int, reps: int = 3):
    """Split modes: collect every rank's located elements (mapped to group
    ids: a halo shard's local ids through its tet_gid / tria_gid), hit codes
    and interpolated rows on every rank, timed on its own after the timed
    steps (reported separately; ParMmg itself consumes the
    results per rank).  With RCCL (backend nccl) through the module's C-ABI
    collective (pmmg_hip_comm_init + pmmg_hip_allgather_points: one
    ncclAllGather of packed records over xGMI), checked against
    torch.distributed's all_gather_into_tensor of the same arrays
    (ranks.allgather_rows, also the path of a gloo rehearsal, whose ranks
    share one GPU and cannot form an RCCL communicator).  Returns the report
    and the gathered (rows, elem, hit) as host arrays in rank order."""
    import torch

    rows = torch.cat([d_mo] + list(d_fo), dim=1)
    hit = d_hit.download()
    elem = d_elem.cpu().numpy()
    if sh is not None:
        elem = sh.to_group_elem(elem, (hit & 15) >= 4)
    eh = torch.from_numpy(np.stack([elem.astype(np.int32), hit.astype(np.int32)], axis=1)).to(rows.device)

    def timed(fn):
        ts = []
        out = None
        for _ in range(reps):
            ranks.barrier(ri)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = fn()
            torch.cuda.synchronize()
            ts.append(ranks.max_over_ranks(ri, time.perf_counter() - t0))
        return float(np.median(ts)), out

    t_torch, (g_rows, g_eh) = timed(lambda: (ranks.allgather_rows(ri, rows, counts),
                                             ranks.allgather_rows(ri, eh, counts)))
    nbytes = sum(counts) * (rows.shape[1] * 8 + 8)
    g_eh = g_eh.cpu().numpy()
    g_rows_np, g_elem, g_hit = g_rows.cpu().numpy(), g_eh[:, 0].copy(), g_eh[:, 1].astype(np.int8)
    rep = {"what": "all-gather of {group elem id, hit code, K doubles} per point, not part of the step",
           "bytes": int(nbytes), "rows": int(g_rows.shape[0]),
           "torch_all_gather_ms": round(1e3 * t_torch, 3)}
    if ri.backend == "nccl":
        try:
            dev = rows.device
            uid = [TransferContext.comm_unique_id() if rank == 0 else None]
            ranks.broadcast_object(ri, uid)
            ctx.comm_init(ri.world, rank, uid[0])
            n_all = int(sum(counts))
            d_elem_g = torch.from_numpy(elem.astype(np.int32)).to(dev)
            outs = [torch.empty((n_all, a.shape[1]), dtype=torch.float64, device=dev) for a in [d_mo] + list(d_fo)]
            e_all = torch.empty((n_all,), dtype=torch.int32, device=dev)
            h_all = torch.empty((n_all,), dtype=torch.int8, device=dev)
            t_c, _ = timed(lambda: ctx.allgather_points(counts, [d_mo] + list(d_fo), outs, d_elem_g, e_all, d_hit,
                                                        h_all))
            c_rows = torch.cat(outs, dim=1).cpu().numpy()
            same = bool(np.array_equal(c_rows, g_rows_np, equal_nan=True)
                        and np.array_equal(e_all.cpu().numpy(), g_elem) and np.array_equal(h_all.cpu().numpy(), g_hit))
            rep.update({"path": "C-ABI pmmg_hip_allgather_points (one ncclAllGather of packed records)",
                        "ms": round(1e3 * t_c, 3), "gbps": round(nbytes / t_c / 1e9, 1),
                        "matches_torch_all_gather": same})
            if same:
                g_rows_np, g_elem, g_hit = c_rows, e_all.cpu().numpy(), h_all.cpu().numpy()
        except Exception as e:  # reported; the torch path's results stand
            rep.update({"path": "torch.distributed all_gather_into_tensor (C-ABI collective failed)",
                        "c_abi_error": str(e), "ms": round(1e3 * t_torch, 3),
                        "gbps": round(nbytes / t_torch / 1e9, 1)})
    else:
        rep.update({"path": f"torch.distributed all_gather_into_tensor ({ri.backend} rehearsal)",
                    "ms": round(1e3 * t_torch, 3), "gbps": round(nbytes / t_torch / 1e9, 1)})
    log(f"[bench r{rank}] all-gather of {nbytes / 1e9:.2f} GB: {rep}")
    return rep, (g_rows_np, g_elem, g_hit)


def split_parity(w, bg, met, fields, new, pclass, shards, gathered, budget_s: float) -> dict:
    """Split modes, rank 0: the all-gathered results of every rank, placed at
    their group points, against an oracle run over the whole group (the
    reference's visitation order cut into one range per thread, as the CPU
    baseline, stopped after `budget_s`): every point the oracle processed is
    checked (tests/parity.py contract: class (i) identity, acceptance, values
    of the reference interpolator in the chosen element), and every point of
    the group must have been located by some rank."""
    from oracle import oracle as O

    g_rows, g_elem, g_hit = gathered
    idx_all = np.concatenate(shards)
    n = new.xyz.shape[0]
    elem = np.zeros(n, np.int32)
    hit = np.zeros(n, np.int8)
    elem[idx_all], hit[idx_all] = g_elem, g_hit
    widths = [met.shape[1]] + [f.shape[1] for f in fields]
    outs, c0 = [], 0
    for wd in widths:
        a = np.full((n, wd), np.nan)
        a[idx_all] = g_rows[:, c0:c0 + wd]
        outs.append(a)
        c0 += wd
    threads, _ = host_cores()
    t0 = time.time()
    new_t = synth.lattice(w.kind, w.n_new, jitter=w.jitter_new, seed=synth.SEED, with_trias=False)
    order = synth.visit_order(new_t)
    del new_t
    B = O.Background(bg, met, fields, w.hausd)
    ref = O.run(B, new.xyz, pclass, order, budget_s=budget_s, threads=threads)
    t_run = time.time() - t0
    pr = parity_report(B, new, pclass, {"elem": elem, "hit": hit, "met": outs[0], "fields": outs[1:]}, ref)
    missing = int(((pclass != 0) & (hit == 0)).sum())
    pr["what"] = ("all-gathered results of every rank (group ids) vs an oracle run over the whole group, every "
                  "point it processed")
    pr["points_group"] = int((pclass != 0).sum())
    pr["points_not_located_by_any_rank"] = missing
    pr["oracle_s"] = round(t_run, 1)
    pr["ok"] = bool(pr["ok"] and missing == 0)
    return pr


def snapshot_timing(ctx, bg, rank: int, reps: int = 3):
    """Device background snapshot (PMMG_create_oldGrp's
    adjacency / boundary trias / tria adjacency, pmmg_hip_build_*) timed on
    its own, outside the transfer step, checked against the host-built
    arrays the step uses."""
    d_tetv = ctx.upload(bg.tetv)
    d_tet8 = ctx.empty((bg.ne, 8), np.int32)  # the caller's old-group array, kept across iterations
    times = []
    ok = True
    for rep in range(reps + 1):  # the first call sizes the context's snapshot scratch (untimed)
        if rep == reps:
            d_tet8.zero()  # the checked call writes every record again
        t0 = time.perf_counter()
        adja, tet8 = ctx.build_adjacency(bg.np, d_tetv, adja=False, tet8=True, out=(None, d_tet8))
        t1 = time.perf_counter()
        triv, adjt = ctx.build_boundary(bg.np, tet8=tet8)
        t2 = time.perf_counter()
        if rep > 0:
            times.append((t1 - t0, t2 - t1))
        ok = ok and bool(np.array_equal(adjt.download(), bg.adjt))
        if rep == reps:
            ok = ok and bool(np.array_equal(tet8.download(), pack_tet8(bg.tetv, bg.adja)))
            ok = ok and bool(np.array_equal(triv.download(), bg.triv))
        for a in (triv, adjt):
            a.free()
    d_tetv.free()
    d_tet8.free()
    t_adj = float(np.median([t[0] for t in times]))
    t_bdy = float(np.median([t[1] for t in times]))
    b_adj = bg.ne * (16 + 32)  # tetv in, tet8 records out
    log(f"[bench r{rank}] snapshot: adjacency {1e3 * t_adj:.2f} ms, boundary {1e3 * t_bdy:.2f} ms, match={ok}")
    return {"what": "pmmg_hip_build_adjacency (tet8 out) + pmmg_hip_build_boundary, not part of the step",
            "ms_adjacency": round(1e3 * t_adj, 3), "ms_boundary": round(1e3 * t_bdy, 3),
            "tets": bg.ne, "trias": bg.nt, "matches_host_builder": ok,
            "adjacency_algorithmic_gbps": round(b_adj / t_adj / 1e9, 1)}


def quality_timing(ctx, w, d_qxyz, d_mo, rank: int, reps: int = 3):
    """PMMG_tetraQual on the new mesh in the device-resident interpolated
    metric (pmmg_hip_tetra_qual), timed on its own
    after the step."""
    new_t = synth.lattice(w.kind, w.n_new, jitter=0.0, with_trias=False)  # connectivity only (same numbering)
    d_tetv = ctx.upload(new_t.tetv)
    ne = new_t.ne
    del new_t
    met = d_mo if w.met_size == 6 else None
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        qual, mn = ctx.tetra_qual(d_qxyz, d_tetv, met)
        times.append(time.perf_counter() - t0)
        qual.free()
    d_tetv.free()
    t = float(np.median(times))
    nb = ne * (16 + 8) + d_qxyz.shape[0] * (24 + (8 * w.met_size if met is not None else 0))
    log(f"[bench r{rank}] tetra quality of {ne} new tetra: {1e3 * t:.3f} ms, min {mn:.4f}")
    return {"what": "pmmg_hip_tetra_qual (PMMG_tetraQual / MMG3D_tetraQual) in the interpolated metric, "
                    "not part of the step", "tets": ne, "ms": round(1e3 * t, 3), "minqual": mn,
            "algorithmic_gbps": round(nb / t / 1e9, 1)}


def host_mode_timing(ctx, w, bg, met, fields, q_xyz, q_pc, rank: int, reps: int = 3):
    """End-to-end rate with host buffers (PMMG_HIP_HOST), as the C host layer
    runs a group inside ParMmg: the vertices and tetra vertex ids go up
    through the context's pinned staging buffers, the adjacency and the
    boundary trias are built on the device (PMMG_create_oldGrp's arrays, not
    uploaded), then the solutions and queries go up, the step runs and the
    rows it wrote come back.  Reported beside the HBM-resident step, never as
    the bench value: the median of `reps` calls (the first also pays the first
    touch of the output pages and of the staging buffers)."""
    nq = q_xyz.shape[0]
    mo = np.empty((nq, w.met_size), np.float64)
    fo = [np.empty((nq, f.shape[1]), np.float64) for f in fields]
    elem, hit = np.empty(nq, np.int32), np.empty(nq, np.int8)
    tb, ts, tl = [], [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        ctx.set_background(bg.xyz, bg.tetv, None, None, None, w.hausd)
        t1 = time.perf_counter()
        ctx.set_solutions(met, fields)
        t2 = time.perf_counter()
        st = ctx.locate_interp(q_xyz, q_pc, mo, fo, elem, hit)
        t3 = time.perf_counter()
        tb.append(t1 - t0)
        ts.append(t2 - t1)
        tl.append(t3 - t2)
    b, s_, l_ = (float(np.median(x)) for x in (tb, ts, tl))
    t = b + s_ + l_
    up = bg.xyz.nbytes + bg.tetv.nbytes + met.nbytes + sum(f.nbytes for f in fields) + q_xyz.nbytes + q_pc.nbytes
    down = mo.nbytes + sum(f.nbytes for f in fo) + elem.nbytes + hit.nbytes
    npts = int(st.nvol + st.nbdy)
    log(f"[bench r{rank}] host-buffer (PCIe-inclusive) call: {1e3 * t:.1f} ms "
        f"(background {1e3 * b:.1f}, solutions {1e3 * s_:.1f}, locate {1e3 * l_:.1f})")
    out = {"what": "one group through host buffers as the C host layer runs it: background (xyz + tetv up, "
                   "adjacency and boundary trias built on the device), solutions up, queries up + the step + the "
                   "written rows down; not the bench value",
           "ms": round(1e3 * t, 2), "ms_background": round(1e3 * b, 2), "ms_solutions": round(1e3 * s_, 2),
           "ms_locate_interp": round(1e3 * l_, 2), "mpts_per_s": round(npts / t / 1e6, 1),
           "bytes_up": int(up), "bytes_down": int(down), "pcie_gbps_effective": round((up + down) / t / 1e9, 1)}
    try:
        out["iteration2"] = host_mode_iteration2(ctx, w, bg, met, fields, rank)
    except Exception as e:  # reported, never fatal to the bench line
        out["iteration2"] = {"error": str(e)}
    return out


def host_mode_iteration2(ctx, w, bg, met, fields, rank: int) -> dict:
    """The next iteration through host buffers (src/libparmmg1.c:653: the
    adapted group becomes the old group): its background is the new mesh just
    transferred into (the new points, with the rows the step wrote) and the
    next new mesh has the first background's points (synthetic stand-in).
    Timed twice: cold (everything uploaded) and carried (pmmg_hip_keep after
    the first iteration, pmmg_hip_carry_over: only the connectivity and the
    next queries go up), outputs compared bit for bit; bytes_up counted by
    the module.

    The adapted mesh must be a valid mesh, as Mmg's output is: its points are
    jittered with the cap of synth_vertices_valid (r06).  Up to r05 this leg
    used the plainly jittered shell, whose lattice connectivity has 0.23 % of
    its tetra inverted along the radial map's crease planes (|y_i| = |y_j|):
    2655 walks cycled through them to the step cap and the exhaustive search
    (tools/walk_emu.py reproduces it on the CPU: 164 of 258k walks at n = 68 /
    72, none once the mesh is valid).  So this leg runs its own first
    iteration, on those points, and keeps that call."""
    new_t = synth.lattice(w.kind, w.n_new, jitter=w.jitter_new, seed=synth.SEED, with_trias=False, valid=True)
    pc1 = synth.classes(new_t)
    mo = np.empty((new_t.np, w.met_size), np.float64)
    fo = [np.empty((new_t.np, f.shape[1]), np.float64) for f in fields]
    ctx.set_background(bg.xyz, bg.tetv, None, None, None, w.hausd)
    ctx.set_solutions(met, fields)
    ctx.locate_interp(new_t.xyz, pc1, mo, fo)
    ctx.keep(0)  # this first iteration's call stays on the device
    q2, pc2 = bg.xyz, synth.classes(bg)
    res = {}
    outs = {}
    for mode in ("cold", "carried"):
        m2 = np.full((q2.shape[0], mo.shape[1]), np.nan)
        f2 = [np.full((q2.shape[0], f.shape[1]), np.nan) for f in fo]
        el2, hit2 = np.zeros(q2.shape[0], np.int32), np.zeros(q2.shape[0], np.int8)
        if mode == "carried":
            ctx.carry_over(0, new_t.np)
        ctx.bytes_up(reset=True)
        t0 = time.perf_counter()
        ctx.set_background(new_t.xyz, new_t.tetv, None, None, None, w.hausd)
        ctx.set_solutions(mo, fo)
        st = ctx.locate_interp(q2, pc2, m2, f2, el2, hit2)
        t = time.perf_counter() - t0
        sd = st.as_dict()
        res[mode] = {"ms": round(1e3 * t, 2), "bytes_up": ctx.bytes_up(reset=True),
                     "located_points": int(st.nvol + st.nbdy),
                     # the walks' hand-overs and the exhaustive searches they needed
                     "locate_stats": locate_stats(st),
                     "device_ms": {"step_total": round(float(st.ms_total), 3),
                                   "volume_fallback": round(float(st.ms_fallback), 3),
                                   "surface_branch": round(float(st.ms_bdy), 3)}}
        outs[mode] = [m2] + f2 + [el2, hit2]
    same = all(np.array_equal(a, b, equal_nan=True) for a, b in zip(outs["cold"], outs["carried"]))
    try:
        res["oracle_check"] = iteration2_oracle_check(new_t, mo, fo, w, q2, pc2, outs["cold"])
    except Exception as e:  # reported, never fatal to the bench line
        res["oracle_check"] = {"error": str(e)}
    res.update({"what": "second iteration through host buffers: background = the new mesh of the first "
                        f"({new_t.ne} tets, {new_t.np} verts), queries = the first background's points; cold vs "
                        "carried over from the device (pmmg_hip_keep / pmmg_hip_carry_over)",
                "bytes_up_saved_frac": round(1 - res["carried"]["bytes_up"] / max(1, res["cold"]["bytes_up"]), 3),
                "bit_identical": bool(same)})
    log(f"[bench r{rank}] host-mode iteration 2: {res}")
    return res


def iteration2_oracle_check(new_t, mo, fo, w, q2, pc2, out, nsample: int = 20000) -> dict:
    """The second iteration's rows against the oracle on its background (the
    first iteration's valid new mesh with the rows written into it): every
    volume point the exhaustive search settled — its element must be the
    reference's lowest accepting index (src/locate_pmmg.c:737-770) or, when
    none accepts, the closest — and a seeded sample of the other volume
    points, with the parity contract of tests/parity.py (orc_check_batch).
    Surface points are not checked here (the background's trias are built on
    the device in this leg)."""
    from oracle import oracle as orc

    m2, f2, el2, hit2 = out[0], out[1:-2], out[-2], out[-1]
    bgo = orc.Background(new_t, mo, fo, w.hausd)
    code = hit2 & 15
    fb = np.nonzero((pc2 == 1) & ((code == 2) | (code == 3)))[0]
    rng = np.random.default_rng(20260)
    vol = np.nonzero(pc2 == 1)[0]
    samp = np.unique(np.concatenate([fb, rng.choice(vol, size=min(nsample, vol.size), replace=False)]))
    rep = orc.check_batch(bgo, q2, pc2, el2, hit2, m2, f2, idx=samp)
    fbc = fb[:200]  # each an O(ne) scan on the CPU
    lowest = sum(int(orc.first_accepting_tetra(bgo, q2[i]) == el2[i]) for i in fbc if code[i] == 2)
    closest = sum(int(orc.first_accepting_tetra(bgo, q2[i]) == 0 and orc.closest_tetra(bgo, q2[i]) == el2[i])
                  for i in fbc if code[i] == 3)
    ok = rep["accept_fail"] == 0 and rep["value_fail"] == 0 and rep["unprocessed"] == 0
    return {"points_checked": int(samp.size), "fallback_points": int(fb.size), "fallback_checked": int(fbc.size),
            "fallback_lowest_accepting_same": lowest, "fallback_closest_same": closest,
            "contract": rep, "ok": bool(ok and lowest + closest == fbc.size)}


LOCATE_KEYS = ("nvol", "nbdy", "nvol_exact", "nvol_stuck", "nvol_limit", "nvol_noseed", "nvol_exhaust",
               "nvol_closest", "nbdy_exhaust", "nbdy_stale", "nbdy_closest", "stepmax")


def locate_stats(st) -> dict:
    """the walks' hand-overs and the exhaustive searches a leg's call needed
    (every leg that can reach a fallback reports them)"""
    d = st.as_dict()
    return {k: int(d[k]) for k in LOCATE_KEYS}


def renumbered_timing(ctx, args, w, step_bg, q_xyz, q_pc, d_mo, d_fo, d_elem, d_hit, rank: int, perm, what: str,
                      records=None):
    """The same step on a renumbering of the new points (perm[new id] = old
    id); the module decides on the device whether the numbering is
    spatially coherent (input order) or Morton-bins the queries.  Reported
    beside the bench value, which is measured on the generator's lattice
    numbering.  Checked against the input-order step: a point located in
    the same element gets bit-identical rows.

    records = the packed solution records in HBM (pack_solutions): the step
    then reads them (pmmg_hip_set_solutions_packed) and writes its rows as
    records of the same layout (pmmg_hip_locate_interp_rec), one 128-byte
    line per point where the reference's layout scatters four arrays' rows."""
    nq = q_xyz.shape[0]
    s_xyz, s_pc = ctx.upload(np.ascontiguousarray(q_xyz[perm])), ctx.upload(np.ascontiguousarray(q_pc[perm]))
    sizes = [w.met_size] + [f.shape[1] for f in d_fo]
    if records is None:
        s_mo = ctx.empty((nq, w.met_size), np.float64)
        s_fo = [ctx.empty(f.shape, np.float64) for f in d_fo]
    else:
        s_rec = ctx.empty((nq, records.shape[1]), np.float64)
    s_elem, s_hit = ctx.empty((nq,), np.int32), ctx.empty((nq,), np.int8)

    def step():
        step_bg()
        if records is None:
            ctx.locate_interp(s_xyz, s_pc, s_mo, s_fo, s_elem, s_hit, sync=False)
        else:
            ctx.set_solutions_packed(records, w.met_size, sizes[1:])
            ctx.locate_interp_rec(s_xyz, s_pc, s_rec, s_elem, s_hit, sync=False)

    for _ in range(args.warmup):
        step()
        ctx.sync()
    ms, vol = [], []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        st = ctx.sync()
        ms.append(st.ms_total)
        vol.append(st.ms_vol)
    wall = (time.perf_counter() - t0) / args.steps
    # the input-order step's outputs (d_*) against the shuffled step's, point by point
    inv = np.argsort(perm)
    e0, e1 = d_elem.download(), s_elem.download()[inv]
    h0, h1 = d_hit.download(), s_hit.download()[inv]
    located = (h0 != 0) & (h1 != 0)
    same = located & (e0 == e1) & (h0 == h1)
    ident = same.copy()
    if records is None:
        got = [b.download()[inv] for b in [s_mo] + s_fo]
    else:
        r = s_rec.download()[inv]
        offs = np.cumsum([0] + sizes)
        got = [r[:, offs[j]:offs[j + 1]] for j in range(len(sizes))]
        s_rec.free()
    for a, x1 in zip([d_mo] + list(d_fo), got):
        x0 = a.download()
        ident &= np.all(x0.view(np.uint64) == np.ascontiguousarray(x1).view(np.uint64), axis=1)
    npts = int(st.nvol + st.nbdy)
    res = {"what": what,
           "morton_binned": bool(st.sorted), "ms_per_step": round(1e3 * wall, 4),
           "mpts_per_s": round(npts / wall / 1e6, 1), "device_ms_total": round(float(np.mean(ms)), 4),
           "volume_stage_ms": round(float(np.mean(vol)), 4),
           "locate_stats": locate_stats(st),
           "located_points": int(located.sum()), "same_element_as_input_order": int(same.sum()),
           "same_element_rows_bit_identical": int((same & ident).sum()),
           "ok": bool(np.all(ident[same])) and int(located.sum()) == npts}
    log(f"[bench r{rank}] renumbered ({what}): {res}")
    for b in [s_xyz, s_pc, s_elem, s_hit] + ([s_mo] + s_fo if records is None else []):
        b.free()
    return res


def surface_solo(ctx, step_bg, q_xyz, q_pc, d_mo, d_fo, d_elem, d_hit, device: int, reps: int = 5) -> dict:
    """The surface branch (k_seed_srf + k_bdy + its fallbacks, second
    stream) timed alone: the same call with every volume point marked
    skipped, the branch starting after the seed grid kernels of the main
    stream as in a large call's step.  In the full step it overlaps the
    volume kernel."""
    pc = np.where(q_pc == 2, 2, 0).astype(np.uint8)
    d_pc = ctx.upload(pc)
    ms_bdy, ms_tot = [], []
    for r in range(reps + 1):
        step_bg(ctx)
        ctx.locate_interp(q_xyz, d_pc, d_mo, d_fo, d_elem, d_hit, sync=False)
        st = ctx.sync()
        if r:
            ms_bdy.append(st.ms_bdy)
            ms_tot.append(st.ms_total)
    d_pc.free()
    return {"what": "surface branch alone (volume points skipped): HIP events of the surface stream, "
                    "starting after the seed grid as in a large call's step",
            "surface_points": int(st.nbdy), "locate_stats": locate_stats(st),
            "ms_branch": round(float(np.median(ms_bdy)), 4),
            "ms_call": round(float(np.median(ms_tot)), 4)}


def graded_leg(args, rank: int, budget_s: float = 60.0) -> dict:
    """cfgG (configs.CFGG): cfg3's lattices graded 1000x towards three planes
    and sheared (elements up to ~1000:1, the geometry of the reference's
    anisotropic torus-with-a-planar-shock runs), the same step timed in its
    own context, with the fp32 filter walk's hand-overs to the exact walk
    (nvol_exact), the longest walk and the steps per point, and every point
    checked against an oracle run (reported beside the bench value)."""
    w = configs.CFGG
    bg, new = configs.build_meshes(w, seed=synth.SEED, with_new_tetra=True)
    visit = synth.visit_order(new)
    pc = synth.classes(new)
    met = synth.solution(w.metric, bg.xyz)
    fields = [synth.solution(f, bg.xyz) for f in w.fields]
    stats = synth.cell_stats(bg)
    ctx = TransferContext(0)
    d_xyz, d_tet8 = ctx.upload(bg.xyz), ctx.upload(pack_tet8(bg.tetv, bg.adja))
    d_triv, d_adjt = ctx.upload(bg.triv), ctx.upload(bg.adjt)
    d_met, d_f = ctx.upload(met), [ctx.upload(f) for f in fields]
    d_q, d_pc = ctx.upload(new.xyz), ctx.upload(pc)
    nq = new.np
    d_mo = ctx.empty((nq, w.met_size), np.float64)
    d_fo = [ctx.empty((nq, f.shape[1]), np.float64) for f in fields]
    d_el, d_hit = ctx.empty((nq,), np.int32), ctx.empty((nq,), np.int8)

    def step():
        ctx.set_background_tet8(d_xyz, d_tet8, d_triv, d_adjt, w.hausd)
        ctx.set_solutions(d_met, d_f)
        ctx.locate_interp(d_q, d_pc, d_mo, d_fo, d_el, d_hit, sync=False)

    for _ in range(max(1, args.warmup)):
        step()
        ctx.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    st = ctx.sync()
    wall = (time.perf_counter() - t0) / args.steps
    gpu = {"elem": d_el.download(), "hit": d_hit.download(), "met": d_mo.download(),
           "fields": [f.download() for f in d_fo]}
    ctx.close()
    npts = int(st.nvol + st.nbdy)
    out = {"what": "cfgG: the step on a graded (1000x towards three planes per mesh, the new mesh's planes moved) "
                   "and sheared cube (cfg3's lattices), own context; not the bench value",
           "workload": w.name, "background_tets": bg.ne, "new_points": nq,
           "size_grading": round(stats["size_grading"], 1), "max_aspect_ratio": round(stats["max_aspect"], 1),
           "ms_per_step": round(1e3 * wall, 4), "mpts_per_s": round(npts / wall / 1e6, 1),
           "volume_stage_ms": round(float(st.ms_vol), 4), "nvol": int(st.nvol), "nvol_exact": int(st.nvol_exact),
           "nvol_exhaust": int(st.nvol_exhaust), "stepmax": int(st.stepmax), "locate_stats": locate_stats(st),
           "walk_steps_per_point": round(st.steps_total / max(1, npts), 3)}
    if not args.no_cpu_baseline:
        from oracle import oracle as O
        threads, _ = host_cores()
        B = O.Background(bg, met, fields, w.hausd)
        ref = O.run(B, new.xyz, pc, visit, budget_s=budget_s, threads=threads)
        out["parity"] = parity_report(B, new, pc, gpu, ref)
    log(f"[bench r{rank}] graded leg: {out}")
    return out


def groups_leg(args, ngroup: int = 10, reps: int = 5, budget_s: float = 30.0) -> dict:
    """ParMmg's loop over a rank's groups (src/interpmesh_pmmg.c:690): ngroup
    cfg2-size groups (own copies of the background, solutions and new points
    in HBM, the new points jittered with their own seeds), timed as one
    pmmg_hip_locate_interp_groups call against the same groups one
    pmmg_hip_locate_interp each; the outputs of the groups call are checked
    bit for bit against the per-group calls', and group 0's against an oracle
    run (parity)."""
    w = configs.CFG2
    ctx = TransferContext(0)
    gs, hosts = [], []
    for i in range(ngroup):
        bg, new, met, fields, pc = build_workload(w, 100 + i)
        nq = new.np
        gs.append(dict(xyz=ctx.upload(bg.xyz), tet8=ctx.upload(pack_tet8(bg.tetv, bg.adja)), triv=ctx.upload(bg.triv),
                       adjt=ctx.upload(bg.adjt), hausd=w.hausd, met=ctx.upload(met),
                       fields=[ctx.upload(f) for f in fields], xyz_new=ctx.upload(new.xyz), pclass=ctx.upload(pc),
                       met_out=ctx.empty((nq, w.met_size), np.float64),
                       fields_out=[ctx.empty((nq, f.shape[1]), np.float64) for f in fields],
                       elem_out=ctx.empty((nq,), np.int32), hit_out=ctx.empty((nq,), np.int8)))
        hosts.append((bg, new, met, fields, pc) if i == 0 else None)

    def one_by_one():
        for g in gs:
            ctx.set_background_tet8(g["xyz"], g["tet8"], g["triv"], g["adjt"], g["hausd"])
            ctx.set_solutions(g["met"], g["fields"])
            ctx.locate_interp(g["xyz_new"], g["pclass"], g["met_out"], g["fields_out"], g["elem_out"], g["hit_out"],
                              sync=False)

    def download():
        return [{"elem": g["elem_out"].download(), "hit": g["hit_out"].download(), "met": g["met_out"].download(),
                 "fields": [f.download() for f in g["fields_out"]]} for g in gs]

    def timed(fn, trials: int = 7):
        """median over `trials` timings of `reps` back-to-back repetitions
        (one repetition of 10 cfg2-size groups is ~1 ms: a single timing
        swung by 20 % between runs on one box, r05w / r05x)"""
        fn()
        ctx.sync()
        ts, es = [], []
        for _ in range(trials):
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            es.append(time.perf_counter() - t0)
            ctx.sync()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)) / (reps * ngroup), float(np.median(es)) / (reps * ngroup)

    t_single, e_single = timed(one_by_one)
    ref_out = download()
    for g in gs:  # the groups call must write every row again
        for a in [g["met_out"], g["elem_out"], g["hit_out"]] + g["fields_out"]:
            a.zero()
    t_groups, e_groups = timed(lambda: ctx.locate_interp_groups(gs, sync=False))
    st = ctx.locate_interp_groups(gs, sync=True)
    out_g = download()
    same = all(np.array_equal(a[k], b[k], equal_nan=True) for a, b in zip(out_g, ref_out)
               for k in ("elem", "hit", "met")) and all(
        np.array_equal(x, y, equal_nan=True) for a, b in zip(out_g, ref_out) for x, y in zip(a["fields"], b["fields"]))
    npts = int(st.nvol + st.nbdy)
    lmax = max(1, int(os.environ.get("PMMG_HIP_GROUP_LANES", "3")))
    rounds = -(-ngroup // lmax)
    lanes = min(ngroup, -(-ngroup // rounds))  # as pmmg_hip_locate_interp_groups deals them
    res = {"what": f"{ngroup} cfg2-size groups (own copies in HBM) in one pmmg_hip_locate_interp_groups call vs one "
                   "pmmg_hip_locate_interp per group (median of 7 timings of 5 repetitions); not the bench value",
           "groups": ngroup, "lanes": lanes, "points_per_group": npts // ngroup,
           "ms_per_group_groups_call": round(1e3 * t_groups, 4), "ms_per_group_single_calls": round(1e3 * t_single, 4),
           "host_enqueue_ms_per_group": {"groups_call": round(1e3 * e_groups, 4), "single_calls": round(1e3 * e_single, 4)},
           "mpts_per_s_groups_call": round(npts / ngroup / t_groups / 1e6, 1),
           "bit_identical_to_single_calls": bool(same), "locate_stats": locate_stats(st)}
    ctx.close()
    if not args.no_cpu_baseline:
        from oracle import oracle as O
        bg, new, met, fields, pc = hosts[0]
        threads, _ = host_cores()
        B = O.Background(bg, met, fields, w.hausd)
        new_t = synth.lattice(w.kind, w.n_new, jitter=w.jitter_new, seed=synth.SEED + 100, with_trias=False)
        ref = O.run(B, new.xyz, pc, synth.visit_order(new_t), budget_s=budget_s, threads=threads)
        res["parity_group0"] = parity_report(B, new, pc, out_g[0], ref)
    log(f"[bench] groups leg: {res}")
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg4", choices=sorted(configs.SHORT))
    ap.add_argument("--sort", default="auto", choices=["auto", "on", "off"],
                    help="query order: Morton binning (on), input order (off), or chosen on the device")
    ap.add_argument("--tpc", type=int, default=0, help="background tetra per volume seed cell (0: module default)")
    ap.add_argument("--layout", default="tet8", choices=["tet8", "separate"],
                    help="HBM layout of the tetra: packed {v[4], adja[4]} records or separate tetv/adja arrays")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=30.0,
                    help="cap of the CPU baseline's locate phase: a bounded sample of ~10-30 s of CPU work (cfg4 on "
                         "16 threads: ~6M of the 20.3M points, a contiguous range of the visitation order per thread); "
                         "the parity check covers every point it processed")
    ap.add_argument("--no-cpu-baseline", action="store_true", help="skip the CPU baseline (and the parity check)")
    ap.add_argument("--split-parity-seconds", type=float, default=30.0,
                    help="split modes: cap of the oracle run (whole group, all threads) that checks the gathered results")
    ap.add_argument("--shard", default="auto", choices=["auto", "group", "morton", "halo"],
                    help="multi-GPU split (auto: halo for N > 1): Morton ranges of the new points against halo "
                         "shards of the background (halo) or a replicated background (morton), results "
                         "all-gathered over RCCL after the timed steps; or one group per rank (group, weak)")
    ap.add_argument("--split", default="rcb", choices=["rcb", "morton"],
                    help="split modes: the new points cut by recursive coordinate bisection (compact boxes of equal "
                         "cost) or into contiguous Morton ranges")
    ap.add_argument("--shard-build", default="parts", choices=["parts", "group"],
                    help="halo mode: each rank's shard assembled from every rank's part of the group (all-to-all), "
                         "or cut from the whole group")
    ap.add_argument("--halo", type=float, default=-1.0,
                    help="halo mode: growth of the range box (< 0: in largest-tetra extents, at least hausd)")
    ap.add_argument("--no-host-mode", action="store_true",
                    help="skip the (separately reported) host-buffer, PCIe-inclusive call")
    ap.add_argument("--no-quality", action="store_true",
                    help="skip the (separately reported) tetra-quality timing of the new mesh")
    ap.add_argument("--no-shuffled", action="store_true",
                    help="skip the (separately reported) step on a shuffled numbering of the new points")
    ap.add_argument("--no-snapshot", action="store_true",
                    help="skip the (separately reported) device background snapshot timing")
    ap.add_argument("--no-surface-solo", action="store_true",
                    help="skip the (separately reported) surface branch timed alone")
    ap.add_argument("--no-groups", action="store_true",
                    help="skip the (separately reported) 10 cfg2-size groups in one groups call")
    ap.add_argument("--no-graded", action="store_true",
                    help="skip the (separately reported) step on the graded and stretched cfgG meshes")
    args = ap.parse_args()

    # PMMG_BENCH_BACKEND=gloo: host-side collectives, ranks share the visible
    # GPUs round-robin (rehearsing several ranks on a one-GPU box)
    backend = os.environ.get("PMMG_BENCH_BACKEND", "nccl")
    ri = ranks.init(backend)
    rank, world, local = ri.rank, ri.world, ri.local
    if backend != "nccl":
        import torch
        local = local % max(1, torch.cuda.device_count())
    shard_mode = args.shard if args.shard != "auto" else ("halo" if world > 1 else "group")

    w = configs.SHORT[args.config]
    split = shard_mode in ("morton", "halo")
    # split modes: every rank builds the same problem and keeps its range
    bg, new, met, fields, pclass = build_workload(w, 0 if split else rank)
    ne_group = bg.ne
    bg_group, met_group, fields_group = bg, met, fields
    counts = None
    halo_info = None
    sh = None
    if split:
        shards = (ranks.rcb_shards if args.split == "rcb" else ranks.morton_shards)(new.xyz, pclass, world)
        mine = shards[rank]
        counts = [len(x) for x in shards]
        q_xyz, q_pc = np.ascontiguousarray(new.xyz[mine]), np.ascontiguousarray(pclass[mine])
        log(f"[bench r{rank}] {args.split} part: {len(mine)} of {int((pclass != 0).sum())} points")
        if shard_mode == "halo":
            from parmmg_amd import shard
            t_sh = time.time()
            built = "whole group (halo_shard_cells)"
            if args.shard_build == "parts":
                # every rank keeps only its part of the group (pmmg_shard_part_pack), the parts are exchanged
                # all-to-all and assembled (pmmg_shard_assemble): the shard the whole-group builder makes
                try:
                    sol = np.concatenate([met] + list(fields), axis=1)
                    part = shard.part_of(bg, sol, rank, world)
                    # the halo and the grid from the parts too (shard.parts_frame: all-reduced extent and box)
                    sh = shard.shard_from_parts(ri, part, q_xyz, args.halo, kind=bg.kind, n=bg.n, hausd=w.hausd)
                    del part
                    c0 = met.shape[1]
                    met, fields = sh.sol[:, :c0].copy(), []
                    for f in fields_group:
                        fields.append(np.ascontiguousarray(sh.sol[:, c0:c0 + f.shape[1]]))
                        c0 += f.shape[1]
                    bg = sh.mesh
                    built = "the ranks' parts (pmmg_shard_part_pack, all-to-all, pmmg_shard_assemble)"
                except Exception as e:  # reported; the whole-group builder stands in
                    log(f"[bench r{rank}] shard from parts failed: {e}")
                    built = f"whole group (the parts' build failed: {e})"
                    sh = None
            if sh is None or args.shard_build != "parts":
                sh = shard.halo_shard_cells(bg, q_xyz, args.halo, hausd=w.hausd)
                bg, met, fields = sh.mesh, sh.rows(met), [sh.rows(f) for f in fields]
            halo_info = {"what": "halo shard of the background around this rank's Morton range (rank 0): the tetra "
                                 "meeting, grown by the halo, the range's box and a halo-sized grid cell holding "
                                 "one of its points", "built_from": built,
                         "tets": bg.ne, "verts": bg.np, "trias": bg.nt, "halo": sh.halo,
                         "tet_fraction_of_group": round(bg.ne / ne_group, 4),
                         "build_s": round(time.time() - t_sh, 2)}
            log(f"[bench r{rank}] halo shard: {bg.ne} of {ne_group} tets, {bg.np} verts, {bg.nt} trias "
                f"(halo {sh.halo:.4g}) in {time.time() - t_sh:.1f}s")
    else:
        q_xyz, q_pc = new.xyz, pclass
    nq = q_xyz.shape[0]

    if args.tpc > 0:
        os.environ["PMMG_HIP_TPC"] = str(args.tpc)  # read by pmmg_hip_create
    ctx = TransferContext(local, sort={"auto": None, "on": True, "off": False}[args.sort])
    d_xyz = ctx.upload(bg.xyz)
    if args.layout == "tet8":
        d_tet8 = ctx.upload(pack_tet8(bg.tetv, bg.adja))
    else:
        d_tetv, d_adja = ctx.upload(bg.tetv), ctx.upload(bg.adja)
    d_triv, d_adjt = ctx.upload(bg.triv), ctx.upload(bg.adjt)
    d_met = ctx.upload(met)
    d_f = [ctx.upload(f) for f in fields]
    d_qxyz, d_pc = ctx.upload(q_xyz), ctx.upload(q_pc)
    if split:
        # outputs as torch tensors in HBM: the all-gather reads them in place
        import torch
        dev = torch.device("cuda", local)
        d_mo = torch.empty((nq, w.met_size), dtype=torch.float64, device=dev)
        d_fo = [torch.empty((nq, f.shape[1]), dtype=torch.float64, device=dev) for f in fields]
        d_elem = torch.empty((nq,), dtype=torch.int32, device=dev)
    else:
        d_mo = ctx.empty((nq, w.met_size), np.float64)
        d_fo = [ctx.empty((nq, f.shape[1]), np.float64) for f in fields]
        d_elem = ctx.empty((nq,), np.int32)
    d_hit = ctx.empty((nq,), np.int8)

    def step_bg(c=None):
        c = ctx if c is None else c
        if args.layout == "tet8":
            c.set_background_tet8(d_xyz, d_tet8, d_triv, d_adjt, w.hausd)
        else:
            c.set_background(d_xyz, d_tetv, d_adja, d_triv, d_adjt, w.hausd)
        c.set_solutions(d_met, d_f)

    def step():
        step_bg()
        ctx.locate_interp(d_qxyz, d_pc, d_mo, d_fo, d_elem, d_hit, sync=False)

    log(f"[bench r{rank}] inputs resident in HBM; warmup {args.warmup} steps")
    for wi in range(args.warmup):
        t_w = time.perf_counter()
        step()
        st0 = ctx.sync()
        log(f"[bench r{rank}] warmup {wi}: {1e3 * (time.perf_counter() - t_w):.2f} ms wall, device {st0.as_dict()}")
    # timed region: barrier + device sync on both sides
    ranks.barrier(ri)
    ctx.sync()
    # the K steps are enqueued back to back (each call only enqueues; the
    # host's enqueue of step i+1 overlaps the device's step i), synchronised
    # once at the end
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ranks.barrier(ri)
    st = ctx.sync()
    elapsed = time.perf_counter() - t0
    log(f"[bench r{rank}] timed {args.steps} steps: {1e3 * elapsed / args.steps:.3f} ms/step")
    st_timed = st  # HIP events of the last timed step (the roofline's stage time)
    # per-stage device times of every step (HIP events): the same K steps
    # again, each followed by a read of its event times (reported as means)
    ms_vol, ms_tot, ms_walk = [], [], []
    for _ in range(args.steps):
        step()
        st = ctx.sync()
        ms_vol.append(st.ms_vol)
        ms_tot.append(st.ms_total)
        ms_walk.append(st.ms_vol_locate)

    npts = int(st.nvol + st.nbdy)
    agg = ranks.aggregate(ri, npts, elapsed, args.steps)
    gather = gathered = None
    if split:
        gather, gathered = allgather_timing(ri, ctx, d_mo, d_fo, d_elem, d_hit, sh, counts, rank)
        npts = agg["points_per_step"]  # the whole problem: bytes per point below are per problem point
    ms_per_step = agg["ms_per_step"]
    value = agg["mpts_per_s"]
    (np_o, ne_o, _), (np_n, _, _) = w.counts()
    B = w.algorithmic_bytes(npts)
    per_pt = B / npts
    kvol_ms = float(st_timed.ms_vol)
    kvol_bytes = per_pt * st.nvol
    achieved = kvol_bytes / (kvol_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(w.name) if not split else (None, "not profiled per rank")
    steps_pp = st.steps_total / max(1, st.nvol + st.nbdy)
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Mpts/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        # N = 1 is the first point of the default N > 1 curve (the same cfg4
        # group split over the GPUs: strong scaling); --shard group is weak
        "scaling": "weak" if (shard_mode == "group" and world > 1) or args.shard == "group" else "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (Kuhn lattices, analytic metric/fields, splitmix64 jitter)",
        "config": {
            "workload": w.name,
            "description": w.description,
            "background_tets": ne_o, "background_verts": np_o, "new_points": np_n,
            "located_points_per_step": npts, "K_doubles_per_vertex": w.K,
            "parallelism": (f"{args.split} parts x{world}, replicated background, RCCL all-gather after the step"
                            if shard_mode == "morton" else
                            f"{args.split} parts x{world}, halo-sharded background, RCCL all-gather after the step"
                            if shard_mode == "halo" else
                            "the whole group on one GPU (N > 1 splits it: RCB parts x halo shards, strong scaling)"
                            if world == 1 else f"one group per GPU x{world} (weak, no data-path collective)"),
            "query_order": args.sort,
            "tetra_layout": args.layout,
            "morton_binned": bool(st.sorted),
        },
        "gbps_algorithmic_step": round(B / (ms_per_step * 1e-3) / 1e9, 1),
        "device_ms": {"step_total": round(float(np.mean(ms_tot)), 4), "volume_stage": round(float(np.mean(ms_vol)), 4),
                      "volume_stage_last_timed_step": round(kvol_ms, 4),
                      "walk": round(float(np.mean(ms_walk)), 4),
                      "prepare": round(st.ms_prepare, 4), "order": round(st.ms_sort, 4),
                      "k_bdy_stream": round(st.ms_bdy, 4), "fallback": round(st.ms_fallback, 4)},
        "locate_stats": {k: v for k, v in st.as_dict().items() if not k.startswith("ms_")},
        "walk_steps_per_point": round(steps_pp, 3),
        "lockstep_efficiency": round(st.steps_total / max(1, 64 * st.wave_iters), 3),
        "roofline": {
            "bound": "hbm",
            "kernel": "volume stage: k_vol (fused fp32 filter walk, exact fp64 acceptance, interpolation) + "
                      "k_vol_walk_exact",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_unit": "HBM/Infinity-Cache bytes per volume stage (its launches in one call): 2 x FETCH_SIZE "
                            "(= 128 B per TCC_EA0_RDREQ, calibrated by tools/calib/fetch_calib, profiles/r02a/calib) "
                            "+ WRITE_SIZE",
            "traffic_source": traffic_src,
            "algorithmic_bytes_per_stage": round(kvol_bytes),
            "stage": "HIP events on the main stream from the end of the query order to the end of the "
                     "interpolation (the surface kernel runs concurrently on a second stream), of the last timed step",
            "algorithmic_bytes_per_point": round(per_pt, 2),
        },
    }
    if gather is not None:
        out["allgather"] = gather
    if halo_info is not None:
        out["halo_shard"] = halo_info
    if not args.no_host_mode and world == 1:
        try:
            out["host_mode"] = host_mode_timing(ctx, w, bg, met, fields, q_xyz, q_pc, rank)
        except Exception as e:  # reported, never fatal to the bench line
            out["host_mode"] = {"error": str(e)}
    if world == 1 and not split and not args.no_surface_solo:
        try:
            out["surface_solo"] = surface_solo(ctx, step_bg, d_qxyz, q_pc, d_mo, d_fo, d_elem, d_hit, local)
        except Exception as e:  # reported, never fatal to the bench line
            out["surface_solo"] = {"error": str(e)}
    if not args.no_shuffled and world == 1 and not split:
        legs = {"mmg_like_order": (synth.mmg_like_perm(nq), "the step on an Mmg-like numbering of the new points (1 in 6 "
                                   "points moved to the end as 'inserted', both parts in the generator's order); not "
                                   "the bench value"),
                "shuffled_order": (np.random.default_rng(2024).permutation(nq), "the step on a random renumbering of "
                                   "the new points (Morton-binned by the module); not the bench value")}
        for name, (perm, what) in legs.items():
            try:
                out[name] = renumbered_timing(ctx, args, w, step_bg, q_xyz, q_pc, d_mo, d_fo, d_elem, d_hit, rank,
                                              perm, what)
            except Exception as e:  # reported, never fatal to the bench line
                out[name] = {"error": str(e)}
        # the shuffled numbering again with the solutions as packed records in and out (the layout a
        # device-resident pipeline keeps across iterations, pmmg_hip_locate_interp_rec)
        try:
            d_rec = ctx.upload(pack_solutions(met, fields))
            out["shuffled_order_records"] = renumbered_timing(
                ctx, args, w, step_bg, q_xyz, q_pc, d_mo, d_fo, d_elem, d_hit, rank, legs["shuffled_order"][0],
                "the shuffled numbering's step with packed solution records in (pmmg_hip_set_solutions_packed) "
                "and out (pmmg_hip_locate_interp_rec): one record line per point written; rows checked "
                "against the input-order step's arrays; not the bench value", records=d_rec)
            d_rec.free()
        except Exception as e:  # reported, never fatal to the bench line (e.g. a layout without packed records)
            out["shuffled_order_records"] = {"error": str(e)}
    gpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not split:
        # outputs of the last timed step (the host-mode call used its own buffers)
        gpu = {"elem": d_elem.download(), "hit": d_hit.download(), "met": d_mo.download(),
               "fields": [f.download() for f in d_fo]}
    if not args.no_quality and not split:
        try:
            out["tetra_qual"] = quality_timing(ctx, w, d_qxyz, d_mo, rank)
        except Exception as e:  # reported, never fatal to the bench line
            out["tetra_qual"] = {"error": str(e)}
    if not args.no_snapshot and halo_info is None:  # (a shard's cut faces are no boundary trias)
        out["snapshot"] = snapshot_timing(ctx, bg, rank)
    ctx.close()
    # the groups leg after the large calls, in ParMmg's order (r05 ran it first: the lanes' streams then shared
    # hardware queues in some processes; r06: 3 lanes of 1 stream)
    if not args.no_groups and world == 1 and not split:
        try:
            out["groups"] = groups_leg(args)
        except Exception as e:  # reported, never fatal to the bench line
            out["groups"] = {"error": str(e)}
    if not args.no_graded and world == 1 and not split and args.config == "cfg4":
        try:
            out["graded"] = graded_leg(args, rank)
        except Exception as e:  # reported, never fatal to the bench line
            out["graded"] = {"error": str(e)}
    if gpu is not None:
        log(f"[bench r{rank}] cpu baseline (oracle) over all points")
        out["cpu_baseline"], B_o, ref = cpu_baseline(w, bg, met, fields, pclass, new, args.cpu_baseline_seconds)
        log(f"[bench r{rank}] parity of the GPU outputs against the oracle run")
        out["parity"] = parity_report(B_o, new, pclass, gpu, ref)
        log(f"[bench r{rank}] parity: {out['parity']}")
    if split and rank == 0 and not args.no_cpu_baseline:
        log(f"[bench r{rank}] parity of the all-gathered results against an oracle run over the group")
        try:
            out["parity"] = split_parity(w, bg_group, met_group, fields_group, new, pclass, shards, gathered,
                                         args.split_parity_seconds)
        except Exception as e:  # reported, never fatal to the bench line
            out["parity"] = {"error": str(e), "ok": False}
        log(f"[bench r{rank}] parity: {out['parity']}")
    if rank == 0:
        print(json.dumps(out), flush=True)
    ranks.barrier(ri)  # the other ranks wait for rank 0's check
    ranks.finalize(ri)


if __name__ == "__main__":
    main()
