"""Benchmark of the old->new mesh transfer step (PMMG_interpMetricsAndFields).

One step = one full pmmg_hip_locate_interp over one group: bbox + seed
grids + Morton sort + volume/surface locate + metric/field interpolation +
fallbacks, with every input already resident in HBM (device-mode C-ABI).

Multi-GPU (torchrun, one process per GPU): every rank owns one group of the
same size, exactly as ParMmg shards the step by group (the per-group work is
independent, src/interpmesh_pmmg.c:690-730), so there is no collective in the
data path and the scaling is weak.  `value` = points located+interpolated by
all ranks / max-over-ranks step time.

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
from parmmg_amd.transfer import TransferContext  # noqa: E402

METRIC = "new-mesh points located+interpolated/sec (Mpts/s) and HBM GB/s, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_workload(w: configs.Workload, rank: int):
    t0 = time.time()
    bg = synth.lattice(w.kind, w.n_old, jitter=0.0)
    new = synth.lattice(w.kind, w.n_new, jitter=w.jitter_new, seed=synth.SEED + rank, with_trias=False,
                        with_tetra=False)
    met = synth.solution(w.metric, bg.xyz)
    fields = [synth.solution(f, bg.xyz) for f in w.fields]
    pclass = synth.classes(new)
    log(f"[bench r{rank}] workload {w.name}: bg {bg.ne} tets / {bg.np} verts / {bg.nt} trias, new {new.np} verts, "
        f"K={w.K}, generated in {time.time() - t0:.1f}s")
    return bg, new, met, fields, pclass


def pmc_traffic(workload: str):
    """HBM bytes per launch of the dominant volume kernel from the newest
    committed rocprofv3 PMC summary (profiles/rNN/pmc_<workload>.json, made by
    tools/prof_summary.py from FETCH_SIZE / WRITE_SIZE passes of this bench),
    or (None, None)."""
    import glob

    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"pmc_{workload}.json")))
    if not paths:
        return None, None
    try:
        with open(paths[-1]) as f:
            d = json.load(f)
        return d.get("k_vol_hbm_bytes_per_call", d.get("k_vol_hbm_bytes_per_launch")), os.path.relpath(paths[-1], ROOT)
    except Exception:
        return None, None


def cpu_baseline(w, bg, new, met, fields, pclass, budget_s: float):
    """The oracle (C restatement of the reference path) as `threads` parallel
    workers on this host's cores, each a sequential reference run (warm start,
    private visited flags) over a contiguous range of the new points, like one
    MPI rank per group: the per-iteration precompute (faceAreas, triaNormals,
    nodeTrias, which the reference's tim=2 timer includes,
    src/libparmmg1.c:823-836) split over the threads, then locate+interpolate
    until `budget_s` seconds are used; the full-step time is the precompute
    plus the measured rate extrapolated to all points."""
    from oracle import oracle as O

    threads = int(os.environ.get("PMMG_CPU_THREADS", "0")) or min(16, os.cpu_count() or 1)
    B = O.Background(bg, met, fields, w.hausd)
    order = np.arange(1, new.np + 1, dtype=np.int32)
    r = O.run(B, new.xyz, pclass, order, budget_s=budget_s, threads=threads)
    t_pre, t_loc = r["t_precompute"], r["t_locate"]
    nproc = int((r["hit"] != 0).sum())
    ntot = int((pclass != 0).sum())
    t_full = t_pre + t_loc * ntot / max(nproc, 1)
    return {
        "value": round(ntot / t_full / 1e6, 4),
        "unit": "Mpts/s",
        "cores": threads,
        "kind": "port",
        "sample": f"oracle (C restatement of the reference path) as {threads} threads, one contiguous range of "
                  f"new points each (like MPI ranks), on {w.name}: precompute over {bg.ne} tets ({t_pre:.2f}s) + "
                  f"locate/interp of {nproc} of {ntot} points ({t_loc:.2f}s, time-bounded), rate extrapolated "
                  f"to all points",
        "t_precompute_s": round(t_pre, 3),
        "t_sample_s": round(t_loc, 3),
        "sample_points": nproc,
    }


def allgather_timing(ri, d_mo, d_fo, d_elem, counts, mine, rank: int, reps: int = 3):
    """Morton mode: collect every rank's located elements and interpolated
    rows on every rank (ranks.allgather_rows: RCCL all_gather_into_tensor over
    xGMI), timed on its own after the timed steps (reported
    separately; ParMmg itself consumes the results per rank).  Checks that the
    gathered element ids cover every processed point."""
    import torch

    rows = torch.cat([d_mo] + list(d_fo), dim=1)
    elem = d_elem.view(-1, 1)
    times = []
    for _ in range(reps):
        ranks.barrier(ri)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g_rows = ranks.allgather_rows(ri, rows, counts)
        g_elem = ranks.allgather_rows(ri, elem, counts)
        torch.cuda.synchronize()
        times.append(ranks.max_over_ranks(ri, time.perf_counter() - t0))
    ok = bool((g_elem > 0).all().item()) and g_rows.shape[0] == sum(counts)
    nbytes = sum(counts) * (rows.shape[1] * 8 + 4)
    t = float(np.median(times))
    log(f"[bench r{rank}] all-gather of {nbytes / 1e9:.2f} GB: {1e3 * t:.2f} ms, complete={ok}")
    return {"what": "RCCL all-gather of {elem, K doubles} per point, not part of the step",
            "ms": round(1e3 * t, 3), "bytes": int(nbytes), "gbps": round(nbytes / t / 1e9, 1), "complete": ok}


def snapshot_timing(ctx, bg, rank: int, reps: int = 3):
    """Device background snapshot (PMMG_create_oldGrp's
    adjacency / boundary trias / tria adjacency, pmmg_hip_build_*) timed on
    its own, outside the transfer step: wall time of the synchronous calls
    (scratch allocation included), median of `reps`, checked against the
    host-built arrays the step uses."""
    d_tetv = ctx.upload(bg.tetv)
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        adja, tet8 = ctx.build_adjacency(bg.np, d_tetv, adja=False, tet8=True)
        t1 = time.perf_counter()
        triv, adjt = ctx.build_boundary(bg.np, tet8=tet8)
        t2 = time.perf_counter()
        times.append((t1 - t0, t2 - t1))
        ok = bool(np.array_equal(adjt.download(), bg.adjt))
        if _ == reps - 1:
            from parmmg_amd.transfer import pack_tet8
            ok = ok and bool(np.array_equal(tet8.download(), pack_tet8(bg.tetv, bg.adja)))
            ok = ok and bool(np.array_equal(triv.download(), bg.triv))
        for a in (tet8, triv, adjt):
            a.free()
    d_tetv.free()
    t_adj = float(np.median([t[0] for t in times]))
    t_bdy = float(np.median([t[1] for t in times]))
    # compulsory bytes: tetv in (16 B/tet), tet8 records out (32 B/tet)
    b_adj = bg.ne * (16 + 32)
    log(f"[bench r{rank}] snapshot: adjacency {1e3 * t_adj:.2f} ms, boundary {1e3 * t_bdy:.2f} ms, match={ok}")
    return {"what": "pmmg_hip_build_adjacency (tet8 out) + pmmg_hip_build_boundary, not part of the step",
            "ms_adjacency": round(1e3 * t_adj, 3), "ms_boundary": round(1e3 * t_bdy, 3),
            "tets": bg.ne, "trias": bg.nt, "matches_host_builder": ok,
            "adjacency_algorithmic_gbps": round(b_adj / t_adj / 1e9, 1)}


def quality_timing(ctx, w, d_qxyz, d_mo, rank: int, reps: int = 3):
    """PMMG_tetraQual on the new mesh in the device-resident interpolated
    metric (pmmg_hip_tetra_qual), timed on its own
    after the step: wall time of the synchronous call, median of `reps`.
    Compulsory bytes: 16 B tetv + 8 B qual per tetra, 24 + 8*met_size B per
    vertex row."""
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


def host_mode_timing(ctx, w, bg, met, fields, q_xyz, q_pc, rank: int, reps: int = 2):
    """End-to-end rate with host buffers (PMMG_HIP_HOST: the background,
    solutions and queries copied H2D and the outputs D2H inside the call, as a
    shim that hands over MMG5 arrays without keeping them resident would),
    reported beside the HBM-resident step, never as the bench value."""
    from parmmg_amd.transfer import pack_tet8
    tet8 = pack_tet8(bg.tetv, bg.adja)
    nq = q_xyz.shape[0]
    mo = np.empty((nq, w.met_size), np.float64)
    fo = [np.empty((nq, f.shape[1]), np.float64) for f in fields]
    elem, hit = np.empty(nq, np.int32), np.empty(nq, np.int8)
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ctx.set_background_tet8(bg.xyz, tet8, bg.triv, bg.adjt, w.hausd)
        ctx.set_solutions(met, fields)
        st = ctx.locate_interp(q_xyz, q_pc, mo, fo, elem, hit)
        times.append(time.perf_counter() - t0)
    t = float(np.median(times))
    nbytes = (bg.xyz.nbytes + tet8.nbytes + bg.triv.nbytes + bg.adjt.nbytes + met.nbytes + sum(f.nbytes for f in fields)
              + q_xyz.nbytes + q_pc.nbytes + mo.nbytes + sum(f.nbytes for f in fo) + elem.nbytes + hit.nbytes)
    npts = int(st.nvol + st.nbdy)
    log(f"[bench r{rank}] host-buffer (PCIe-inclusive) call: {1e3 * t:.1f} ms, {nbytes / 1e9:.2f} GB moved")
    return {"what": "one pmmg_hip_locate_interp with host (pageable) buffers: H2D of background, solutions and "
                    "queries + the step + D2H of the outputs; not the bench value",
            "ms": round(1e3 * t, 2), "mpts_per_s": round(npts / t / 1e6, 1), "bytes_moved": int(nbytes),
            "pcie_gbps_effective": round(nbytes / t / 1e9, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg4", choices=sorted(configs.SHORT))
    ap.add_argument("--sort", default="auto", choices=["auto", "on", "off"],
                    help="query order: Morton binning (on), input order (off), or automatic")
    ap.add_argument("--locate", default="walk", choices=["walk", "scan"],
                    help="volume location: grid-seeded adjacency walks or the tetra-centric scan")
    ap.add_argument("--fused", action="store_true", help="volume walk and interpolation as one kernel")
    ap.add_argument("--tpc", type=int, default=0, help="background tetra per volume seed cell (0: module default)")
    ap.add_argument("--spc", type=int, default=0, help="sampled tetra per seed cell (0: module default)")
    ap.add_argument("--layout", default="tet8", choices=["tet8", "separate"],
                    help="HBM layout of the tetra: packed {v[4], adja[4]} records or separate tetv/adja arrays")
    ap.add_argument("--solutions", default="separate", choices=["packed", "separate"],
                    help="HBM layout of the metric/fields: packed per-vertex records or one array per solution")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--shard", default="group", choices=["group", "morton", "halo"],
                    help="multi-GPU split: one group per rank (weak scaling, ParMmg's own sharding); one problem "
                         "cut into contiguous Morton ranges of the new points, background replicated, results "
                         "all-gathered over RCCL after the timed steps (morton); or Morton ranges against halo "
                         "shards of the background, results kept per rank (halo; strong scaling, SURVEY.md 8(e))")
    ap.add_argument("--halo", type=float, default=-1.0,
                    help="halo mode: growth of the range box (< 0: in largest-tetra extents)")
    ap.add_argument("--no-host-mode", action="store_true",
                    help="skip the (separately reported) host-buffer, PCIe-inclusive call")
    ap.add_argument("--no-quality", action="store_true",
                    help="skip the (separately reported) tetra-quality timing of the new mesh")
    ap.add_argument("--no-snapshot", action="store_true",
                    help="skip the (separately reported) device background snapshot timing")
    args = ap.parse_args()

    # PMMG_BENCH_BACKEND=gloo: host-side collectives, ranks share the visible
    # GPUs round-robin (rehearsing several ranks on a one-GPU box)
    backend = os.environ.get("PMMG_BENCH_BACKEND", "nccl")
    ri = ranks.init(backend)
    rank, world, local = ri.rank, ri.world, ri.local
    if backend != "nccl":
        import torch
        local = local % max(1, torch.cuda.device_count())

    w = configs.SHORT[args.config]
    split = args.shard in ("morton", "halo")
    morton = args.shard == "morton"
    # Morton / halo mode: every rank builds the same problem and keeps its range
    bg, new, met, fields, pclass = build_workload(w, 0 if split else rank)
    ne_group = bg.ne
    mine = None
    halo_info = None
    if split:
        shards = ranks.morton_shards(new.xyz, pclass, world)
        mine = shards[rank]
        counts = [len(x) for x in shards]
        q_xyz, q_pc = np.ascontiguousarray(new.xyz[mine]), np.ascontiguousarray(pclass[mine])
        log(f"[bench r{rank}] Morton range {len(mine)} of {int((pclass != 0).sum())} points")
        if args.shard == "halo":
            from parmmg_amd import shard
            t_sh = time.time()
            lo, hi = shard.range_box(q_xyz)
            sh = shard.halo_shard(bg, lo, hi, args.halo)
            bg, met, fields = sh.mesh, sh.rows(met), [sh.rows(f) for f in fields]
            halo_info = {"what": "halo shard of the background around this rank's Morton range (rank 0)",
                         "tets": bg.ne, "verts": bg.np, "trias": bg.nt, "halo": sh.halo,
                         "tet_fraction_of_group": round(bg.ne / ne_group, 4),
                         "build_s": round(time.time() - t_sh, 2)}
            log(f"[bench r{rank}] halo shard: {bg.ne} of {ne_group} tets, {bg.np} verts, {bg.nt} trias "
                f"(halo {sh.halo:.4g}) in {time.time() - t_sh:.1f}s")
    else:
        q_xyz, q_pc = new.xyz, pclass
    nq = q_xyz.shape[0]

    for name in ("tpc", "spc"):
        if getattr(args, name) > 0:
            os.environ["PMMG_HIP_" + name.upper()] = str(getattr(args, name))  # read by pmmg_hip_create
    ctx = TransferContext(local, fused=args.fused, sort={"auto": None, "on": True, "off": False}[args.sort],
                          scan=args.locate == "scan")
    from parmmg_amd.transfer import pack_tet8
    d_xyz = ctx.upload(bg.xyz)
    if args.layout == "tet8":
        d_tet8 = ctx.upload(pack_tet8(bg.tetv, bg.adja))
    else:
        d_tetv, d_adja = ctx.upload(bg.tetv), ctx.upload(bg.adja)
    d_triv, d_adjt = ctx.upload(bg.triv), ctx.upload(bg.adjt)
    from parmmg_amd.transfer import pack_solutions
    if args.solutions == "packed":
        rec, *recmeta = pack_solutions(met, fields)
        d_rec = ctx.upload(rec)
    else:
        d_met = ctx.upload(met)
        d_f = [ctx.upload(f) for f in fields]
    d_qxyz, d_pc = ctx.upload(q_xyz), ctx.upload(q_pc)
    if morton:
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

    def step():
        if args.layout == "tet8":
            ctx.set_background_tet8(d_xyz, d_tet8, d_triv, d_adjt, w.hausd)
        else:
            ctx.set_background(d_xyz, d_tetv, d_adja, d_triv, d_adjt, w.hausd)
        if args.solutions == "packed":
            ctx.set_solutions_packed(d_rec, *recmeta)
        else:
            ctx.set_solutions(d_met, d_f)
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
    ms_vol = []
    ms_tot = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        st = ctx.sync()  # per-step event times of this step (sync adds no device work)
        ms_vol.append(st.ms_vol)
        ms_tot.append(st.ms_total)
    ranks.barrier(ri)
    ctx.sync()
    elapsed = time.perf_counter() - t0
    log(f"[bench r{rank}] timed {args.steps} steps: {1e3 * elapsed / args.steps:.3f} ms/step")

    npts = int(st.nvol + st.nbdy)
    agg = ranks.aggregate(ri, npts, elapsed, args.steps)
    gather = None
    if morton:
        gather = allgather_timing(ri, d_mo, d_fo, d_elem, counts, mine, rank)
    if split:
        npts = agg["points_per_step"]  # the whole problem: bytes per point below are per problem point
    ms_per_step = agg["ms_per_step"]
    value = agg["mpts_per_s"]
    (np_o, ne_o, _), (np_n, _, _) = w.counts()
    B = w.algorithmic_bytes(npts)
    per_pt = B / npts
    kvol_ms = float(np.mean(ms_vol))
    kvol_bytes = per_pt * st.nvol
    achieved = kvol_bytes / (kvol_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(w.name)
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Mpts/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong" if split else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (Kuhn lattices, analytic metric/fields, splitmix64 jitter)",
        "config": {
            "workload": w.name,
            "description": w.description,
            "background_tets": ne_o, "background_verts": np_o, "new_points": np_n,
            "located_points_per_gpu": npts, "K_doubles_per_vertex": w.K,
            "parallelism": (f"Morton-range shards x{world}, replicated background, RCCL all-gather after the step"
                            if morton else
                            f"Morton-range shards x{world}, halo-sharded background, results kept per rank"
                            if split else f"one group per GPU x{world} (weak, no data-path collective)"),
            "query_order": args.sort,
            "locate": args.locate,
            "tetra_layout": args.layout,
            "solution_layout": args.solutions,
            "volume_kernels": "fused" if args.fused else "walk+interp",
            "morton_binned": bool(st.sorted),
        },
        "gbps_algorithmic_step": round(B / (ms_per_step * 1e-3) / 1e9, 1),
        "device_ms": {"step_total": round(float(np.mean(ms_tot)), 4), "k_vol": round(kvol_ms, 4),
                      "k_vol_locate": round(st.ms_vol_locate, 4),
                      "prepare": round(st.ms_prepare, 4), "sort": round(st.ms_sort, 4),
                      "k_bdy": round(st.ms_bdy, 4), "fallback": round(st.ms_fallback, 4)},
        "locate_stats": {k: v for k, v in st.as_dict().items() if not k.startswith("ms_")},
        "roofline": {
            "bound": "hbm",
            "kernel": "k_vol_fused" if args.fused else "k_vol_walk + k_vol_interp (volume stage)",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_unit": "bytes per volume stage = all walk + interpolation launches of one call "
                            "(FETCH_SIZE x2 + WRITE_SIZE)",
            "traffic_source": traffic_src,
            "algorithmic_bytes_per_stage": round(kvol_bytes),
            "stage": "volume stage of one transfer call: the walk and interpolation launches of its query chunks "
                     "(chunks overlap on two streams when PMMG_HIP_CHUNKS > 1), timed by HIP events from the first walk to the last "
                     "interpolation",
            "algorithmic_bytes_per_point": round(per_pt, 2),
        },
    }
    if gather is not None:
        out["allgather"] = gather
    if halo_info is not None:
        out["halo_shard"] = halo_info
    if not args.no_host_mode and world == 1 and args.solutions == "separate":
        try:
            out["host_mode"] = host_mode_timing(ctx, w, bg, met, fields, q_xyz, q_pc, rank)
        except Exception as e:  # reported, never fatal to the bench line
            out["host_mode"] = {"error": str(e)}
    if not args.no_quality and not split:
        try:
            out["tetra_qual"] = quality_timing(ctx, w, d_qxyz, d_mo, rank)
        except Exception as e:  # reported, never fatal to the bench line
            out["tetra_qual"] = {"error": str(e)}
    if not args.no_snapshot and halo_info is None:  # (a shard's cut faces are no boundary trias)
        out["snapshot"] = snapshot_timing(ctx, bg, rank)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and halo_info is None:
        log(f"[bench r{rank}] cpu baseline (oracle) on a bounded sample")
        out["cpu_baseline"] = cpu_baseline(w, bg, new, met, fields, pclass, args.cpu_baseline_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    ranks.finalize(ri)


if __name__ == "__main__":
    main()
