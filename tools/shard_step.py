"""One rank's share of the N-GPU halo split, timed alone on one GPU: what
`bench.py --gpus N` (halo shards, the north_star's split of one cfg4 group)
gives each rank, without the other ranks contending for the card.  The
per-rank step time at N ranks bounds the driver's strong-scaling curve.

    python tools/shard_step.py --config cfg4 --world 8 --ranks 0,7 --steps 10
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# the measurement build of the module (its PMMG_HIP_* A/B switches; the same
# kernels as the product library otherwise)
os.environ.setdefault("PMMG_HIP_SO", os.path.join(ROOT, "parmmg_amd", "libpmmg_hip_measure.so"))

import bench  # noqa: E402
from parmmg_amd import configs, ranks, shard  # noqa: E402
from parmmg_amd.transfer import TransferContext, pack_tet8  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--ranks", default="0")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--bdy-weight", type=int, default=ranks.BDY_WEIGHT, help="cost of a surface point in the split")
    ap.add_argument("--split", default="rcb", choices=["rcb", "morton"], help="partition of the new points")
    ap.add_argument("--mode", default="cells", choices=["cells", "box"], help="halo shard: cell union or range box")
    ap.add_argument("--variants", default="", help='";"-separated PMMG_HIP_* settings NAME=v,... (sort=0/1: the '
                                                   'context option), each timed on every rank')
    a = ap.parse_args()
    w = configs.SHORT[a.config]
    bg0, new, met0, fields0, pclass = bench.build_workload(w, 0)
    split = ranks.rcb_shards if a.split == "rcb" else ranks.morton_shards
    shards = split(new.xyz, pclass, a.world, a.bdy_weight)
    for r in [int(x) for x in a.ranks.split(",")]:
        mine = shards[r]
        q_xyz, q_pc = np.ascontiguousarray(new.xyz[mine]), np.ascontiguousarray(pclass[mine])
        if a.mode == "cells":
            sh = shard.halo_shard_cells(bg0, q_xyz, -1.0, hausd=w.hausd)
        else:
            sh = shard.halo_shard(bg0, *shard.range_box(q_xyz), -1.0, hausd=w.hausd)
        bg, met, fields = sh.mesh, sh.rows(met0), [sh.rows(f) for f in fields0]
        for var in a.variants.split(";"):
            run_rank(a, w, r, var, bg, bg0, met, fields, q_xyz, q_pc)


def run_rank(a, w, r, var, bg, bg0, met, fields, q_xyz, q_pc):
    """one rank's share timed under one variant of the module settings"""
    sort = None
    for k in [k for k in os.environ if k.startswith("PMMG_HIP_") and k != "PMMG_HIP_SO"]:
        os.environ.pop(k)
    for item in filter(None, var.split(",")):
        k, v = item.split("=")
        if k.lower() == "sort":
            sort = v == "1"
        else:
            os.environ["PMMG_HIP_" + k.upper()] = v
    with TransferContext(0, sort=sort) as ctx:
        d = dict(xyz=ctx.upload(bg.xyz), tet8=ctx.upload(pack_tet8(bg.tetv, bg.adja)), triv=ctx.upload(bg.triv),
                 adjt=ctx.upload(bg.adjt), met=ctx.upload(met), f=[ctx.upload(f) for f in fields],
                 q=ctx.upload(q_xyz), pc=ctx.upload(q_pc))
        nq = q_xyz.shape[0]
        mo = ctx.empty((nq, w.met_size), np.float64)
        fo = [ctx.empty((nq, f.shape[1]), np.float64) for f in fields]
        el, hit = ctx.empty((nq,), np.int32), ctx.empty((nq,), np.int8)

        def step():
            ctx.set_background_tet8(d["xyz"], d["tet8"], d["triv"], d["adjt"], w.hausd)
            ctx.set_solutions(d["met"], d["f"])
            ctx.locate_interp(d["q"], d["pc"], mo, fo, el, hit, sync=False)

        for _ in range(a.warmup):
            step()
            ctx.sync()
        ms = {k: [] for k in ("ms_total", "ms_prepare", "ms_sort", "ms_vol", "ms_vol_locate", "ms_bdy",
                              "ms_fallback")}
        t0 = time.perf_counter()
        for _ in range(a.steps):  # back to back, as bench.py times them
            step()
        ctx.sync()
        wall = (time.perf_counter() - t0) / a.steps
        for _ in range(a.steps):  # per-step device times
            step()
            st = ctx.sync()
            for k in ms:
                ms[k].append(getattr(st, k))
        res = {"rank": r, "variant": var, "world": a.world, "mode": a.mode, "nvol_exhaust": int(st.nvol_exhaust),
               "nvol_closest": int(st.nvol_closest), "nbdy_exhaust": int(st.nbdy_exhaust),
               "nbdy_cone": int(st.nbdy_cone), "nbdy_wedge": int(st.nbdy_wedge), "nbdy_fanscan": int(st.nbdy_fanscan),
               "points": int(st.nvol + st.nbdy), "nbdy": int(st.nbdy), "sorted": int(st.sorted),
               "steps_pp": round(st.steps_total / max(1, st.nvol + st.nbdy), 3), "shard_tets": bg.ne,
               "shard_tet_fraction": round(bg.ne / bg0.ne, 4), "ms_per_step_wall": round(1e3 * wall, 4)}
        res.update({k: round(float(np.median(v)), 4) for k, v in ms.items()})
        print(res, flush=True)


if __name__ == "__main__":
    main()
