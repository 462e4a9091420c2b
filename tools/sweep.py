"""Interleaved A/B sweep of module options in ONE process (rule: perf deltas
from interleaved rounds, not separate invocations).

  python tools/sweep.py --config cfg3 --tpc 8,16,32,64 --rounds 3
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from parmmg_amd import configs, synth  # noqa: E402
from parmmg_amd.transfer import TransferContext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--tpc", default="8,16,32,64")
    ap.add_argument("--nosort", default="0")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="", help='e.g. "chain=0;chain=16;chain=16,sort=1"')
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    w = configs.SHORT[args.config]
    bg = synth.lattice(w.kind, w.n_old)
    new = synth.lattice(w.kind, w.n_new, jitter=w.jitter_new, with_trias=False)
    met = synth.solution(w.metric, bg.xyz)
    fields = [synth.solution(f, bg.xyz) for f in w.fields]
    pc = synth.classes(new)
    base = TransferContext(0)
    from parmmg_amd.transfer import pack_solutions, pack_tet8
    rec, *recmeta = pack_solutions(met, fields)
    d = dict(xyz=base.upload(bg.xyz), tetv=base.upload(bg.tetv), adja=base.upload(bg.adja),
             tet8=base.upload(pack_tet8(bg.tetv, bg.adja)), rec=base.upload(rec), recmeta=recmeta,
             triv=base.upload(bg.triv), adjt=base.upload(bg.adjt), met=base.upload(met),
             f=[base.upload(f) for f in fields], q=base.upload(new.xyz), pc=base.upload(pc),
             mo=base.empty((new.np, w.met_size), np.float64),
             fo=[base.empty((new.np, f.shape[1]), np.float64) for f in fields],
             el=base.empty((new.np,), np.int32), hit=base.empty((new.np,), np.int8))
    variants = []
    tet8s, packeds = set(), set()
    if args.variants:
        # "chain=16,sort=1;chain=0" -> TransferContext keyword sets (sort: 1 on, 0 off)
        for spec in args.variants.split(";"):
            kw = {}
            for name in ("TPC", "SPC", "QPB", "MAXSTEP", "CAP", "SEEDMODE", "SEEDRUN", "STREAMS", "S2START", "CARRY", "WALKW", "SEEDGRID", "SEEDATOM", "RUNORDER", "CHUNKS", "BBOXSTRIDE", "SEED8", "COOP", "WALKB", "S2PRIO", "BDYEARLY", "INTERPB"):
                os.environ.pop("PMMG_HIP_" + name, None)
            for item in filter(None, spec.split(",")):
                k, v = item.split("=")
                if k == "tet8":
                    tet8s.add(spec)
                elif k == "packed":
                    packeds.add(spec)
                elif k in ("tpc", "spc", "qpb", "maxstep", "cap", "seedmode", "seedrun", "streams", "s2start", "carry", "walkw", "seedgrid", "seedatom", "runorder", "chunks", "bboxstride", "seed8", "coop", "walkb", "s2prio", "bdyearly", "interpb"):
                    os.environ["PMMG_HIP_" + k.upper()] = v  # read by pmmg_hip_create
                else:
                    kw[k] = bool(int(v)) if k in ("sort", "fused", "scan") else int(v)
            variants.append(((spec, ""), TransferContext(0, **kw)))
    for tpc in ([] if args.variants else [int(t) for t in args.tpc.split(",")]):
        for ns in [int(x) for x in args.nosort.split(",")]:
            os.environ["PMMG_HIP_TPC"] = str(tpc)
            # ns: 0 morton, 1 input order, 2 auto, 3 tetra-centric scan, 4 fused auto, 5 fused input order
            kw = [dict(sort=True), dict(sort=False), dict(), dict(scan=True), dict(fused=True),
                  dict(fused=True, sort=False)][ns]
            variants.append(((tpc, ns), TransferContext(0, **kw)))
    res = {k: [] for k, _ in variants}
    for r in range(args.rounds):
        for key, ctx in variants:
            for s in range(args.steps + 1):
                if key[0] in tet8s:
                    ctx.set_background_tet8(d["xyz"], d["tet8"], d["triv"], d["adjt"], w.hausd)
                else:
                    ctx.set_background(d["xyz"], d["tetv"], d["adja"], d["triv"], d["adjt"], w.hausd)
                if key[0] in packeds:
                    ctx.set_solutions_packed(d["rec"], *d["recmeta"])
                else:
                    ctx.set_solutions(d["met"], d["f"])
                ctx.locate_interp(d["q"], d["pc"], d["mo"], d["fo"], d["el"], d["hit"], sync=False)
                st = ctx.sync()
                if s > 0:
                    res[key].append(st.as_dict())
    print(f"{'tpc':>5} {'nosort':>6} {'total':>8} {'prep':>7} {'sort':>7} {'locate':>7} {'interp':>7} {'bdy':>7} {'fb':>7} {'steps/pt':>8}")
    for key, _ in variants:
        a = res[key]
        m = lambda k: float(np.median([x[k] for x in a]))  # noqa: E731
        spp = a[-1]["steps_total"] / max(1, a[-1]["nvol"] + a[-1]["nbdy"])
        print(f"{str(key[0]):>5} {str(key[1]):>6} {m('ms_total'):8.3f} {m('ms_prepare'):7.3f} {m('ms_sort'):7.3f} "
              f"{m('ms_vol_locate'):7.3f} {m('ms_vol') - m('ms_vol_locate'):7.3f} {m('ms_bdy'):7.3f} "
              f"{m('ms_fallback'):7.3f} {spp:8.2f}")


if __name__ == "__main__":
    main()
