"""Interleaved A/B sweep of module settings: rounds x variants, each variant
run in its own process (one live context, so every variant gets the same
hardware queues: a second live context's streams can share one queue, which
serialises its surface branch with its volume kernel and biases the A/B).  Each variant is a set of
PMMG_HIP_* environment values read by pmmg_hip_create (and sort=0/1, the
context's query-order option):

  python tools/sweep.py --config cfg4 --variants "TPC=8;TPC=4;TPC=16" --rounds 3
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# the measurement build of the module (its PMMG_HIP_* A/B switches; the same
# kernels as the product library otherwise)
os.environ.setdefault("PMMG_HIP_SO", os.path.join(ROOT, "parmmg_amd", "libpmmg_hip_measure.so"))

from parmmg_amd import configs, synth  # noqa: E402
from parmmg_amd.transfer import TransferContext, pack_tet8  # noqa: E402


def query_perm(xyz: np.ndarray, n: int, spec: str) -> np.ndarray:
    """Test-only renumbering of the new points (the module keeps input order
    when it is coherent, so this changes the order waves are dispatched in):
    zslabZ  lattice points by (z // Z, y, z % Z, x)   (cube lattices)
    rodsB   runs of 64 consecutive points sorted by the B-bit-per-axis Morton
            code of each run's first point"""
    lo, hi = xyz.min(0), xyz.max(0)
    if spec.startswith("zslab"):
        Z = int(spec[5:])
        q = np.rint((xyz - lo) / (hi - lo) * n).astype(np.int64)
        key = (((q[:, 2] // Z) * (n + 1) + q[:, 1]) * Z + q[:, 2] % Z) * (n + 1) + q[:, 0]
        return np.argsort(key, kind="stable")
    if spec.startswith("rods"):
        B = int(spec[4:])
        first = xyz[::64]
        q = np.minimum(((first - lo) / (hi - lo) * (1 << B)).astype(np.int64), (1 << B) - 1)
        key = np.zeros(q.shape[0], np.int64)
        for b in range(B):
            for d in range(3):
                key |= ((q[:, d] >> b) & 1) << (3 * b + d)
        rods = np.argsort(key, kind="stable")
        idx = (rods[:, None] * 64 + np.arange(64)[None, :]).ravel()
        return idx[idx < xyz.shape[0]]
    if spec == "mmg":  # Mmg-like: one point in six appended at the end (bench.py's mmg_like_order leg)
        return synth.mmg_like_perm(xyz.shape[0])
    if spec == "shuffle":  # a numbering with no spatial coherence (the module then Morton-bins)
        return np.random.default_rng(12345).permutation(xyz.shape[0])
    raise ValueError(spec)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4")
    ap.add_argument("--variants", default="TPC=8", help='";"-separated variants of ","-separated NAME=value')
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--child", default=None, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.child is None:
        return parent(args)
    w = configs.SHORT[args.config]
    bg, new = configs.build_meshes(w)
    met = synth.solution(w.metric, bg.xyz)
    fields = [synth.solution(f, bg.xyz) for f in w.fields]
    pc = synth.classes(new)
    variants = [args.child]

    def make_ctx(spec):
        """one context alive at a time: every variant gets the same hardware
        queues (a second live context's streams can share one queue, which
        serialises its surface branch with its volume kernel)"""
        for k in list(os.environ):
            if k.startswith("PMMG_HIP_") and k != "PMMG_HIP_SO":
                os.environ.pop(k)
        sort = None
        for item in filter(None, spec.split(",")):
            k, v = item.split("=")
            if k.lower() == "sort":  # context option: 1 Morton bins, 0 input order
                sort = v == "1"
            elif k.lower() in ("sol", "perm", "packed", "so", "recout"):  # measurement only: slots / renumbering / packed
                # records / build / output records (pmmg_hip_locate_interp_rec, with packed=1)
                pass
            else:
                os.environ["PMMG_HIP_" + k.upper()] = v
        ctx = TransferContext(0, sort=sort)
        for k in list(os.environ):
            if k.startswith("PMMG_HIP_") and k != "PMMG_HIP_SO":
                os.environ.pop(k)
        return ctx

    base = make_ctx(args.child)  # the only live context: it owns the inputs and runs the variant
    d = dict(xyz=base.upload(bg.xyz), tet8=base.upload(pack_tet8(bg.tetv, bg.adja)), triv=base.upload(bg.triv),
             adjt=base.upload(bg.adjt), met=base.upload(met), f=[base.upload(f) for f in fields],
             q=base.upload(new.xyz), pc=base.upload(pc), mo=base.empty((new.np, w.met_size), np.float64),
             fo=[base.empty((new.np, f.shape[1]), np.float64) for f in fields],
             el=base.empty((new.np,), np.int32), hit=base.empty((new.np,), np.int8))
    cols = ["ms_total", "ms_prepare", "ms_sort", "ms_vol_locate", "ms_vol", "ms_bdy", "ms_fallback"]
    res = {v: {c: [] for c in cols + ["steps_pp", "iters", "exact"]} for v in variants}
    from parmmg_amd.transfer import pack_solutions
    d["rec"] = base.upload(pack_solutions(met, fields))
    qperm = {}
    for spec in variants:
        pspec = dict(item.split("=") for item in spec.split(",") if item).get("perm")
        if pspec:
            perm = query_perm(new.xyz, w.n_new, pspec)
            qperm[spec] = (base.upload(np.ascontiguousarray(new.xyz[perm])), base.upload(np.ascontiguousarray(pc[perm])))

    def sols(spec):
        which = dict(item.split("=") for item in spec.split(",") if item).get("sol", "all")
        return {"none": (None, []), "met": (d["met"], []), "all": (d["met"], d["f"])}[which]

    for r in range(1):
        for spec in variants:
            ctx = base
            for s in range(args.steps + 1):
                ctx.set_background_tet8(d["xyz"], d["tet8"], d["triv"], d["adjt"], w.hausd)
                if dict(item.split("=") for item in spec.split(",") if item).get("packed") == "1":
                    ctx.set_solutions_packed(d["rec"], w.met_size, [f.shape[1] for f in fields])
                else:
                    ctx.set_solutions(*sols(spec))
                q, qpc = qperm.get(spec, (d["q"], d["pc"]))
                if dict(item.split("=") for item in spec.split(",") if item).get("recout") == "1":
                    if "ro" not in d:
                        d["ro"] = base.empty((new.np, d["rec"].shape[1]), np.float64)
                    ctx.locate_interp_rec(q, qpc, d["ro"], d["el"], d["hit"], sync=False)
                else:
                    ctx.locate_interp(q, qpc, d["mo"], d["fo"], d["el"], d["hit"], sync=False)
                st = ctx.sync()
                if s == 0:
                    continue  # first call of a round: warm-up
                for c in cols:
                    res[spec][c].append(getattr(st, c))
                res[spec]["steps_pp"].append(st.steps_total / max(1, st.nvol + st.nbdy))
                res[spec]["iters"].append(st.wave_iters)
                res[spec]["exact"].append(st.nvol_exact)
    import json

    print("RESULT " + json.dumps(res[args.child]), flush=True)


def parent(args):
    import json
    import subprocess

    variants = [v for v in args.variants.split(";") if v]
    cols = ["ms_total", "ms_prepare", "ms_sort", "ms_vol_locate", "ms_vol", "ms_bdy", "ms_fallback"]
    res = {v: {} for v in variants}
    for r in range(args.rounds):
        for spec in variants:
            env = dict(os.environ)
            so = dict(item.split("=") for item in spec.split(",") if item).get("so")
            if so:  # another build of the module for this variant (e.g. the previous commit's, for an A/B)
                env["PMMG_HIP_SO"] = os.path.join(ROOT, so)
            p = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--config", args.config, "--steps",
                                str(args.steps), "--child", spec], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env)
            line = [x for x in p.stdout.splitlines() if x.startswith("RESULT ")]
            if p.returncode != 0 or not line:
                print(p.stdout[-2000:])
                raise SystemExit(f"variant {spec} failed")
            for k, v in json.loads(line[-1][7:]).items():
                res[spec].setdefault(k, []).extend(v)
        print(f"round {r} done", flush=True)
    hdr = f"{'variant':28s}" + "".join(f"{c[3:]:>11s}" for c in cols) + f"{'steps/pt':>10s}{'wave_it':>10s}{'exact':>8s}"
    print(hdr)
    for spec in variants:
        row = f"{spec:28s}" + "".join(f"{np.median(res[spec][c]):11.3f}" for c in cols)
        row += f"{np.median(res[spec]['steps_pp']):10.3f}{np.median(res[spec]['iters']):10.0f}"
        row += f"{np.median(res[spec]['exact']):8.0f}"
        print(row, flush=True)
    print("ms_total per call, min / max over all rounds (one process per variant and round):")
    for spec in variants:
        print(f"{spec:28s}{np.min(res[spec]['ms_total']):11.3f}{np.max(res[spec]['ms_total']):11.3f}", flush=True)


if __name__ == "__main__":
    main()
