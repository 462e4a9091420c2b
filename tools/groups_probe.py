"""Bisect the groups call's slowdown after a large call in the same process
(0.102 vs 0.082 ms per cfg2-size group).
Each variant runs in its own process: a prologue, then bench.groups_leg.

  python tools/groups_probe.py --rounds 2 --variants "base;streams2;alloc8;big_auto;big_noauto;host"

prologues:
  base          nothing
  streamsN      N HIP streams created and destroyed (hipStreamCreate, ctypes)
  keepstreamsN  N HIP streams created and kept alive
  nullcopy      one synchronous hipMemcpy (null stream)
  allocG        G GiB hipMalloc'ed in 256 MiB pieces, then freed
  big_auto      one cfg3 call in device mode, auto order (the binning's third stream is created), context closed
  big_noauto    the same with the input order forced (no third stream)
  host          one cfg3 call through host buffers (the copy stream is created), context closed
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import subprocess
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def hip():
    h = ctypes.CDLL("libamdhip64.so")
    h.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    h.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    h.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    h.hipFree.argtypes = [ctypes.c_void_p]
    return h


def prologue(spec: str):
    import bench
    from parmmg_amd import configs
    from parmmg_amd.transfer import TransferContext

    if spec == "base":
        return None
    if spec.startswith("streams") or spec.startswith("keepstreams"):
        n = int(spec.split("streams")[1])
        h = hip()
        ss = []
        for _ in range(n):
            s = ctypes.c_void_p()
            assert h.hipStreamCreate(ctypes.byref(s)) == 0
            ss.append(s)
        if spec.startswith("streams"):
            for s in ss:
                h.hipStreamDestroy(s)
            return None
        return ss
    if spec == "nullcopy":  # a synchronous copy on the null stream (creates the device's default queue user)
        h = hip()
        h.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        p, x = ctypes.c_void_p(), ctypes.c_int(1)
        assert h.hipMalloc(ctypes.byref(p), 64) == 0
        assert h.hipMemcpy(p, ctypes.byref(x), 4, 1) == 0
        h.hipFree(p)
        return None
    if spec.startswith("alloc"):
        gib = int(spec[5:])
        h = hip()
        ps = []
        for _ in range(gib * 4):
            p = ctypes.c_void_p()
            assert h.hipMalloc(ctypes.byref(p), 256 << 20) == 0
            ps.append(p)
        for p in ps:
            h.hipFree(p)
        return None
    w = configs.CFG3
    bg, new, met, fields, pc = bench.build_workload(w, 0)
    n = new.np
    mo, fo = np.zeros((n, met.shape[1])), [np.zeros((n, f.shape[1])) for f in fields]
    if spec == "host":
        ctx = TransferContext(0)
        ctx.set_background(bg.xyz, bg.tetv, bg.adja, bg.triv, bg.adjt, w.hausd)
        ctx.set_solutions(met, fields)
        ctx.locate_interp(new.xyz, pc, mo, fo)
        ctx.close()
        return None
    from parity import run_dev

    ctx = TransferContext(0, sort=None if spec == "big_auto" else False)
    run_dev(ctx, bg, new.xyz, met, fields, pc, w.hausd)
    ctx.close()
    return None


def child(spec: str):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import bench

    keep = prologue(spec)
    res = bench.groups_leg(types.SimpleNamespace(no_cpu_baseline=True))
    print("RESULT " + json.dumps({"groups": res["ms_per_group_groups_call"],
                                  "single": res["ms_per_group_single_calls"]}), flush=True)
    del keep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="base;big_auto")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--child", default=None)
    a = ap.parse_args()
    if a.child is not None:
        return child(a.child)
    vs = [v for v in a.variants.split(";") if v]
    res = {v: {"groups": [], "single": []} for v in vs}
    for r in range(a.rounds):
        for v in vs:
            p = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--child", v], stdout=subprocess.PIPE,
                               stderr=subprocess.STDOUT, text=True, timeout=600)
            line = [x for x in p.stdout.splitlines() if x.startswith("RESULT ")]
            if p.returncode != 0 or not line:
                print(p.stdout[-3000:])
                raise SystemExit(f"variant {v} failed")
            d = json.loads(line[-1][7:])
            for k in d:
                res[v][k].append(d[k])
            print(f"round {r} {v}: {d}", flush=True)
    print(f"{'variant':16s} {'groups ms/group':>16s} {'single ms/group':>16s}")
    for v in vs:
        print(f"{v:16s} {np.median(res[v]['groups']):16.4f} {np.median(res[v]['single']):16.4f}   "
              f"groups {['%.4f' % x for x in res[v]['groups']]}")


if __name__ == "__main__":
    main()
