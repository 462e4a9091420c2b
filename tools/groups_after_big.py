"""The groups leg after a large call in the same process (a large call
creates the high-priority surface stream; r04zf's bench line measured its
groups leg at 0.24 ms per group against 0.093 in a process without one):
    python tools/groups_after_big.py [big_config [auto|on|off]]"""
import os
import sys
import types

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from parmmg_amd import configs  # noqa: E402
from parmmg_amd.transfer import TransferContext  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
w = configs.SHORT.get(name)
if w is not None:
    bg, new, met, fields, pc = bench.build_workload(w, 0)
    sort = {"auto": None, "on": True, "off": False}[sys.argv[2] if len(sys.argv) > 2 else "auto"]
    ctx = TransferContext(0, sort=sort)
    ctx.set_background(bg.xyz, bg.tetv, bg.adja, bg.triv, bg.adjt, w.hausd)
    ctx.set_solutions(met, fields)
    n = new.np
    mo, fo = np.zeros((n, met.shape[1])), [np.zeros((n, f.shape[1])) for f in fields]
    for _ in range(2):
        st = ctx.locate_interp(new.xyz, pc, mo, fo)
    print(f"big call: {w.name}, {n} points, sorted={st.sorted}", flush=True)
    ctx.close()
res = bench.groups_leg(types.SimpleNamespace(no_cpu_baseline=True))
print("groups:", res["ms_per_group_groups_call"], "single:", res["ms_per_group_single_calls"], flush=True)
