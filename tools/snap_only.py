"""The device background snapshot alone (pmmg_hip_build_adjacency +
pmmg_hip_build_boundary) on a config's background, for kernel traces:
    python tools/snap_only.py [cfg4] [reps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parmmg_amd import configs, synth  # noqa: E402
from parmmg_amd.transfer import TransferContext  # noqa: E402

w = configs.SHORT[sys.argv[1] if len(sys.argv) > 1 else "cfg4"]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
bg = synth.lattice(w.kind, w.n_old, jitter=0.0)
with TransferContext(0) as ctx:
    d_tetv = ctx.upload(bg.tetv)
    d_tet8 = ctx.empty((bg.ne, 8), np.int32)
    for r in range(reps):
        t0 = time.perf_counter()
        ctx.build_adjacency(bg.np, d_tetv, adja=False, tet8=True, out=(None, d_tet8))
        t1 = time.perf_counter()
        triv, adjt = ctx.build_boundary(bg.np, tet8=d_tet8)
        t2 = time.perf_counter()
        print(f"rep {r}: adjacency {1e3 * (t1 - t0):.2f} ms, boundary {1e3 * (t2 - t1):.2f} ms", flush=True)
        triv.free()
        adjt.free()
