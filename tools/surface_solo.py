"""The surface branch of cfg4 alone (volume points marked skipped), for
kernel traces: prints the stats of each call.

  rocprofv3 --kernel-trace --stats -d out -- python3 tools/surface_solo.py --steps 5
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--env", default="", help="PMMG_HIP_* settings, NAME=value,...")
    args = ap.parse_args()
    for item in filter(None, args.env.split(",")):
        k, v = item.split("=")
        os.environ["PMMG_HIP_" + k.upper()] = v
    w = configs.SHORT[args.config]
    bg, new = configs.build_meshes(w)
    met = synth.solution(w.metric, bg.xyz)
    fields = [synth.solution(f, bg.xyz) for f in w.fields]
    pc = synth.classes(new)
    pc = np.where(pc == 2, 2, 0).astype(np.uint8)
    with TransferContext(0) as ctx:
        d = dict(xyz=ctx.upload(bg.xyz), tet8=ctx.upload(pack_tet8(bg.tetv, bg.adja)), triv=ctx.upload(bg.triv),
                 adjt=ctx.upload(bg.adjt), met=ctx.upload(met), f=[ctx.upload(f) for f in fields],
                 q=ctx.upload(new.xyz), pc=ctx.upload(pc), mo=ctx.empty((new.np, w.met_size), np.float64),
                 fo=[ctx.empty((new.np, f.shape[1]), np.float64) for f in fields],
                 el=ctx.empty((new.np,), np.int32), hit=ctx.empty((new.np,), np.int8))
        for s in range(args.steps + 1):
            ctx.set_background_tet8(d["xyz"], d["tet8"], d["triv"], d["adjt"], w.hausd)
            ctx.set_solutions(d["met"], d["f"])
            ctx.locate_interp(d["q"], d["pc"], d["mo"], d["fo"], d["el"], d["hit"], sync=False)
            st = ctx.sync()
            n = max(1, st.nbdy)
            print(f"call {s}: nbdy {st.nbdy} steps/pt {st.steps_total / n:.3f} stepmax {st.stepmax} "
                  f"face {st.nbdy_face} edge {st.nbdy_edge} vertex {st.nbdy_vertex} wedge {st.nbdy_wedge} "
                  f"cone {st.nbdy_cone} exhaust {st.nbdy_exhaust} ms_bdy {st.ms_bdy:.4f} ms_total {st.ms_total:.4f}",
                  flush=True)


if __name__ == "__main__":
    main()
