"""Generate the committed golden vectors of tests/golden/.

Inputs are the reference's own fixtures (libexamples/adaptation_example0:
cube.mesh, cube-met.sol, cube-solphys.sol, copied here as data) plus one
synthetic Kuhn lattice; the adapted mesh of the cube is its uniform 1:8
refinement (the reference adapts with Mmg, which is not available).
Expected outputs come from the CPU oracle (oracle/pmmg_oracle.c) in
reference visitation order with the reference's persistent cone state
(ORC_MODE_FAITHFUL).  The reference itself cannot be built here (no Mmg), so
these vectors pin regressions of the oracle and of the HIP module; the
analytic known answers of tests/test_oracle.py pin the oracle's arithmetic.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from parmmg_amd import medit, synth  # noqa: E402
from parmmg_amd.synth import Mesh  # noqa: E402


def cube_case():
    m = medit.read_mesh(os.path.join(HERE, "cube.mesh"))
    adja = medit.tetra_adjacency(m["tetv"])
    triv = medit.boundary_trias(m["tetv"], adja)
    adjt = medit.tria_adjacency(triv)
    bg = Mesh(0, 0, m["xyz"], m["tetv"], adja, triv, adjt, np.zeros(m["xyz"].shape[0], np.uint8))
    met = medit.read_sol(os.path.join(HERE, "cube-met.sol"))[0]
    fields = medit.read_sol(os.path.join(HERE, "cube-solphys.sol"))
    xyz_new, tet_new, _ = medit.refine8(m["xyz"], m["tetv"])
    on_bdy = np.any((np.abs(xyz_new) < 1e-12) | (np.abs(xyz_new - 1.0) < 1e-12), axis=1)
    pclass = np.where(on_bdy, 2, 1).astype(np.uint8)
    visit = synth.visit_order(Mesh(0, 0, xyz_new, tet_new, tet_new, np.zeros((0, 3), np.int32),
                                   np.zeros((0, 3), np.int32), on_bdy.astype(np.uint8)))
    return bg, met, fields, xyz_new, pclass, visit


def lattice_case():
    bg = synth.lattice(synth.CUBE, 4)
    new = synth.lattice(synth.CUBE, 5, jitter=0.2)
    met = synth.solution(synth.F_ANI, bg.xyz)
    fields = [synth.solution(w, bg.xyz) for w in (synth.F_SCALAR, synth.F_VECTOR, synth.F_TENSOR)]
    return bg, met, fields, new.xyz, synth.classes(new, req_every=9), synth.visit_order(new)


def save(name, bg, met, fields, xyz_new, pclass, visit):
    B = O.Background(bg, met, fields, 0.01)
    r = O.run(B, xyz_new, pclass, visit, O.MODE_FAITHFUL)
    arrs = dict(bg_xyz=bg.xyz, bg_tetv=bg.tetv, bg_adja=bg.adja, bg_triv=bg.triv, bg_adjt=bg.adjt, met=met,
                new_xyz=xyz_new, pclass=pclass, visit=visit, out_elem=r["elem"], out_hit=r["hit"],
                out_loc=r["loc"], out_minbary=r["minbary"], out_met=r["met"], nfield=np.array(len(fields)))
    for j, f in enumerate(fields):
        arrs[f"field{j}"] = f
        arrs[f"out_field{j}"] = r["fields"][j]
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrs)
    print(name, "points", xyz_new.shape[0], "hits", np.bincount(r["hit"]))


if __name__ == "__main__":
    save("cube_refine8", *cube_case())
    save("lattice_4_5_aniso", *lattice_case())
