"""The workloads of BASELINE.json ``configs``.

Each config names a background lattice, an adapted lattice, the metric and
the solution fields.  Sizes (tetra / vertices) match SURVEY.md §8(d) exactly.
"""
from __future__ import annotations

from dataclasses import dataclass

from . import synth


@dataclass(frozen=True)
class Workload:
    name: str
    kind: int          # synth.CUBE / synth.SHELL
    n_old: int         # background lattice cells per side
    n_new: int         # adapted lattice cells per side
    metric: int        # synth.F_ISO / synth.F_ANI
    fields: tuple      # synth.F_* of each solution field
    hausd: float = 0.01  # Mmg default Hausdorff parameter
    jitter_new: float = 0.2
    description: str = ""
    # graded / stretched variant (synth.graded): (centre of the background's
    # clustering planes, centre of the new mesh's, grading per axis, shear)
    grade: tuple | None = None

    @property
    def met_size(self) -> int:
        return 6 if self.metric == synth.F_ANI else 1

    def field_sizes(self) -> list[int]:
        return [{synth.F_ISO: 1, synth.F_ANI: 6, synth.F_SCALAR: 1, synth.F_VECTOR: 3, synth.F_TENSOR: 6,
                 synth.F_AFFINE: 1, synth.F_AFFINE_VEC: 3, synth.F_CONST_TENSOR: 6}[f] for f in self.fields]

    @property
    def K(self) -> int:
        """doubles per vertex across the metric and all fields"""
        return self.met_size + sum(self.field_sizes())

    def counts(self):
        return synth.counts(self.kind, self.n_old), synth.counts(self.kind, self.n_new)

    def algorithmic_bytes(self, np_new_located: int | None = None) -> int:
        """B = np_n(24 + 4 + 8K) + ne_o*32 + np_o(24 + 8K)   (SURVEY.md §8(d))."""
        (np_o, ne_o, _), (np_n, _, _) = self.counts()
        if np_new_located is not None:
            np_n = np_new_located
        K = self.K
        return np_n * (24 + 4 + 8 * K) + ne_o * 32 + np_o * (24 + 8 * K)


def build_meshes(w: Workload, seed: int = synth.SEED, with_new_tetra: bool = False):
    """(background, new mesh) of a workload: lattices, graded when w.grade
    (the new points jittered in lattice space before the map, so by
    +-jitter of their local cell size)."""
    bg = synth.lattice(w.kind, w.n_old, jitter=0.0)
    new = synth.lattice(w.kind, w.n_new, jitter=w.jitter_new, seed=seed, with_trias=False,
                        with_tetra=with_new_tetra)
    if w.grade is not None:
        c_old, c_new, grading, shear = w.grade
        bg = synth.graded(bg, c_old, grading, shear)
        new = synth.graded(new, c_new, grading, shear)
    return bg, new


CFG2 = Workload("cfg2-cube1M-iso", synth.CUBE, 55, 58, synth.F_ISO, (synth.F_SCALAR,),
                description="1M-tet synthetic unit cube, analytic iso metric, 1 scalar field")
CFG3 = Workload("cfg3-cube20M-aniso", synth.CUBE, 150, 159, synth.F_ANI,
                (synth.F_SCALAR, synth.F_VECTOR, synth.F_TENSOR),
                description="20M-tet cube, 6-component aniso metric + 3 fields")
CFG4 = Workload("cfg4-shell100M-aniso", synth.SHELL, 268, 284, synth.F_ANI,
                (synth.F_SCALAR, synth.F_VECTOR, synth.F_TENSOR),
                description="100M-tet sphere/shell, aniso metric + 3 fields")
CFG5 = Workload("cfg5-cube500M-iso", synth.CUBE, 437, 464, synth.F_ISO,
                (synth.F_SCALAR, synth.F_AFFINE, synth.F_SCALAR, synth.F_AFFINE, synth.F_SCALAR),
                description="500M-tet cube, iso metric + 5 fields")

# graded and stretched (not a BASELINE config: the parity / robustness case
# of the reference's anisotropic torus-with-a-planar-shock runs,
# cmake/testing/pmmg_tests.cmake:52-63): cfg3's lattices with the cell size
# graded 1000x towards three planes per mesh (the new mesh's planes moved
# against the background's, as an adapted mesh follows a moving shock) and
# sheared; elements up to ~1000:1 near the planes
GRADE = ((0.5, 0.5, 0.5), (0.52, 0.47, 0.515), (1000.0, 1000.0, 1000.0), 0.3)
CFGG = Workload("cfgG-cube20M-graded-aniso", synth.CUBE, 150, 159, synth.F_ANI,
                (synth.F_SCALAR, synth.F_VECTOR, synth.F_TENSOR), grade=GRADE,
                description="20M-tet cube graded 1000x towards three planes and sheared (elements up to ~1000:1), "
                            "aniso metric + 3 fields")

ALL = {w.name: w for w in (CFG2, CFG3, CFG4, CFG5, CFGG)}
SHORT = {"cfg2": CFG2, "cfg3": CFG3, "cfg4": CFG4, "cfg5": CFG5, "cfgG": CFGG}


def small(kind: int = synth.CUBE, n_old: int = 6, n_new: int = 7, ani: bool = True) -> Workload:
    """Oracle-sized variant used by the parity tests."""
    if ani:
        return Workload(f"small-{kind}-{n_old}-{n_new}-ani", kind, n_old, n_new, synth.F_ANI,
                        (synth.F_SCALAR, synth.F_VECTOR, synth.F_TENSOR))
    return Workload(f"small-{kind}-{n_old}-{n_new}-iso", kind, n_old, n_new, synth.F_ISO,
                    (synth.F_SCALAR, synth.F_AFFINE))
