"""Synthetic meshes and solutions — numpy front-end of
``csrc/pmmg_synth.c``.  Test and benchmark support, not part of the transfer
path itself."""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from ._native import synth_lib

CUBE, SHELL = 0, 1
SEED = 0x5EED2025

# analytic solutions of pmmg_synth.h
F_ISO, F_ANI, F_SCALAR, F_VECTOR, F_TENSOR, F_AFFINE, F_AFFINE_VEC, F_CONST_TENSOR = range(8)


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


@dataclass
class Mesh:
    """A tetrahedral mesh in the C-ABI layout (row r = entity r+1, 1-based ids)."""

    kind: int
    n: int
    xyz: np.ndarray                 # (np, 3) float64
    tetv: np.ndarray                # (ne, 4) int32
    adja: np.ndarray                # (ne, 4) int32, 4*k+i
    triv: np.ndarray                # (nt, 3) int32
    adjt: np.ndarray                # (nt, 3) int32, 3*k+i
    isbdy: np.ndarray               # (np,) uint8
    extra: dict = field(default_factory=dict)

    @property
    def np(self) -> int:
        return int(self.xyz.shape[0])

    @property
    def ne(self) -> int:
        return int(self.tetv.shape[0])

    @property
    def nt(self) -> int:
        return int(self.triv.shape[0])


def counts(kind: int, n: int) -> tuple[int, int, int]:
    out = (ctypes.c_int64 * 3)()
    if not synth_lib().synth_counts(kind, n, out):
        raise ValueError(f"invalid lattice kind={kind} n={n}")
    return int(out[0]), int(out[1]), int(out[2])


def lattice(kind: int, n: int, jitter: float = 0.0, seed: int = SEED, with_trias: bool = True,
            with_tetra: bool = True, valid: bool = False) -> Mesh:
    """with_tetra=False: vertices and boundary flags only (a new mesh whose
    points are the queries; no connectivity is generated).  valid=True: the
    jitter capped per vertex so that the lattice's tetra stay positive
    (synth_vertices_valid) — for a jittered mesh that later serves as a
    background (the shell's radial map leaves slivers that the plain jitter
    inverts: 0.23 % of the tetra at jitter 0.2)."""
    lib = synth_lib()
    npt, ne, nt = counts(kind, n)
    xyz = np.empty((npt, 3), np.float64)
    isbdy = np.empty(npt, np.uint8)
    gen = lib.synth_vertices_valid if valid else lib.synth_vertices
    if not gen(kind, n, float(jitter), seed, _ptr(xyz), _ptr(isbdy)):
        raise RuntimeError("synth_vertices failed")
    if not with_tetra:
        empty4 = np.zeros((0, 4), np.int32)
        return Mesh(kind, n, xyz, empty4, empty4, np.zeros((0, 3), np.int32), np.zeros((0, 3), np.int32), isbdy)
    tetv = np.empty((ne, 4), np.int32)
    adja = np.empty((ne, 4), np.int32)
    if not lib.synth_tetra(kind, n, _ptr(tetv), _ptr(adja)):
        raise RuntimeError("synth_tetra failed")
    if with_trias:
        triv = np.empty((nt, 3), np.int32)
        adjt = np.empty((nt, 3), np.int32)
        got = lib.synth_trias(ne, _ptr(tetv), _ptr(adja), _ptr(triv), _ptr(adjt))
        if got != nt:
            raise RuntimeError(f"synth_trias produced {got} trias, expected {nt}")
    else:
        triv = np.zeros((0, 3), np.int32)
        adjt = np.zeros((0, 3), np.int32)
    return Mesh(kind, n, xyz, tetv, adja, triv, adjt, isbdy)


def solution(which: int, xyz: np.ndarray) -> np.ndarray:
    lib = synth_lib()
    size = lib.synth_field_size(which)
    out = np.empty((xyz.shape[0], size), np.float64)
    if not lib.synth_field(which, xyz.shape[0], _ptr(np.ascontiguousarray(xyz)), _ptr(out)):
        raise RuntimeError("synth_field failed")
    return out


def visit_order(new: Mesh) -> np.ndarray:
    """Reference point visitation order (first appearance in new-tetra order)."""
    order = np.empty(new.np, np.int32)
    cnt = synth_lib().synth_visit_order(new.ne, _ptr(new.tetv), new.np, _ptr(order))
    return order[:cnt]


def classes(new: Mesh, req_every: int = 0) -> np.ndarray:
    pc = np.empty(new.np, np.uint8)
    synth_lib().synth_classes(new.np, _ptr(new.isbdy), int(req_every), _ptr(pc))
    return pc


# ---------------------------------------------------------------- graded / stretched meshes
#
# The reference's anisotropic runs remesh a torus around a planar shock
# (cmake/testing/pmmg_tests.cmake:52-63): the adapted meshes are strongly
# graded towards the shock and their elements there are flat.  Here a cube
# lattice is mapped per vertex: each axis d by a sinh clustering around the
# plane x_d = c_d (cell size grows by grading[d] from that plane to the
# farther face), then sheared so the planes are oblique (z += shear * (x -
# 1/2)).  Cells at the centre are grading-times smaller than at the corners
# in every direction; cells on one plane far from the others are flat
# (aspect ratio up to the grading).  The map is monotone per axis, so every
# Kuhn tetra keeps a positive volume; faces stay planar and map onto
# themselves for every centre, so the boundary points of a new mesh graded
# around other planes lie on the background's surface.


def shock_map(t: np.ndarray, z_s: float, grading: float) -> np.ndarray:
    """[0, 1] -> [0, 1], z(t) = z_s + A sinh(beta (t - t_s)): the cell size
    dz/dt is smallest at the shock and `grading` times larger at the farther
    face (beta = acosh(grading) / max(t_s, 1 - t_s))."""
    t = np.asarray(t, np.float64)
    if grading <= 1.0:
        return t.copy()

    def solve(beta):
        lo, hi = 1e-12, 1.0 - 1e-12  # t_s: sinh(beta t_s) / sinh(beta (1 - t_s)) = z_s / (1 - z_s)
        for _ in range(200):
            mid = 0.5 * (lo + hi)
            if np.sinh(beta * mid) * (1.0 - z_s) < np.sinh(beta * (1.0 - mid)) * z_s:
                lo = mid
            else:
                hi = mid
        return 0.5 * (lo + hi)

    beta, t_s = 1.0, 0.5
    for _ in range(50):  # fixed point: beta depends on the farther side, t_s on beta
        t_s = solve(beta)
        beta = float(np.arccosh(grading)) / max(t_s, 1.0 - t_s)
    A = z_s / np.sinh(beta * t_s)
    z = z_s + A * np.sinh(beta * (t - t_s))
    z[t <= 0.0] = 0.0
    z[t >= 1.0] = 1.0
    return z


def graded(lat: Mesh, centre=(0.5, 0.5, 0.5), grading=(1000.0, 1000.0, 1000.0), shear: float = 0.3) -> Mesh:
    """A cube lattice (synth.CUBE, coordinates in [0, 1]^3) graded towards the
    planes x_d = centre[d] and sheared (see above); connectivity unchanged."""
    if lat.kind != CUBE:
        raise ValueError("graded meshes are built from cube lattices")
    xyz = lat.xyz.copy()
    for d in range(3):
        xyz[:, d] = shock_map(xyz[:, d], centre[d], grading[d])
    xyz[:, 2] += shear * (xyz[:, 0] - 0.5)
    m = Mesh(lat.kind, lat.n, np.ascontiguousarray(xyz), lat.tetv, lat.adja, lat.triv, lat.adjt, lat.isbdy,
             dict(lat.extra))
    m.extra["graded"] = dict(centre=tuple(centre), grading=tuple(grading), shear=shear)
    return m


def cell_stats(m: Mesh) -> dict:
    """Element-size grading and stretching of a mesh: the ratio of the
    largest to the smallest tetra edge-length scale (cube root of |volume|)
    and the largest aspect ratio (longest edge / shortest edge of a tetra)."""
    p = m.xyz[m.tetv - 1]
    e = np.stack([p[:, 1] - p[:, 0], p[:, 2] - p[:, 0], p[:, 3] - p[:, 0],
                  p[:, 2] - p[:, 1], p[:, 3] - p[:, 1], p[:, 3] - p[:, 2]], axis=1)
    L = np.linalg.norm(e, axis=2)
    vol = np.abs(np.einsum("ij,ij->i", e[:, 0], np.cross(e[:, 1], e[:, 2]))) / 6.0
    h = np.cbrt(vol)
    return {"size_grading": float(h.max() / h.min()), "max_aspect": float((L.max(1) / L.min(1)).max()),
            "min_volume": float(vol.min())}


def mmg_like_perm(nq: int) -> np.ndarray:
    """A numbering of the new points like Mmg's output after an adaptation
    (src/libparmmg1.c:692-741: the group is renumbered, then Mmg keeps the
    retained vertices in their order and appends the vertices it inserts,
    in creation order): one point in six (a splitmix64 hash of its id,
    spread evenly over the domain) counts as inserted and moves to the end,
    both parts keeping the generator's order.  perm[new id] = old id."""
    ids = np.arange(nq, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = ids * np.uint64(0x9E3779B97F4A7C15) + np.uint64(0x5EED2025)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    ins = (z % np.uint64(6)) == 0
    return np.concatenate([np.nonzero(~ins)[0], np.nonzero(ins)[0]])
