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
            with_tetra: bool = True) -> Mesh:
    """with_tetra=False: vertices and boundary flags only (a new mesh whose
    points are the queries; no connectivity is generated)."""
    lib = synth_lib()
    npt, ne, nt = counts(kind, n)
    xyz = np.empty((npt, 3), np.float64)
    isbdy = np.empty(npt, np.uint8)
    if not lib.synth_vertices(kind, n, float(jitter), seed, _ptr(xyz), _ptr(isbdy)):
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
