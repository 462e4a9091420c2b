"""Halo-sharded background (BASELINE.json cfg5).

A rank owning a contiguous Morton range of the new points (ranks.morton_shards)
keeps only the background tetra whose bounding box meets the range's box
grown by a halo (csrc/pmmg_shard.c), instead of a replica of the whole group.
The shard is an ordinary background group for the transfer step: its local
ids ascend with the global ones, adjacency across the cut becomes a wall, and
the local->global id maps turn located elements back into group ids.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from ._native import host_lib
from .synth import Mesh

DEFAULT_HALO = -1.0  # the largest tetra extent around the range's box (and never less than hausd)
MAX_CELLS = 1 << 27  # occupancy grid of halo_shard_cells (coarser cells past that: a looser, still safe shard)


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


@dataclass
class HaloShard:
    mesh: Mesh              # local background (1-based local ids)
    tet_gid: np.ndarray     # (ne_local,) int32, 1-based group tetra id
    vert_gid: np.ndarray    # (np_local,) int32, 1-based group vertex id
    tria_gid: np.ndarray    # (nt_local,) int32, 1-based group tria id
    halo: float             # absolute halo used

    def rows(self, sol: np.ndarray) -> np.ndarray:
        """Vertex rows of a group solution restricted to the shard."""
        return np.ascontiguousarray(sol[self.vert_gid - 1])

    def to_group_elem(self, elem: np.ndarray, is_tria: np.ndarray) -> np.ndarray:
        """Local element ids (tetra, or trias where is_tria) -> group ids; 0 stays 0."""
        out = np.zeros_like(elem)
        e = elem.astype(np.int64)
        tet = (e > 0) & ~is_tria
        tri = (e > 0) & is_tria
        out[tet] = self.tet_gid[e[tet] - 1]
        out[tri] = self.tria_gid[e[tri] - 1]
        return out


def range_box(xyz: np.ndarray):
    """Bounding box of a rank's points (an empty range gives an empty box)."""
    if xyz.shape[0] == 0:
        return np.zeros(3), -np.ones(3)
    return xyz.min(axis=0), xyz.max(axis=0)


def max_tet_extent(bg: Mesh) -> float:
    return float(host_lib().pmmg_max_tet_extent(bg.np, _p(bg.xyz), bg.ne, _p(bg.tetv)))


def halo_shard(bg: Mesh, lo, hi, halo: float = DEFAULT_HALO, hausd: float = 0.0) -> HaloShard:
    """Shard of `bg` around the box [lo, hi] (halo < 0: in units of the
    largest tetra extent).  The halo is never less than 1.01 * hausd: a tria
    accepts a surface point within hausd of its plane (PMMG_locateChkDistTria,
    locate_pmmg.c:347-366) and the wedge / cone tests reach hausd too, so a
    thinner halo could drop the lowest-index accepting tria of a point and
    change the exhaustive search's answer against the whole group."""
    lib = host_lib()
    lo = np.ascontiguousarray(lo, np.float64)
    hi = np.ascontiguousarray(hi, np.float64)
    h = -halo * max_tet_extent(bg) if halo < 0 else float(halo)
    h = max(h, 1.01 * float(hausd))
    tet_map = np.empty(bg.ne, np.int32)
    vert_map = np.empty(bg.np, np.int32)
    counts = (ctypes.c_int64 * 2)()
    if not lib.pmmg_shard_mark(bg.np, _p(bg.xyz), bg.ne, _p(bg.tetv), _p(lo), _p(hi), h, _p(tet_map),
                               _p(vert_map), counts):
        raise ValueError("pmmg_shard_mark: invalid background")
    return _fill(bg, tet_map, vert_map, counts, h)


def halo_shard_cells(bg: Mesh, q_xyz: np.ndarray, halo: float = DEFAULT_HALO, hausd: float = 0.0,
                     cell_factor: float = 1.0) -> HaloShard:
    """Shard of `bg` around the points q_xyz: the tetra whose bounding box,
    grown by the halo, meets the points' box and a cell (side cell_factor x
    halo) of a grid over the group that holds one of the points.  Same guarantees as halo_shard
    (every tetra or tria that can accept a point is kept, the halo is never
    less than 1.01 * hausd), far fewer tetra for a Morton range whose box is
    large (a range of a shell)."""
    lib = host_lib()
    h = -halo * max_tet_extent(bg) if halo < 0 else float(halo)
    h = max(h, 1.01 * float(hausd))
    cell = cell_factor * h
    ext = bg.xyz.max(axis=0) - bg.xyz.min(axis=0)
    cell = max(cell, float(np.cbrt(np.prod(ext + 2 * cell) / MAX_CELLS)))  # a mask of at most ~MAX_CELLS bytes
    g_lo = bg.xyz.min(axis=0) - cell
    g_n = np.maximum(1, np.ceil((bg.xyz.max(axis=0) + cell - g_lo) / cell).astype(np.int64))
    occ = np.zeros(int(np.prod(g_n)), np.uint8)
    if q_xyz.shape[0]:
        c = np.clip(np.floor((q_xyz - g_lo) / cell).astype(np.int64), 0, g_n - 1)
        occ[c[:, 0] + g_n[0] * (c[:, 1] + g_n[1] * c[:, 2])] = 1
    g_lo = np.ascontiguousarray(g_lo, np.float64)
    g_n32 = np.ascontiguousarray(g_n, np.int32)
    tet_map = np.empty(bg.ne, np.int32)
    vert_map = np.empty(bg.np, np.int32)
    counts = (ctypes.c_int64 * 2)()
    lo, hi = (np.ascontiguousarray(x, np.float64) for x in range_box(q_xyz))
    if not lib.pmmg_shard_mark_cells(bg.np, _p(bg.xyz), bg.ne, _p(bg.tetv), _p(lo), _p(hi), _p(g_lo), cell,
                                     _p(g_n32), _p(occ), h, _p(tet_map), _p(vert_map), counts):
        raise ValueError("pmmg_shard_mark_cells: invalid background")
    return _fill(bg, tet_map, vert_map, counts, h)


def _fill(bg: Mesh, tet_map, vert_map, counts, h: float) -> HaloShard:
    lib = host_lib()
    nk, nv = int(counts[0]), int(counts[1])
    xyz = np.empty((nv, 3), np.float64)
    tetv = np.empty((nk, 4), np.int32)
    adja = np.empty((nk, 4), np.int32)
    triv = np.empty((bg.nt, 3), np.int32)
    adjt = np.empty((bg.nt, 3), np.int32)
    tet_gid = np.empty(nk, np.int32)
    vert_gid = np.empty(nv, np.int32)
    tria_gid = np.empty(bg.nt, np.int32)
    nt = lib.pmmg_shard_fill(bg.np, _p(bg.xyz), bg.ne, _p(bg.tetv), _p(bg.adja), bg.nt, _p(bg.triv),
                             _p(bg.adjt), _p(tet_map), _p(vert_map), _p(xyz), _p(tetv), _p(adja), _p(triv),
                             _p(adjt), _p(tet_gid), _p(vert_gid), _p(tria_gid))
    if nt < 0:
        raise ValueError("pmmg_shard_fill: invalid background")
    isbdy = bg.isbdy[vert_gid - 1] if bg.isbdy is not None and bg.isbdy.size == bg.np else np.zeros(nv, np.uint8)
    mesh = Mesh(bg.kind, bg.n, xyz, tetv, adja, np.ascontiguousarray(triv[:nt]), np.ascontiguousarray(adjt[:nt]),
                np.ascontiguousarray(isbdy))
    return HaloShard(mesh, tet_gid, vert_gid, np.ascontiguousarray(tria_gid[:nt]), h)
