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
    sol: np.ndarray | None = None  # (np_local, K) vertex rows, when built from parts (shard_from_parts)

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


class _Region(ctypes.Structure):
    """pmmg_shard_region of csrc/pmmg_host.h"""
    _fields_ = [("box_lo", ctypes.c_void_p), ("box_hi", ctypes.c_void_p), ("g_lo", ctypes.c_double * 3),
                ("cell", ctypes.c_double), ("g_n", ctypes.c_int * 3), ("occ", ctypes.c_void_p),
                ("halo", ctypes.c_double)]


@dataclass
class Region:
    """What a rank's points need of the background (pmmg_shard_mark_cells's
    test): the points' box, and an occupancy mask of the grid cells that hold
    one of them, both grown by the halo when elements are tested."""
    lo: np.ndarray
    hi: np.ndarray
    g_lo: np.ndarray
    cell: float
    g_n: np.ndarray
    occ: np.ndarray  # uint8, g_n[0] * g_n[1] * g_n[2] (x fastest)
    halo: float

    def c(self) -> _Region:
        self._keep = [np.ascontiguousarray(self.lo, np.float64), np.ascontiguousarray(self.hi, np.float64),
                      np.ascontiguousarray(self.occ, np.uint8)]
        return _Region(_p(self._keep[0]), _p(self._keep[1]), (ctypes.c_double * 3)(*[float(x) for x in self.g_lo]),
                       float(self.cell), (ctypes.c_int * 3)(*[int(x) for x in self.g_n]), _p(self._keep[2]),
                       float(self.halo))


def grid_for(lo, hi, h: float, cell_factor: float = 1.0):
    """The occupancy grid over a group's box [lo, hi] for halo h (cells of
    cell_factor x h, coarser past MAX_CELLS): (g_lo, cell, g_n)."""
    lo, hi = np.asarray(lo, np.float64), np.asarray(hi, np.float64)
    cell = cell_factor * h
    ext = hi - lo
    cell = max(cell, float(np.cbrt(np.prod(ext + 2 * cell) / MAX_CELLS)))  # a mask of at most ~MAX_CELLS bytes
    g_lo = lo - cell
    g_n = np.maximum(1, np.ceil((hi + cell - g_lo) / cell).astype(np.int64))
    return g_lo, cell, g_n


def region_of(q_xyz: np.ndarray, g_lo, cell: float, g_n, h: float) -> Region:
    occ = np.zeros(int(np.prod(g_n)), np.uint8)
    if q_xyz.shape[0]:
        c = np.clip(np.floor((q_xyz - g_lo) / cell).astype(np.int64), 0, g_n - 1)
        occ[c[:, 0] + g_n[0] * (c[:, 1] + g_n[1] * c[:, 2])] = 1
    lo, hi = range_box(q_xyz)
    return Region(np.asarray(lo, np.float64), np.asarray(hi, np.float64), np.asarray(g_lo, np.float64), float(cell),
                  np.asarray(g_n, np.int64), occ, float(h))


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
    g_lo, cell, g_n = grid_for(bg.xyz.min(axis=0), bg.xyz.max(axis=0), h, cell_factor)
    reg = region_of(q_xyz, g_lo, cell, g_n, h)
    g_lo = np.ascontiguousarray(g_lo, np.float64)
    g_n32 = np.ascontiguousarray(g_n, np.int32)
    tet_map = np.empty(bg.ne, np.int32)
    vert_map = np.empty(bg.np, np.int32)
    counts = (ctypes.c_int64 * 2)()
    lo, hi = (np.ascontiguousarray(x, np.float64) for x in (reg.lo, reg.hi))
    if not lib.pmmg_shard_mark_cells(bg.np, _p(bg.xyz), bg.ne, _p(bg.tetv), _p(lo), _p(hi), _p(g_lo), cell,
                                     _p(g_n32), _p(reg.occ), h, _p(tet_map), _p(vert_map), counts):
        raise ValueError("pmmg_shard_mark_cells: invalid background")
    # trias: those meeting the region (the rule the part builders share; every
    # tria that can accept one of the points is among them)
    tria_map = np.empty(bg.nt, np.int32)
    creg = reg.c()
    if lib.pmmg_shard_mark_trias(bg.np, _p(bg.xyz), bg.nt, _p(bg.triv), ctypes.byref(creg), _p(tria_map)) < 0:
        raise ValueError("pmmg_shard_mark_trias: invalid background")
    return _fill(bg, tet_map, vert_map, counts, h, tria_map)


def _fill(bg: Mesh, tet_map, vert_map, counts, h: float, tria_map=None) -> HaloShard:
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
    if tria_map is None:  # the boundary trias with all three vertices in the shard
        nt = lib.pmmg_shard_fill(bg.np, _p(bg.xyz), bg.ne, _p(bg.tetv), _p(bg.adja), bg.nt, _p(bg.triv),
                                 _p(bg.adjt), _p(tet_map), _p(vert_map), _p(xyz), _p(tetv), _p(adja), _p(triv),
                                 _p(adjt), _p(tet_gid), _p(vert_gid), _p(tria_gid))
    else:
        nt = lib.pmmg_shard_fill_region(bg.np, _p(bg.xyz), bg.ne, _p(bg.tetv), _p(bg.adja), bg.nt, _p(bg.triv),
                                        _p(bg.adjt), _p(tet_map), _p(vert_map), _p(tria_map), _p(xyz), _p(tetv),
                                        _p(adja), _p(triv), _p(adjt), _p(tet_gid), _p(vert_gid), _p(tria_gid))
    if nt < 0:
        raise ValueError("pmmg_shard_fill: invalid background")
    isbdy = bg.isbdy[vert_gid - 1] if bg.isbdy is not None and bg.isbdy.size == bg.np else np.zeros(nv, np.uint8)
    mesh = Mesh(bg.kind, bg.n, xyz, tetv, adja, np.ascontiguousarray(triv[:nt]), np.ascontiguousarray(adjt[:nt]),
                np.ascontiguousarray(isbdy))
    return HaloShard(mesh, tet_gid, vert_gid, np.ascontiguousarray(tria_gid[:nt]), h)


# ---------------------------------------------------------------- shards from the ranks' parts
#
# A distributed group: rank r holds only its part (pmmg_shard_part of
# csrc/pmmg_host.h) — here the group's tetra and trias cut into contiguous
# id ranges, with every vertex they use.  Each rank packs for every rank d
# the records of its part that d's region needs (pmmg_shard_part_pack), an
# all-to-all exchanges them, and each rank assembles its shard
# (pmmg_shard_assemble): the shard halo_shard_cells builds from the whole
# group, without any rank holding the whole group.


class _Part(ctypes.Structure):
    _fields_ = [("np", ctypes.c_int), ("ne", ctypes.c_int), ("nt", ctypes.c_int), ("K", ctypes.c_int),
                ("vert_gid", ctypes.c_void_p), ("xyz", ctypes.c_void_p), ("sol", ctypes.c_void_p),
                ("tet_gid", ctypes.c_void_p), ("tetv", ctypes.c_void_p), ("adja", ctypes.c_void_p),
                ("tria_gid", ctypes.c_void_p), ("triv", ctypes.c_void_p), ("adjt", ctypes.c_void_p)]


@dataclass
class Part:
    """A rank's part of a background group (global 1-based ids, ascending)."""
    vert_gid: np.ndarray
    xyz: np.ndarray
    sol: np.ndarray      # (np, K)
    tet_gid: np.ndarray
    tetv: np.ndarray     # global vertex ids
    adja: np.ndarray     # the group's codes
    tria_gid: np.ndarray
    triv: np.ndarray
    adjt: np.ndarray

    def c(self) -> _Part:
        K = int(self.sol.shape[1]) if self.sol is not None and self.sol.ndim == 2 else 0
        self._keep = [np.ascontiguousarray(a) for a in (self.vert_gid, self.xyz, self.sol, self.tet_gid, self.tetv,
                                                        self.adja, self.tria_gid, self.triv, self.adjt)]
        k = self._keep
        return _Part(int(k[0].shape[0]), int(k[3].shape[0]), int(k[6].shape[0]), K, *[_p(a) for a in k])


def part_of(bg: Mesh, sol: np.ndarray, r: int, world: int) -> Part:
    """Rank r's part of the group `bg` (test / bench stand-in for a
    distributed mesh): tetra and trias in contiguous id ranges, every vertex
    they use, with its solution rows sol[np, K]."""
    k0, k1 = bg.ne * r // world, bg.ne * (r + 1) // world
    t0, t1 = bg.nt * r // world, bg.nt * (r + 1) // world
    used = np.zeros(bg.np + 1, bool)
    used[bg.tetv[k0:k1].ravel()] = True
    used[bg.triv[t0:t1].ravel()] = True
    vg = np.nonzero(used)[0].astype(np.int32)
    return Part(vg, bg.xyz[vg - 1], np.ascontiguousarray(sol[vg - 1]), np.arange(k0 + 1, k1 + 1, dtype=np.int32),
                np.ascontiguousarray(bg.tetv[k0:k1]), np.ascontiguousarray(bg.adja[k0:k1]),
                np.arange(t0 + 1, t1 + 1, dtype=np.int32), np.ascontiguousarray(bg.triv[t0:t1]),
                np.ascontiguousarray(bg.adjt[t0:t1]))


def pack_part(part: Part, reg: Region) -> np.ndarray:
    """pmmg_shard_part_pack: the records of `part` that `reg` needs (bytes)."""
    lib = host_lib()
    cp, cr = part.c(), reg.c()
    n = lib.pmmg_shard_part_pack(ctypes.byref(cp), ctypes.byref(cr), None, 0)
    if n < 0:
        raise ValueError("pmmg_shard_part_pack: invalid part or region")
    buf = np.empty(int(n), np.uint8)
    if lib.pmmg_shard_part_pack(ctypes.byref(cp), ctypes.byref(cr), _p(buf), int(n)) != n:
        raise ValueError("pmmg_shard_part_pack failed")
    return buf


def assemble(bufs, K: int, kind: int = 0, n: int = 0, halo: float = 0.0) -> HaloShard:
    """pmmg_shard_assemble: the shard from every rank's buffer for this rank."""
    lib = host_lib()
    bufs = [np.ascontiguousarray(b, np.uint8) for b in bufs]
    ptrs = (ctypes.c_void_p * max(1, len(bufs)))(*[_p(b).value for b in bufs])
    lens = np.array([b.shape[0] for b in bufs], np.int64)
    counts = (ctypes.c_int64 * 3)()
    if not lib.pmmg_shard_assemble(len(bufs), ptrs, _p(lens), int(K), counts, *([None] * 9)):
        raise ValueError("pmmg_shard_assemble: inconsistent buffers")
    nv, nk, nt = (int(x) for x in counts)
    xyz, sol = np.empty((nv, 3)), np.empty((nv, K))
    tetv, adja = np.empty((nk, 4), np.int32), np.empty((nk, 4), np.int32)
    triv, adjt = np.empty((nt, 3), np.int32), np.empty((nt, 3), np.int32)
    tg, vg, rg = np.empty(nk, np.int32), np.empty(nv, np.int32), np.empty(nt, np.int32)
    if not lib.pmmg_shard_assemble(len(bufs), ptrs, _p(lens), int(K), counts, _p(xyz), _p(sol), _p(tetv), _p(adja),
                                   _p(triv), _p(adjt), _p(tg), _p(vg), _p(rg)):
        raise ValueError("pmmg_shard_assemble failed")
    mesh = Mesh(kind, n, xyz, tetv, adja, triv, adjt, np.zeros(nv, np.uint8))
    return HaloShard(mesh, tg, vg, rg, halo, sol)


def parts_frame(ri, part: Part, halo: float = DEFAULT_HALO, hausd: float = 0.0, cell_factor: float = 1.0):
    """The halo and the occupancy grid every rank's shard needs, from the
    ranks' parts alone (collective over ri's process group): the largest tetra
    extent and the bounding box of every part's vertices, reduced over the
    ranks (max / min / max), then halo_shard_cells's rules — halo < 0 in units
    of that extent, never less than 1.01 * hausd, grid_for over the box.
    Returns (h, g_lo, cell, g_n), identical on every rank and equal to what
    halo_shard_cells derives from the whole group (whose vertices are all
    used by some part's tetra or trias)."""
    import torch
    import torch.distributed as dist

    ext = 0.0
    if part.tetv.shape[0]:
        loc = (np.searchsorted(part.vert_gid, part.tetv) + 1).astype(np.int32)
        ext = float(host_lib().pmmg_max_tet_extent(int(part.xyz.shape[0]), _p(np.ascontiguousarray(part.xyz)),
                                                   int(loc.shape[0]), _p(np.ascontiguousarray(loc))))
    lo, hi = range_box(part.xyz)
    if part.xyz.shape[0] == 0:
        lo, hi = np.full(3, np.inf), np.full(3, -np.inf)
    dev = torch.device("cuda", torch.cuda.current_device()) if ri.backend == "nccl" else torch.device("cpu")
    v = torch.tensor(np.concatenate([[ext], -np.asarray(lo, np.float64), np.asarray(hi, np.float64)]),
                     dtype=torch.float64, device=dev)
    dist.all_reduce(v, op=dist.ReduceOp.MAX)
    v = v.cpu().numpy()
    h = -halo * float(v[0]) if halo < 0 else float(halo)
    h = max(h, 1.01 * float(hausd))
    g_lo, cell, g_n = grid_for(-v[1:4], v[4:7], h, cell_factor)
    return h, g_lo, cell, g_n


def shard_from_parts(ri, part: Part, q_xyz: np.ndarray, halo: float, g_lo=None, cell: float = 0.0, g_n=None,
                     kind: int = 0, n: int = 0, hausd: float = 0.0) -> HaloShard:
    """This rank's halo shard built from the ranks' parts (collective over
    ri's process group): every rank's region all-gathered, this rank's part
    packed for every rank, one all-to-all of the buffers (torch.distributed:
    gloo on the CPU, RCCL with device buffers), the received buffers
    assembled.  g_lo None: the halo (halo < 0: in units of the largest tetra
    extent) and the grid are derived from the parts (parts_frame), so that no
    rank needs the whole group; else `halo` (absolute) and the grid must be the
    same on every rank.  The halo is never less than 1.01 * hausd (see
    halo_shard)."""
    import torch
    import torch.distributed as dist

    if g_lo is None:
        halo, g_lo, cell, g_n = parts_frame(ri, part, halo, hausd)
    halo = max(float(halo), 1.01 * float(hausd))
    reg = region_of(q_xyz, g_lo, cell, g_n, halo)
    world = dist.get_world_size()
    regs = [None] * world
    dist.all_gather_object(regs, (reg.lo, reg.hi, np.packbits(reg.occ)))
    nocc = reg.occ.shape[0]
    out = [pack_part(part, Region(lo, hi, reg.g_lo, reg.cell, reg.g_n, np.unpackbits(occ)[:nocc], halo))
           for lo, hi, occ in regs]
    dev = torch.device("cuda", torch.cuda.current_device()) if ri.backend == "nccl" else torch.device("cpu")
    send_sizes = torch.tensor([b.shape[0] for b in out], dtype=torch.int64, device=dev)
    recv_sizes = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv_sizes, send_sizes)
    rs = [int(x) for x in recv_sizes.cpu()]
    send = torch.from_numpy(np.concatenate(out) if out else np.empty(0, np.uint8)).to(dev)
    recv = torch.empty(sum(rs), dtype=torch.uint8, device=dev)
    dist.all_to_all_single(recv, send, rs, [b.shape[0] for b in out])
    recv = recv.cpu().numpy()
    offs = np.concatenate([[0], np.cumsum(rs)])
    bufs = [recv[offs[i]:offs[i + 1]] for i in range(world)]
    K = int(part.sol.shape[1]) if part.sol is not None and part.sol.ndim == 2 else 0
    return assemble(bufs, K, kind, n, halo)
