"""Minimal Medit ASCII reader (.mesh / .sol) for the reference's fixtures.

Follows the formats PMMG_loadMesh_centralized / PMMG_loadAllSols_centralized
read through Mmg (reference src/inout_pmmg.c:488, :748): keyword blocks
``Vertices``, ``Tetrahedra``, ``Triangles``; ``SolAtVertices`` with a type
list (1 scalar, 2 vector, 3 symmetric tensor).  Medit stores a 3D tensor as
m11 m12 m22 m13 m23 m33; MMG5 keeps m11 m12 m13 m22 m23 m33 in memory, so
tensors are reordered on read (MMG5_loadSolAtVertices_lines does the same
swap of entries 2 and 3).
"""
from __future__ import annotations

import numpy as np


def _tokens(path: str) -> list[str]:
    out = []
    with open(path) as f:
        for line in f:
            line = line.split("#", 1)[0]
            out.extend(line.split())
    return out


def read_mesh(path: str) -> dict:
    t = _tokens(path)
    res = {"xyz": np.zeros((0, 3)), "tetv": np.zeros((0, 4), np.int32), "triv": np.zeros((0, 3), np.int32)}
    i = 0
    while i < len(t):
        kw = t[i]
        if kw == "Vertices":
            n = int(t[i + 1])
            a = np.array(t[i + 2:i + 2 + 4 * n], dtype=np.float64).reshape(n, 4)
            res["xyz"] = np.ascontiguousarray(a[:, :3])
            res["vref"] = a[:, 3].astype(np.int32)
            i += 2 + 4 * n
        elif kw == "Tetrahedra":
            n = int(t[i + 1])
            a = np.array(t[i + 2:i + 2 + 5 * n], dtype=np.int64).reshape(n, 5)
            res["tetv"] = np.ascontiguousarray(a[:, :4].astype(np.int32))
            i += 2 + 5 * n
        elif kw == "Triangles":
            n = int(t[i + 1])
            a = np.array(t[i + 2:i + 2 + 4 * n], dtype=np.int64).reshape(n, 4)
            res["triv"] = np.ascontiguousarray(a[:, :3].astype(np.int32))
            i += 2 + 4 * n
        elif kw in ("MeshVersionFormatted", "Dimension"):
            i += 2
        else:
            i += 1
    return res


def read_sol(path: str) -> list[np.ndarray]:
    """Returns one (np, size) array per solution of a SolAtVertices block."""
    t = _tokens(path)
    i = t.index("SolAtVertices")
    n = int(t[i + 1])
    ntyp = int(t[i + 2])
    types = [int(x) for x in t[i + 3:i + 3 + ntyp]]
    sizes = [{1: 1, 2: 3, 3: 6}[ty] for ty in types]
    tot = sum(sizes)
    vals = np.array(t[i + 3 + ntyp:i + 3 + ntyp + tot * n], dtype=np.float64).reshape(n, tot)
    out, c = [], 0
    for s in sizes:
        a = np.ascontiguousarray(vals[:, c:c + s])
        if s == 6:  # Medit m11 m12 m22 m13 m23 m33 -> MMG5 m11 m12 m13 m22 m23 m33
            a = np.ascontiguousarray(a[:, [0, 1, 3, 2, 4, 5]])
        out.append(a)
        c += s
    return out


def tetra_adjacency(tetv: np.ndarray) -> np.ndarray:
    """adja (4*k+i encoding, 0 = boundary) by face matching, as MMG3D_hashTetra builds it."""
    ne = tetv.shape[0]
    idir = np.array([[1, 2, 3], [0, 3, 2], [0, 1, 3], [0, 2, 1]])
    faces = np.sort(tetv[:, idir], axis=2).reshape(-1, 3).astype(np.int64)  # (4ne, 3)
    code = (np.arange(ne)[:, None] + 1) * 4 + np.arange(4)[None, :]
    code = code.reshape(-1)
    key = (faces[:, 0] << 42) | (faces[:, 1] << 21) | faces[:, 2]
    order = np.argsort(key, kind="stable")
    ks = key[order]
    adja = np.zeros(4 * ne, np.int32)
    same = np.nonzero(ks[1:] == ks[:-1])[0]
    a, b = order[same], order[same + 1]
    adja[a] = code[b]
    adja[b] = code[a]
    return adja.reshape(ne, 4)


def boundary_trias(tetv: np.ndarray, adja: np.ndarray) -> np.ndarray:
    idir = np.array([[1, 2, 3], [0, 3, 2], [0, 1, 3], [0, 2, 1]])
    k, f = np.nonzero(adja == 0)
    return np.ascontiguousarray(tetv[k[:, None], idir[f]].astype(np.int32))


def tria_adjacency(triv: np.ndarray) -> np.ndarray:
    """adjt (3*k+i encoding, 0 = open edge); edge i is opposite vertex i."""
    nt = triv.shape[0]
    a = triv[:, [1, 2, 0]].astype(np.int64)
    b = triv[:, [2, 0, 1]].astype(np.int64)
    lo, hi = np.minimum(a, b).reshape(-1), np.maximum(a, b).reshape(-1)
    key = (lo << 32) | hi
    code = ((np.arange(nt)[:, None] + 1) * 3 + np.arange(3)[None, :]).reshape(-1)
    order = np.argsort(key, kind="stable")
    ks = key[order]
    adjt = np.zeros(3 * nt, np.int32)
    same = np.nonzero(ks[1:] == ks[:-1])[0]
    x, y = order[same], order[same + 1]
    adjt[x] = code[y]
    adjt[y] = code[x]
    return adjt.reshape(nt, 3)


def refine8(xyz: np.ndarray, tetv: np.ndarray):
    """Uniform 1:8 refinement (edge midpoints; each tetra -> 4 corner + 4
    octahedron tetra).  Returns (xyz_new, tetv_new, is_midpoint)."""
    edges = np.array([[0, 1], [0, 2], [0, 3], [1, 2], [1, 3], [2, 3]])
    e = np.sort(tetv[:, edges].reshape(-1, 2), axis=1)
    uniq, inv = np.unique(e, axis=0, return_inverse=True)
    inv = inv.reshape(-1, 6)
    npo = xyz.shape[0]
    mid = 0.5 * (xyz[uniq[:, 0] - 1] + xyz[uniq[:, 1] - 1])
    xyz_new = np.vstack([xyz, mid])
    m = inv + npo + 1  # midpoint ids of edges 01 02 03 12 13 23
    v = tetv
    t = [
        np.stack([v[:, 0], m[:, 0], m[:, 1], m[:, 2]], 1),
        np.stack([m[:, 0], v[:, 1], m[:, 3], m[:, 4]], 1),
        np.stack([m[:, 1], m[:, 3], v[:, 2], m[:, 5]], 1),
        np.stack([m[:, 2], m[:, 4], m[:, 5], v[:, 3]], 1),
        np.stack([m[:, 0], m[:, 1], m[:, 2], m[:, 4]], 1),
        np.stack([m[:, 0], m[:, 1], m[:, 4], m[:, 3]], 1),
        np.stack([m[:, 1], m[:, 2], m[:, 4], m[:, 5]], 1),
        np.stack([m[:, 1], m[:, 3], m[:, 4], m[:, 5]], 1),
    ]
    tet_new = np.ascontiguousarray(np.concatenate(t, 0).astype(np.int32))
    is_mid = np.r_[np.zeros(npo, bool), np.ones(mid.shape[0], bool)]
    return np.ascontiguousarray(xyz_new), tet_new, is_mid


# ---------------------------------------------------------------- C reader
# pmmg_medit_read_mesh / pmmg_medit_read_sol of libpmmg_host (csrc/pmmg_medit.c),
# the reader a C shim or program uses; the numpy reader above is the fixture
# tool the tests compare it with.

import ctypes as _ct  # noqa: E402


class _CMesh(_ct.Structure):
    _fields_ = [("np", _ct.c_int), ("ne", _ct.c_int), ("nt", _ct.c_int), ("xyz", _ct.POINTER(_ct.c_double)),
                ("vref", _ct.POINTER(_ct.c_int)), ("tetv", _ct.POINTER(_ct.c_int)), ("tref", _ct.POINTER(_ct.c_int)),
                ("triv", _ct.POINTER(_ct.c_int)), ("trref", _ct.POINTER(_ct.c_int))]


_MAXSOL = 32


class _CSol(_ct.Structure):
    _fields_ = [("np", _ct.c_int), ("nsol", _ct.c_int), ("type", _ct.c_int * _MAXSOL), ("size", _ct.c_int * _MAXSOL),
                ("val", _ct.POINTER(_ct.c_double) * _MAXSOL)]


def _arr(ptr, n, dtype, cols):
    if n == 0:
        return np.zeros((0, cols) if cols > 1 else (0,), dtype)
    a = np.ctypeslib.as_array(ptr, shape=(n * cols,)).astype(dtype, copy=True)
    return a.reshape(n, cols) if cols > 1 else a


def read_mesh_c(path: str) -> dict:
    """The C reader (libpmmg_host): xyz, vref, tetv, tref, triv, trref."""
    from ._native import host_lib

    lib = host_lib()
    m = _CMesh()
    err = _ct.create_string_buffer(512)
    if not lib.pmmg_medit_read_mesh(path.encode(), _ct.byref(m), err, 512):
        raise ValueError(err.value.decode())
    try:
        return {"xyz": _arr(m.xyz, m.np, np.float64, 3), "vref": _arr(m.vref, m.np, np.int32, 1),
                "tetv": _arr(m.tetv, m.ne, np.int32, 4), "tref": _arr(m.tref, m.ne, np.int32, 1),
                "triv": _arr(m.triv, m.nt, np.int32, 3), "trref": _arr(m.trref, m.nt, np.int32, 1)}
    finally:
        lib.pmmg_medit_free_mesh(_ct.byref(m))


def read_sol_c(path: str) -> list[np.ndarray]:
    """The C reader: one (np, size) array per solution (MMG5 tensor order)."""
    from ._native import host_lib

    lib = host_lib()
    s = _CSol()
    err = _ct.create_string_buffer(512)
    if not lib.pmmg_medit_read_sol(path.encode(), _ct.byref(s), err, 512):
        raise ValueError(err.value.decode())
    try:
        return [_arr(s.val[j], s.np, np.float64, s.size[j]).reshape(s.np, s.size[j]) for j in range(s.nsol)]
    finally:
        lib.pmmg_medit_free_sol(_ct.byref(s))
